// Exact-fp32 GEMM with fused epilogues for the learner's torso-FC / LSTM
// input projection / their gradients (v_mfma_f32_32x32x2_f32: f32 in, f32
// accumulate, one rounding per product).
//
// Reference: experiment.py:185-198 (Linear(256) + ReLU on the flattened
// conv features, concat [torso, clip(r), one_hot(a), instruction]) and the
// LSTMBlockCell's x W_x projection (:228-235); their gradients are the
// backward of the same products.  Every learner GEMM is one of
//   C[M, N] (+)= op(A)[M, K] op(B)[K, N]      op = identity or transpose
// with the epilogue  v = acc [+ bias[n]] [* (mask[m, n] > 0)] [relu] [+= C]
// and two learner-specific extras:
//   * ones_row: op(A) gets an extra row of ones, whose result row is the
//     column sum of op(B) over K - the bias gradient of a weight-gradient
//     GEMM (db = 1^T dY) comes out of the same pass, accumulated into
//     `colsum`;
//   * aug: the core-input columns [clip(r), one_hot(a), 0...] are written
//     next to the FC output (C's columns N .. ldc-1), so the concat of
//     experiment.py:191-198 is never a separate kernel.
//
// Tiling: 64 x 64 output tile per 256-thread workgroup (2 x 2 waves of one
// 32 x 32 MFMA accumulator each), K in steps of 32 staged through a double-
// buffered LDS image [row][k] (pitch 36 floats: conflict-free 16-B reads)
// with the next step's global loads in flight under the current 16 MFMAs
// (steps of 16 left ~0.25 us of MFMA work to cover each step's loads).  The
// k order inside a step is permuted (MFMA (c, s) uses k = 16 h + 4 c + s for
// lane half h) on both operands, so each lane reads its 16 k values of a
// step with four ds_read_b128.  Large-K products (the weight gradients, K = T*B = 3232)
// split K over grid.z into per-split partial slabs that one reduction
// kernel sums in split order: deterministic, no float atomics.
#include "gemm_f32.h"
#include "knobs.h"

#include <algorithm>
#include <cstdlib>

namespace sa {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int BM = 64, BN = 64, BK = 32, PK = BK + 4;  // pitch: odd 16-B units

struct Args {
  const float* A;
  const float* B;
  int M, N, K, lda, ldb, ta, tb, ones_row;
  int splits, kchunk;
  float* part;  // [splits][Mr][N] when splits > 1
  GemmEpilogue ep;
};

// epilogue of one output element (row m < M)
__device__ __forceinline__ void store_out(const GemmEpilogue& e, int m, int n, float v) {
  if (e.bias != nullptr) v += e.bias[n];
  if (e.mask != nullptr) v = e.mask[static_cast<int64_t>(m) * e.ldm + n] > 0.f ? v : 0.f;
  if (e.relu) v = fmaxf(v, 0.f);
  float* c = e.C + static_cast<int64_t>(m) * e.ldc + n;
  if (e.accumulate) v += *c;
  *c = v;
}

// the core-input columns [clip(r), one_hot(a), 0...] of row m (aug mode)
__device__ __forceinline__ void store_aug(const GemmEpilogue& e, int m, int j) {
  // j in [0, ldc - N): column N + j
  float v = 0.f;
  if (j == 0) {
    v = fminf(fmaxf(e.aug_reward[m], -1.f), 1.f);  // core input: always abs_one
  } else if (j - 1 == static_cast<int>(e.aug_action[m])) {
    v = 1.f;
  }
  e.C[static_cast<int64_t>(m) * e.ldc + e.aug_c0 + j] = v;
}

// RM: 32-row MFMA blocks per wave (workgroup tile (64 RM) x 64): RM = 2 for
// the tall learner GEMMs (M = T*B = 3232) reuses each B fragment twice
template <int RM>
__global__ __launch_bounds__(256) void gemm_f32_kernel(Args a) {
  constexpr int BMt = BM * RM;
  __shared__ __attribute__((aligned(16))) float As[2][BMt * PK];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * PK];
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int h = lane >> 5, l32 = lane & 31;
  const int m0 = blockIdx.x * BMt, n0 = blockIdx.y * BN;
  const int Mr = a.M + a.ones_row;
  const int kbeg = blockIdx.z * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);
  constexpr int KQ = BK / 16;  // f4 per thread and operand per K step and 64 rows

  // global -> register staging of one K step
  f4 ra[RM][KQ], rb[KQ];
  auto load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < KQ; ++j) {
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        f4 va = {0.f, 0.f, 0.f, 0.f};
        if (!a.ta) {  // A[m][k]: thread = (m, k quad)
          const int m = m0 + 64 * r + (t >> 2), k = k0 + 4 * (t & 3) + 16 * j;
          if (m < a.M && k < kend)
            va = *reinterpret_cast<const f4*>(a.A + static_cast<int64_t>(m) * a.lda + k);
          else if (m == a.M && a.ones_row && k < kend)
            va = f4{1.f, 1.f, 1.f, 1.f};
        } else {  // A[k][m]: thread = (k, m quad)
          const int k = k0 + (t >> 4) + 16 * j, m = m0 + 64 * r + 4 * (t & 15);
          if (k < kend) {
            if (m + 3 < a.M) {
              va = *reinterpret_cast<const f4*>(a.A + static_cast<int64_t>(k) * a.lda + m);
            } else {
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                if (m + q < a.M) va[q] = a.A[static_cast<int64_t>(k) * a.lda + m + q];
                else if (m + q == a.M && a.ones_row) va[q] = 1.f;
              }
            }
          }
        }
        ra[r][j] = va;
      }
      f4 vb = {0.f, 0.f, 0.f, 0.f};
      if (!a.tb) {  // B[k][n]: thread = (k, n quad)
        const int k = k0 + (t >> 4) + 16 * j, n = n0 + 4 * (t & 15);
        if (k < kend && n < a.N)
          vb = *reinterpret_cast<const f4*>(a.B + static_cast<int64_t>(k) * a.ldb + n);
      } else {  // B[n][k]: thread = (n, k quad)
        const int n = n0 + (t >> 2), k = k0 + 4 * (t & 3) + 16 * j;
        if (n < a.N && k < kend)
          vb = *reinterpret_cast<const f4*>(a.B + static_cast<int64_t>(n) * a.ldb + k);
      }
      rb[j] = vb;
    }
  };
  auto commit = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < KQ; ++j) {
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        if (!a.ta) {
          *reinterpret_cast<f4*>(&As[buf][(64 * r + (t >> 2)) * PK + 4 * (t & 3) + 16 * j]) =
              ra[r][j];
        } else {
          const int k = (t >> 4) + 16 * j, m = 64 * r + 4 * (t & 15);
#pragma unroll
          for (int q = 0; q < 4; ++q) As[buf][(m + q) * PK + k] = ra[r][j][q];
        }
      }
      if (!a.tb) {
        const int k = (t >> 4) + 16 * j, n = 4 * (t & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) Bs[buf][(n + q) * PK + k] = rb[j][q];
      } else {
        *reinterpret_cast<f4*>(&Bs[buf][(t >> 2) * PK + 4 * (t & 3) + 16 * j]) = rb[j];
      }
    }
  };

  f16v acc[RM];
#pragma unroll
  for (int r = 0; r < RM; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[r][e] = 0.f;
  // wave rows: 32-row blocks wm * 32 RM + 32 r; lane half h consumes
  // k = (BK / 2) h + s in MFMA s of a step
  const int arow = (wm * 32 * RM + l32) * PK + (BK / 2) * h;
  const int brow = (wn * 32 + l32) * PK + (BK / 2) * h;
  int buf = 0;
  if (kbeg < kend) {
    load(kbeg);
    commit(0);
    __syncthreads();
  }
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    const bool more = k0 + BK < kend;
    if (more) load(k0 + BK);  // in flight under the MFMAs
#pragma unroll
    for (int c = 0; c < BK / 8; ++c) {
      const f4 bv = *reinterpret_cast<const f4*>(&Bs[buf][brow + 4 * c]);
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        const f4 av = *reinterpret_cast<const f4*>(&As[buf][arow + 32 * r * PK + 4 * c]);
#pragma unroll
        for (int s = 0; s < 4; ++s)
          acc[r] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], acc[r], 0, 0, 0);
      }
    }
    if (more) {
      commit(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  // D[i][j]: j = lane & 31, i = (e & 3) + 8 (e >> 2) + 4 h
  const int n = n0 + wn * 32 + l32;
  if (a.splits > 1) {
    float* p = a.part + static_cast<int64_t>(blockIdx.z) * Mr * a.N;
#pragma unroll
    for (int r = 0; r < RM; ++r)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm * 32 * RM + 32 * r + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (m < Mr && n < a.N) p[static_cast<int64_t>(m) * a.N + n] = acc[r][e];
      }
    return;
  }
#pragma unroll
  for (int r = 0; r < RM; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int m = m0 + wm * 32 * RM + 32 * r + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (n >= a.N) continue;
      if (m < a.M) store_out(a.ep, m, n, acc[r][e]);
      else if (m == a.M && a.ones_row) a.ep.colsum[n] += acc[r][e];
    }
  if (a.ep.aug_c0 > 0 && blockIdx.y == 0) {
    const int naug = a.ep.ldc - a.ep.aug_c0;
    for (int e = t; e < BMt * naug; e += 256) {
      const int m = m0 + e / naug;
      if (m < a.M) store_aug(a.ep, m, e % naug);
    }
  }
}

// The same tile program with the operand layout (TA, TB) compile-time and
// every global load a range-checked buffer load (an out-of-range element -
// past M / N / the K chunk - gets an offset past the buffer's end and reads
// zero), so the K-step loads carry no branches: the generic kernel's
// runtime layout switches and per-load bounds branches (123 exec branches,
// 78 scalar edge loads in its ISA) made the compiler wait on loads early.
// Needs M % 4 == 0 when TA (whole m quads) and N % 4 == 0 when !TB.
constexpr uint32_t kGemmOOB = 0xFFFFFFF0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gemm_rsrc(const float* p, int64_t floats) {
  const int64_t bytes = floats * 4;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0,
                                           static_cast<int>(bytes >= 0xFFFFFF00ll
                                                                ? 0xFFFFFF00u
                                                                : static_cast<uint32_t>(bytes)),
                                           0x00020000);
}
__device__ __forceinline__ f4 gemm_bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

template <int RM, bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f32_bl_kernel(Args a) {
  constexpr int BMt = BM * RM;
  __shared__ __attribute__((aligned(16))) float As[2][BMt * PK];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * PK];
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int h = lane >> 5, l32 = lane & 31;
  const int m0 = blockIdx.x * BMt, n0 = blockIdx.y * BN;
  const int Mr = a.M + a.ones_row;
  const int kbeg = blockIdx.z * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);
  constexpr int KQ = BK / 16;
  const auto ar = gemm_rsrc(a.A, TA ? static_cast<int64_t>(a.K) * a.lda
                                    : static_cast<int64_t>(a.M) * a.lda);
  const auto br = gemm_rsrc(a.B, TB ? static_cast<int64_t>(a.N) * a.ldb
                                    : static_cast<int64_t>(a.K) * a.ldb);
  // per-thread fixed parts of the operand addresses
  f4 ra[RM][KQ], rb[KQ];
  auto load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < KQ; ++j) {
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        if constexpr (!TA) {  // A[m][k]: thread = (m, k quad)
          const int m = m0 + 64 * r + (t >> 2), k = k0 + 4 * (t & 3) + 16 * j;
          const bool in = m < a.M && k < kend;
          f4 v = gemm_bload(ar, in ? static_cast<uint32_t>(m * a.lda + k) * 4u : kGemmOOB);
          if (a.ones_row && m == a.M && k < kend) v = f4{1.f, 1.f, 1.f, 1.f};
          ra[r][j] = v;
        } else {  // A[k][m]: thread = (k, m quad)
          const int k = k0 + (t >> 4) + 16 * j, m = m0 + 64 * r + 4 * (t & 15);
          const bool in = k < kend && m < a.M;
          f4 v = gemm_bload(ar, in ? static_cast<uint32_t>(k * a.lda + m) * 4u : kGemmOOB);
          if (a.ones_row && m == a.M && k < kend) v[0] = 1.f;
          ra[r][j] = v;
        }
      }
      if constexpr (!TB) {  // B[k][n]: thread = (k, n quad)
        const int k = k0 + (t >> 4) + 16 * j, n = n0 + 4 * (t & 15);
        const bool in = k < kend && n < a.N;
        rb[j] = gemm_bload(br, in ? static_cast<uint32_t>(k * a.ldb + n) * 4u : kGemmOOB);
      } else {  // B[n][k]: thread = (n, k quad)
        const int n = n0 + (t >> 2), k = k0 + 4 * (t & 3) + 16 * j;
        const bool in = n < a.N && k < kend;
        rb[j] = gemm_bload(br, in ? static_cast<uint32_t>(n * a.ldb + k) * 4u : kGemmOOB);
      }
    }
  };
  // LDS images: an operand whose global rows run along K (A[m][k], B[n][k])
  // is stored [m or n][k] (pitch PK: conflict-free 16-B k-quad reads); one
  // whose rows run along M / N (A[k][m] when TA, B[k][n] when !TB) is
  // stored as it comes, [k][m or n] with 16-B stores, and read one k at a
  // time (consecutive lanes, consecutive m / n: conflict-free 4-B reads).
  // Transposing those on the commit (four 4-B stores per quad, rows 4 PK
  // apart) cost 9-14 bank-conflict cycles per LDS instruction (PMC).
  auto commit = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < KQ; ++j) {
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        if constexpr (!TA) {
          *reinterpret_cast<f4*>(&As[buf][(64 * r + (t >> 2)) * PK + 4 * (t & 3) + 16 * j]) =
              ra[r][j];
        } else {
          const int k = (t >> 4) + 16 * j, m = 64 * r + 4 * (t & 15);
          *reinterpret_cast<f4*>(&As[buf][k * BMt + m]) = ra[r][j];
        }
      }
      if constexpr (!TB) {
        const int k = (t >> 4) + 16 * j, n = 4 * (t & 15);
        *reinterpret_cast<f4*>(&Bs[buf][k * BN + n]) = rb[j];
      } else {
        *reinterpret_cast<f4*>(&Bs[buf][(t >> 2) * PK + 4 * (t & 3) + 16 * j]) = rb[j];
      }
    }
  };

  f16v acc[RM];
#pragma unroll
  for (int r = 0; r < RM; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[r][e] = 0.f;
  const int arow = (wm * 32 * RM + l32) * PK + (BK / 2) * h;
  const int brow = (wn * 32 + l32) * PK + (BK / 2) * h;
  const int kh = (BK / 2) * h;
  int buf = 0;
  if (kbeg < kend) {
    load(kbeg);
    commit(0);
    __syncthreads();
  }
  // branch-free loop body: the step after the last loads only zeros (every
  // element out of the K chunk) into the idle buffer, which nothing reads;
  // a conditional load / commit made the compiler copy the accumulators
  // through VGPRs at the loop header, right behind the last MFMA
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    load(k0 + BK);  // in flight under the MFMAs
#pragma unroll
    for (int c = 0; c < BK / 8; ++c) {
      // k = BK/2 h + 4 c + s for MFMA s of lane half h (both operands)
      f4 bv;
      if constexpr (TB) {
        bv = *reinterpret_cast<const f4*>(&Bs[buf][brow + 4 * c]);
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) bv[s] = Bs[buf][(kh + 4 * c + s) * BN + wn * 32 + l32];
      }
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        f4 av;
        if constexpr (!TA) {
          av = *reinterpret_cast<const f4*>(&As[buf][arow + 32 * r * PK + 4 * c]);
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s)
            av[s] = As[buf][(kh + 4 * c + s) * BMt + wm * 32 * RM + 32 * r + l32];
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
          acc[r] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], acc[r], 0, 0, 0);
      }
    }
    commit(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  const int n = n0 + wn * 32 + l32;
  if (a.splits > 1) {
    float* p = a.part + static_cast<int64_t>(blockIdx.z) * Mr * a.N;
#pragma unroll
    for (int r = 0; r < RM; ++r)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm * 32 * RM + 32 * r + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (m < Mr && n < a.N) p[static_cast<int64_t>(m) * a.N + n] = acc[r][e];
      }
    return;
  }
#pragma unroll
  for (int r = 0; r < RM; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int m = m0 + wm * 32 * RM + 32 * r + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (n >= a.N) continue;
      if (m < a.M) store_out(a.ep, m, n, acc[r][e]);
      else if (m == a.M && a.ones_row) a.ep.colsum[n] += acc[r][e];
    }
  if (a.ep.aug_c0 > 0 && blockIdx.y == 0) {
    const int naug = a.ep.ldc - a.ep.aug_c0;
    for (int e = t; e < BMt * naug; e += 256) {
      const int m = m0 + e / naug;
      if (m < a.M) store_aug(a.ep, m, e % naug);
    }
  }
}

// Fixed-order sum of the split partials + the epilogue.
__global__ __launch_bounds__(256) void gemm_f32_reduce_kernel(Args a) {
  const int Mr = a.M + a.ones_row;
  const int64_t total = static_cast<int64_t>(Mr) * a.N;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i < total) {
    const int m = static_cast<int>(i / a.N), n = static_cast<int>(i - static_cast<int64_t>(m) * a.N);
    float s = 0.f;
    for (int z = 0; z < a.splits; ++z) s += a.part[static_cast<int64_t>(z) * total + i];
    if (m < a.M) store_out(a.ep, m, n, s);
    else a.ep.colsum[n] += s;
  }
  if (a.ep.aug_c0 > 0) {
    const int naug = a.ep.ldc - a.ep.aug_c0;
    const int64_t j = i;  // one aug element per thread over the first M*naug threads
    if (j < static_cast<int64_t>(a.M) * naug)
      store_aug(a.ep, static_cast<int>(j / naug), static_cast<int>(j % naug));
  }
}

}  // namespace

int64_t gemm_f32_part_floats(int M, int N, int K, int ones_row, int splits) {
  (void)K;
  return splits > 1 ? static_cast<int64_t>(splits) * (M + ones_row) * N : 0;
}

// 128-row workgroup tiles (RM = 2) for tall products are opt-in
// (SA_GEMM_RM=2 for M + ones_row >= 1024): the learner step measured 10.61 -
// 10.63 ms with them against 10.51 ms with 64-row tiles (fewer workgroups
// per GEMM on 256 CUs, 55 KB of LDS each)
static int gemm_rm(int Mr) {
  static const int force = sa::measure_knob("SA_GEMM_RM", 1);
  return force == 2 && Mr >= 1024 ? 2 : 1;
}

int gemm_f32_splits(int M, int N, int K, int ones_row) {
  const int bm = BM * gemm_rm(M + ones_row);
  const int tiles = ((M + ones_row + bm - 1) / bm) * ((N + BN - 1) / BN);
  int s = 1;
  // enough workgroups to fill 256 CUs twice over (SA_GEMM_WG_TARGET), each
  // K chunk >= 128
  static const int target = std::max(1, sa::measure_knob("SA_GEMM_WG_TARGET", 512));
  while (tiles * s < target && K / (2 * s) >= 128 && s < 16) s *= 2;
  return s;
}

bool gemm_f32_launch(const float* A, const float* B, int M, int N, int K, int lda,
                     int ldb, bool ta, bool tb, bool ones_row, int splits, float* part,
                     const GemmEpilogue& ep, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return false;
  // K quads are read as f4 only where K is an operand's column index
  // (!ta: A[m][k], tb: B[n][k]); op(A) = A^T with B[k][n] reads K by rows
  if (lda % 4 || ldb % 4 || (K % 4 && (!ta || tb))) return false;
  if (ones_row && ep.colsum == nullptr) return false;
  if (splits > 1 && part == nullptr) return false;
  Args a{};
  a.A = A;
  a.B = B;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb;
  a.ta = ta; a.tb = tb; a.ones_row = ones_row;
  a.splits = std::max(1, splits);
  a.kchunk = ((K + a.splits - 1) / a.splits + BK - 1) / BK * BK;
  a.part = part;
  a.ep = ep;
  const int Mr = M + (ones_row ? 1 : 0);
  const int rm = gemm_rm(Mr);
  dim3 grid((Mr + BM * rm - 1) / (BM * rm), (N + BN - 1) / BN, a.splits);
  // branch-free buffer-load variant (SA_GEMM_BL=0: the generic kernel):
  // whole quads along every f4 operand axis, byte offsets within 32 bits
  static const int bl = sa::env_knob("SA_GEMM_BL", 1);
  const int64_t abytes = (ta ? static_cast<int64_t>(K) * lda : static_cast<int64_t>(M) * lda) * 4;
  const int64_t bbytes = (tb ? static_cast<int64_t>(N) * ldb : static_cast<int64_t>(K) * ldb) * 4;
  if (bl && (!ta || M % 4 == 0) && (tb || N % 4 == 0) && abytes < 0xFFFFFF00ll &&
      bbytes < 0xFFFFFF00ll) {
    auto k = rm == 2
                 ? (ta ? (tb ? gemm_f32_bl_kernel<2, true, true> : gemm_f32_bl_kernel<2, true, false>)
                       : (tb ? gemm_f32_bl_kernel<2, false, true>
                             : gemm_f32_bl_kernel<2, false, false>))
                 : (ta ? (tb ? gemm_f32_bl_kernel<1, true, true> : gemm_f32_bl_kernel<1, true, false>)
                       : (tb ? gemm_f32_bl_kernel<1, false, true>
                             : gemm_f32_bl_kernel<1, false, false>));
    hipLaunchKernelGGL(k, grid, dim3(256), 0, stream, a);
  } else if (rm == 2)
    hipLaunchKernelGGL(gemm_f32_kernel<2>, grid, dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL(gemm_f32_kernel<1>, grid, dim3(256), 0, stream, a);
  if (a.splits > 1) {
    const int64_t total = static_cast<int64_t>(Mr) * N;
    const int64_t aug = ep.aug_c0 > 0 ? static_cast<int64_t>(M) * (ep.ldc - ep.aug_c0) : 0;
    const int64_t work = std::max(total, aug);
    hipLaunchKernelGGL(gemm_f32_reduce_kernel, dim3(static_cast<unsigned>((work + 255) / 256)),
                       dim3(256), 0, stream, a);
  }
  return true;
}

}  // namespace sa
