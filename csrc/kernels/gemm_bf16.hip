// bf16-operand GEMM on v_mfma_f32_32x32x16_bf16 (fp32 accumulate) with the
// bf16 learner's fused epilogues - the hand-written replacement of the
// library GEMMs the bf16 learner used for its torso FC, LSTM input
// projection and their gradients.
//
// Reference: experiment.py:185-198 (Linear(256) + ReLU on the flattened conv
// features, concat [torso, clip(r), one_hot(a), instruction]) and the
// LSTMBlockCell's x W_x projection (:228-235), plus their gradients.  Every
// product is  C[M, N] (+)= op(A)[M, K] op(B)[K, N]  (op = identity or
// transpose) with the epilogue of gemm_bf16.h; the ones row (bias gradient
// as the column sums of op(B)) and the core-input columns come out of the
// same pass, exactly as in the exact-fp32 twin (gemm_f32.hip).
//
// Tiling (CDNA4, 64-wide waves): 64 x 64 output tile per 256-thread
// workgroup, 2 x 2 waves of one 32 x 32 accumulator (16 fp32 per lane); K in
// steps of 64 through a double-buffered LDS image [row][k] for BOTH operands
// (pitch 72 bf16 = 9 16-B units, odd: a lane's 16-B fragment reads are
// conflict-free), the next step's global loads in flight under the current
// step's 4 MFMAs per wave.  An operand whose contiguous index is K (A
// row-major, B^T) is copied with 16-B loads and stores; one whose contiguous
// index is M / N (A^T of the weight gradients, B of the forward) is loaded
// as two 16-B rows k, k+1 and written as packed k-pairs (ds_write_b32), so
// the MFMA fragments (8 consecutive k of one row) are always one
// ds_read_b128.  Large-K products (the weight gradients, K = T*B) split K
// over grid.z into fp32 partial slabs that one kernel sums in split order:
// deterministic, no float atomics.
#include "gemm_bf16.h"
#include "knobs.h"

#include <algorithm>
#include <cstdlib>

namespace sa {
namespace {

typedef float f16v __attribute__((ext_vector_type(16)));
typedef __bf16 s8v __attribute__((ext_vector_type(8)));
typedef unsigned short bf16_t;

constexpr int BM = 64, BN = 64, BK = 64, PK = BK + 8;
constexpr bf16_t kOne = 0x3F80;  // bf16 1.0

struct Args {
  const bf16_t* A;
  const bf16_t* B;
  int M, N, K, lda, ldb, ta, tb, ones_row;
  int splits, kchunk;
  float* part;  // [splits][Mr][N] when splits > 1
  GemmBf16Epilogue ep;
};

__device__ __forceinline__ bf16_t to_bf16(float v) {
  // plain conversion: v_cvt_pk_bf16_f32 on gfx950 (round to nearest even,
  // NaN stays NaN)
  return __builtin_bit_cast(bf16_t, static_cast<__bf16>(v));
}
__device__ __forceinline__ float from_bf16(bf16_t v) {
  return __uint_as_float(static_cast<unsigned>(v) << 16);
}

__device__ __forceinline__ void store_out(const GemmBf16Epilogue& e, int m, int n, float v) {
  if (e.bias != nullptr) v += e.bias[n];
  if (e.mask != nullptr) v = from_bf16(e.mask[static_cast<int64_t>(m) * e.ldm + n]) > 0.f ? v : 0.f;
  if (e.relu) v = fmaxf(v, 0.f);
  const int64_t o = static_cast<int64_t>(m) * e.ldc + n;
  if (e.c_bf16) {
    static_cast<bf16_t*>(e.C)[o] = to_bf16(v);
  } else {
    float* c = static_cast<float*>(e.C) + o;
    if (e.accumulate) v += *c;
    *c = v;
  }
}

__device__ __forceinline__ void store_aug(const GemmBf16Epilogue& e, int m, int j) {
  float v = 0.f;
  if (j == 0) {
    v = fminf(fmaxf(e.aug_reward[m], -1.f), 1.f);  // core input: always abs_one
  } else if (j - 1 == static_cast<int>(e.aug_action[m])) {
    v = 1.f;
  }
  const int64_t o = static_cast<int64_t>(m) * e.ldc + e.aug_c0 + j;
  if (e.c_bf16) static_cast<bf16_t*>(e.C)[o] = to_bf16(v);
  else static_cast<float*>(e.C)[o] = v;
}

// 8 bf16 of row `r` (valid rows < R) at columns [c, c + 8) with the ones row
// at r == R (ones: op(A)'s extra row) - the K-contiguous operands
__device__ __forceinline__ uint4 load_row8(const bf16_t* base, int ld, int r, int R,
                                           bool ones, int c, int cend) {
  uint4 v = make_uint4(0, 0, 0, 0);
  if (c < cend) {
    if (r < R) {
      v = *reinterpret_cast<const uint4*>(base + static_cast<int64_t>(r) * ld + c);
    } else if (ones && r == R) {
      const unsigned o2 = kOne | (static_cast<unsigned>(kOne) << 16);
      v = make_uint4(o2, o2, o2, o2);
    }
  }
  return v;
}

// 8 bf16 of K-row `k` (valid k < kend) at M/N columns [c, c + 8) (valid
// columns < R, ones column at R) - the M/N-contiguous operands
__device__ __forceinline__ uint4 load_col8(const bf16_t* base, int ld, int k, int kend,
                                           int c, int R, bool ones) {
  uint4 v = make_uint4(0, 0, 0, 0);
  if (k >= kend) return v;
  const bf16_t* p = base + static_cast<int64_t>(k) * ld + c;
  if (c + 8 <= R) return *reinterpret_cast<const uint4*>(p);
  unsigned w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    bf16_t x = 0;
    if (c + q < R) x = p[q];
    else if (ones && c + q == R) x = kOne;
    w[q >> 1] |= static_cast<unsigned>(x) << (16 * (q & 1));
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ unsigned half(const uint4& v, int q) {
  const unsigned w = q < 2 ? (q == 0 ? v.x : v.y) : (q == 2 ? v.z : v.w);
  return w;
}

// 16-B loads through a buffer descriptor: an element range past the
// operand's end (offset kOOB) reads zeros, so the K-step loads of the
// layout-specialised kernel carry no bounds branches (callers guarantee
// whole 8-element chunks along M / N: R % 8 == 0)
constexpr uint32_t kOOB = 0xFFFFFFF0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bf_rsrc(const bf16_t* p, int64_t elems) {
  const int64_t bytes = elems * 2;
  return __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(p), 0,
      static_cast<int>(bytes >= 0xFFFFFF00ll ? 0xFFFFFF00u : static_cast<uint32_t>(bytes)),
      0x00020000);
}
__device__ __forceinline__ uint4 bl16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// TA / TB: the operand layouts as compile-time constants (BL: branch-free
// buffer loads, whole 8-element chunks along M and N)
template <bool TA, bool TB, bool BL>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) bf16_t As[2][BM * PK];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][BN * PK];
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int h = lane >> 5, l32 = lane & 31;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int Mr = a.M + a.ones_row;
  const int kbeg = blockIdx.z * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);

  // global -> register staging of one K step: two 16-B loads per operand
  // and thread.  K-contiguous: thread = (row t>>3 + 32 j, k chunk 8 (t&7));
  // M/N-contiguous: thread = (k pair t>>3, column chunk 8 (t&7)), rows
  // k = 2 (t>>3) and 2 (t>>3) + 1.
  uint4 ra[2], rb[2];
  const auto arr = bf_rsrc(a.A, TA ? static_cast<int64_t>(a.K) * a.lda
                                   : static_cast<int64_t>(a.M) * a.lda);
  const auto brr = bf_rsrc(a.B, TB ? static_cast<int64_t>(a.N) * a.ldb
                                   : static_cast<int64_t>(a.K) * a.ldb);
  const unsigned o2 = kOne | (static_cast<unsigned>(kOne) << 16);
  auto load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (BL) {
        if constexpr (!TA) {  // A[m][k]: row m, k chunk
          const int r = m0 + (t >> 3) + 32 * j, c = k0 + 8 * (t & 7);
          const bool in = r < a.M && c < kend;
          uint4 v = bl16(arr, in ? static_cast<uint32_t>(r * a.lda + c) * 2u : kOOB);
          if (a.ones_row && r == a.M && c < kend) v = make_uint4(o2, o2, o2, o2);
          ra[j] = v;
        } else {  // A[k][m]: K-row k, m chunk
          const int k = k0 + 2 * (t >> 3) + j, c = m0 + 8 * (t & 7);
          const bool in = k < kend && c < a.M;
          uint4 v = bl16(arr, in ? static_cast<uint32_t>(k * a.lda + c) * 2u : kOOB);
          if (a.ones_row && c == a.M && k < kend) v.x = kOne;
          ra[j] = v;
        }
        if constexpr (TB) {  // B[n][k]
          const int r = n0 + (t >> 3) + 32 * j, c = k0 + 8 * (t & 7);
          const bool in = r < a.N && c < kend;
          rb[j] = bl16(brr, in ? static_cast<uint32_t>(r * a.ldb + c) * 2u : kOOB);
        } else {  // B[k][n]
          const int k = k0 + 2 * (t >> 3) + j, c = n0 + 8 * (t & 7);
          const bool in = k < kend && c < a.N;
          rb[j] = bl16(brr, in ? static_cast<uint32_t>(k * a.ldb + c) * 2u : kOOB);
        }
      } else {
        if constexpr (!TA)
          ra[j] = load_row8(a.A, a.lda, m0 + (t >> 3) + 32 * j, a.M, a.ones_row,
                            k0 + 8 * (t & 7), kend);
        else
          ra[j] = load_col8(a.A, a.lda, k0 + 2 * (t >> 3) + j, kend, m0 + 8 * (t & 7), a.M,
                            a.ones_row);
        if constexpr (TB)
          rb[j] = load_row8(a.B, a.ldb, n0 + (t >> 3) + 32 * j, a.N, false,
                            k0 + 8 * (t & 7), kend);
        else
          rb[j] = load_col8(a.B, a.ldb, k0 + 2 * (t >> 3) + j, kend, n0 + 8 * (t & 7), a.N,
                            false);
      }
    }
  };
  auto commit_op = [&](bf16_t* S, const uint4 (&r)[2], bool kcontig) __attribute__((always_inline)) {
    if (kcontig) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        *reinterpret_cast<uint4*>(S + ((t >> 3) + 32 * j) * PK + 8 * (t & 7)) = r[j];
    } else {
      // column c = 8 (t&7) + q gets the k pair (2 (t>>3), 2 (t>>3) + 1)
      unsigned* S32 = reinterpret_cast<unsigned*>(S);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const unsigned lo = (half(r[0], q >> 1) >> (16 * (q & 1))) & 0xFFFFu;
        const unsigned hi = (half(r[1], q >> 1) >> (16 * (q & 1))) & 0xFFFFu;
        S32[((8 * (t & 7) + q) * PK >> 1) + (t >> 3)] = lo | (hi << 16);
      }
    }
  };
  auto commit = [&](int buf) __attribute__((always_inline)) {
    commit_op(As[buf], ra, !TA);
    commit_op(Bs[buf], rb, TB);
  };

  f16v acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  // lane (row l32, half h) feeds k = 16 kk + 8 h + j (j = 0..7) of MFMA kk
  const int arow = (wm * 32 + l32) * PK + 8 * h;
  const int brow = (wn * 32 + l32) * PK + 8 * h;
  int buf = 0;
  if (kbeg < kend) {
    load(kbeg);
    commit(0);
    __syncthreads();
  }
  // branch-free loop body (the step after the last loads zeros - every k is
  // past the chunk - into the idle buffer, which nothing reads): with a
  // conditional load / commit the compiler copied the accumulators through
  // VGPRs at the loop header every step (gemm_f32.hip's finding)
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    load(k0 + BK);  // in flight under the MFMAs
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const s8v av = *reinterpret_cast<const s8v*>(&As[buf][arow + 16 * kk]);
      const s8v bv = *reinterpret_cast<const s8v*>(&Bs[buf][brow + 16 * kk]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
    }
    commit(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  // D[i][j]: j = lane & 31, i = (e & 3) + 8 (e >> 2) + 4 h
  const int n = n0 + wn * 32 + l32;
  if (a.splits > 1) {
    float* p = a.part + static_cast<int64_t>(blockIdx.z) * Mr * a.N;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int m = m0 + wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (m < Mr && n < a.N) p[static_cast<int64_t>(m) * a.N + n] = acc[e];
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int m = m0 + wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
    if (n >= a.N) continue;
    if (m < a.M) store_out(a.ep, m, n, acc[e]);
    else if (m == a.M && a.ones_row) a.ep.colsum[n] += acc[e];
  }
  if (a.ep.aug_c0 > 0 && blockIdx.y == 0) {
    const int naug = a.ep.ldc - a.ep.aug_c0;
    for (int e = t; e < BM * naug; e += 256) {
      const int m = m0 + e / naug;
      if (m < a.M) store_aug(a.ep, m, e % naug);
    }
  }
}

// Fixed-order sum of the split partials + the epilogue.
__global__ __launch_bounds__(256) void gemm_bf16_reduce_kernel(Args a) {
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
    if (i < static_cast<int64_t>(a.M) * naug)
      store_aug(a.ep, static_cast<int>(i / naug), static_cast<int>(i % naug));
  }
}

}  // namespace

int64_t gemm_bf16_part_floats(int M, int N, int K, int ones_row, int splits) {
  (void)K;
  return splits > 1 ? static_cast<int64_t>(splits) * (M + ones_row) * N : 0;
}

int gemm_bf16_splits(int M, int N, int K, int ones_row) {
  const int tiles = ((M + ones_row + BM - 1) / BM) * ((N + BN - 1) / BN);
  int s = 1;
  // enough workgroups to fill 256 CUs twice over (SA_GEMM16_WG_TARGET), each
  // K chunk >= 256 (SA_GEMM16_MIN_K)
  static const int target = std::max(1, sa::measure_knob("SA_GEMM16_WG_TARGET", 512));
  static const int min_k = std::max(32, sa::measure_knob("SA_GEMM16_MIN_K", 256));
  while (tiles * s < target && K / (2 * s) >= min_k && s < 16) s *= 2;
  return s;
}

bool gemm_bf16_launch(const uint16_t* A, const uint16_t* B, int M, int N, int K,
                      int lda, int ldb, bool ta, bool tb, bool ones_row, int splits,
                      float* part, const GemmBf16Epilogue& ep, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return false;
  if (lda % 8 || ldb % 8) return false;
  if (K % 8 && (!ta || tb)) return false;  // 16-B k chunks of a K-contiguous operand
  if (ones_row && ep.colsum == nullptr) return false;
  if (ep.accumulate && ep.c_bf16) return false;
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
  dim3 grid((Mr + BM - 1) / BM, (N + BN - 1) / BN, a.splits);
  // layout-specialised kernels; the branch-free buffer-load form needs whole
  // 8-element chunks along the M / N-contiguous operands and 32-bit offsets
  // (SA_GEMM_BL=0: bounds-checked loads)
  static const int blenv = sa::env_knob("SA_GEMM_BL", 1);
  const int64_t abytes = (ta ? static_cast<int64_t>(K) * lda : static_cast<int64_t>(M) * lda) * 2;
  const int64_t bbytes = (tb ? static_cast<int64_t>(N) * ldb : static_cast<int64_t>(K) * ldb) * 2;
  const bool bl = blenv && (!ta || M % 8 == 0) && (tb || N % 8 == 0) && abytes < 0xFFFFFF00ll &&
                  bbytes < 0xFFFFFF00ll;
  void (*kern)(Args);
  if (bl)
    kern = ta ? (tb ? gemm_bf16_kernel<true, true, true> : gemm_bf16_kernel<true, false, true>)
              : (tb ? gemm_bf16_kernel<false, true, true> : gemm_bf16_kernel<false, false, true>);
  else
    kern = ta ? (tb ? gemm_bf16_kernel<true, true, false> : gemm_bf16_kernel<true, false, false>)
              : (tb ? gemm_bf16_kernel<false, true, false> : gemm_bf16_kernel<false, false, false>);
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, a);
  if (a.splits > 1) {
    const int64_t total = static_cast<int64_t>(Mr) * N;
    const int64_t aug = ep.aug_c0 > 0 ? static_cast<int64_t>(M) * (ep.ldc - ep.aug_c0) : 0;
    const int64_t work = std::max(total, aug);
    hipLaunchKernelGGL(gemm_bf16_reduce_kernel, dim3(static_cast<unsigned>((work + 255) / 256)),
                       dim3(256), 0, stream, a);
  }
  return true;
}

}  // namespace sa
