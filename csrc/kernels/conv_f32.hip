// Exact-fp32 NHWC conv kernels on v_mfma_f32_16x16x4_f32 (see conv_f32.h).
//
// MFMA operand maps (cdna_hip_programming.md §3, 16x16x4 f32):
//   A[i = l&15][k = l>>4], B[k = l>>4][j = l&15], D[i = 4(l>>4)+r][j = l&15].
// Forward / dgrad compute D^T = Wk^T X^T: i = output channel, j = pixel, so a
// lane ends with 4 consecutive channels of one pixel (one 16-B NHWC store).
// The k index of MFMA v in a 16-channel block b is channel 16b + 4g + v for
// lane group g = l>>4, on BOTH operands, so each lane fetches its 4 channels
// of a tap with one ds_read_b128 and feeds 4 consecutive MFMAs.
//
// Tiling (forward): a workgroup (4 waves) owns R full-width output rows of
// one image and an output-channel slice; the source rows it needs are staged
// into LDS once (zero padding / dilation / uint8 -> x/255 / ReLU applied on
// the way in), its weight slice as [tap][co][ci].  Pixels are linearised in
// 16-pixel MFMA groups, dealt round-robin to the waves, two at a time.
// LDS pixel pitches keep every ds_read_b128 group (4 x 16 lanes,
// MI355X_MICROARCH.md §LDS) conflict-free: pitch/4 = 2 mod 4 in 16-B units.
//
// Weight gradient: the reduction runs over pixels (k = 4 pixels per MFMA);
// rows i = (tap, ci) [+ one ones-row for the bias], columns j = co.  Waves
// split the rows (WSM groups) and/or the pixels (4/WSM groups, combined in
// LDS in a fixed order); each workgroup walks a fixed tile list and writes
// its partial sums, and one reduce kernel sums the partials in slot order:
// bitwise reproducible run to run (no float atomics).
#include "conv_f32.h"
#include "knobs.h"

#include <vector>

#include <utility>

#include <algorithm>
#include <cstdlib>
#include <cmath>

namespace sa {
namespace cf32 {

namespace {
int g_cu_reserve = -1;  // -1: not read yet (SA_CU_RESERVE)
}  // namespace

int conv_cu_reserve(int r) {
  if (g_cu_reserve < 0) {
    const int v = sa::measure_knob("SA_CU_RESERVE", 0);
    g_cu_reserve = v < 0 ? 0 : (v > 16 ? 16 : v);
  }
  const int old = g_cu_reserve;
  if (r >= 0 && r <= 16) g_cu_reserve = r;
  return old;
}

int conv_cus() { return 256 - 8 * conv_cu_reserve(-1); }

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kThreads = 256;
constexpr size_t kLdsSoft = 80 * 1024;   // two workgroups per CU
constexpr size_t kLdsHard = 156 * 1024;  // one workgroup per CU

// Launch-shape knobs (knobs.h measure_knob: measurement builds only; the
// defaults are the tuned values): resident workgroups per CU targeted by the
// persistent forward / stage-head grids (capped by LDS), and the maximum
// number of weight-gradient slots.
int occupancy(size_t lds_bytes, int cap) {
  const int fit = static_cast<int>((160 * 1024) / (lds_bytes + 512));
  return std::max(1, std::min(cap, fit));
}

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// pixel pitch (floats) of the forward LDS images: 16-B units = 2 mod 4
__host__ __device__ constexpr int fwd_pitch(int c) { return c >= 16 ? c + 8 : c; }
// pixel pitch of the wgrad input image: the A operand is read with
// ds_read_b32 (lane halves of 2 pixels x 16 consecutive channels), so the
// pitch is the smallest >= c that is 16 mod 32 dwords (16 -> 16, 32 -> 48;
// c + 16 made the 16-channel image 2-way bank conflicted: 2.8 conflict
// cycles per LDS instruction in rocprof)
__host__ __device__ constexpr int wg_pitch(int c) {
  return c >= 16 ? c + (48 - c % 32) % 32 : c;
}
static_assert(wg_pitch(16) == 16 && wg_pitch(32) == 48 && wg_pitch(64) == 80 &&
                  wg_pitch(128) == 144, "wg_pitch");

template <int VPL>
__device__ __forceinline__ void lds_get(const float* p, float (&v)[VPL]) {
  if constexpr (VPL == 4) {
    const f4 t = *reinterpret_cast<const f4*>(p);
    v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
  } else if constexpr (VPL == 2) {
    const f2 t = *reinterpret_cast<const f2*>(p);
    v[0] = t[0]; v[1] = t[1];
  } else {
    v[0] = *p;
  }
}

// Stages image rows [0, rows) x cols [0, Wl) (CINP channels, `pitch` floats
// per pixel) of the zero-padded, D-dilated source into LDS: image position
// (j0 + r, c - pl) holds source pixel ((j0 + r) / D, (c - pl) / D) when both
// are non-negative multiples of D inside the source, else zeros.
template <int CINP, int SRC>
__device__ __forceinline__ void stage_image(const void* __restrict__ src, int n, int Hs,
                                            int Ws, int Cs, int j0, int pl, int D,
                                            int rows, int Wl, int pitch, bool relu,
                                            float* __restrict__ x_s) {
  constexpr int CH = CINP / 4;
  const int total = rows * Wl * CH;
  for (int e = threadIdx.x; e < total; e += kThreads) {
    const int ch = e % CH;
    const int pix = e / CH;
    const int r = pix / Wl;
    const int c = pix - r * Wl;
    int j = j0 + r, i = c - pl;
    f4 v = {0.f, 0.f, 0.f, 0.f};
    bool ok = j >= 0 && i >= 0;
    if (D > 1) {
      ok = ok && (j % D) == 0 && (i % D) == 0;
      j /= D;
      i /= D;
    }
    ok = ok && j < Hs && i < Ws;
    if (ok) {
      const int64_t pixel = (static_cast<int64_t>(n) * Hs + j) * Ws + i;
      if constexpr (SRC == kSrcU8) {
        // tf.to_float(frame) / 255 (reference experiment.py:153-155)
        const uint8_t* p = static_cast<const uint8_t*>(src) + pixel * Cs;
        v[0] = static_cast<float>(p[0]) / 255.f;
        if (Cs > 1) v[1] = static_cast<float>(p[1]) / 255.f;
        if (Cs > 2) v[2] = static_cast<float>(p[2]) / 255.f;
        if (Cs > 3) v[3] = static_cast<float>(p[3]) / 255.f;
      } else {
        if (4 * ch < Cs) {
          v = *reinterpret_cast<const f4*>(static_cast<const float*>(src) + pixel * Cs +
                                           4 * ch);
          if (relu) {
            v[0] = fmaxf(v[0], 0.f); v[1] = fmaxf(v[1], 0.f);
            v[2] = fmaxf(v[2], 0.f); v[3] = fmaxf(v[3], 0.f);
          }
        }
      }
    }
    *reinterpret_cast<f4*>(x_s + pix * pitch + 4 * ch) = v;
  }
}

// ------------------------------------------------------------------ forward
// Persistent: each workgroup loads its weight slice into LDS ONCE and walks
// tiles blockIdx.x, blockIdx.x + gridDim.x, ...; the next tile's source
// chunks are loaded into registers (kMaxC 16-B chunks per thread, address
// math, padding/dilation/uint8 conversion/ReLU applied on load) while the
// current tile computes, and committed to LDS between two barriers.  Every
// wave computes all of its groups of the tile (<= kGmax, kept in registers)
// before the epilogue, so the epilogue's global loads (residual / mask) never
// force the in-flight prefetch to drain early (vmcnt is in order).
constexpr int kGmax = 4;   // 16-pixel groups per wave per tile
constexpr int kMaxC = 8;   // staged 16-B chunks per thread per tile
// forward staging depth per input width: 64+ channel layers (the shallow
// torso's 9x12 stage) need 16 chunks for a whole 5-row output image per tile
// instead of a 4-row tile plus a 1-row tail tile
// and 32-channel layers 9: the 18x24 res32 convs then take 8-row tiles (12
// MFMA groups = 3 per wave, balanced) instead of 7-row tiles (11 groups:
// 3,3,3,2 per wave, the short wave idling at the tile barrier)
__host__ __device__ constexpr int fwd_maxc(int cinp) {
  return cinp >= 64 ? 16 : (cinp == 32 ? 9 : kMaxC);
}

// Pre-pool gradient at (n, y, x), channels 4ch..4ch+3, gathered from the
// pooled gradient dP [N, Hp, Wp, C] through the argmax codes: windows in
// ascending (py, px) order, as maxpool_bwd_kernel (bitwise the same sums).
__device__ __forceinline__ f4 pool_grad_gather(const float* __restrict__ dP,
                                               const PoolGeom& pg, int n, int y, int x,
                                               int C, int ch) {
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const int py_hi = (y + pg.pbh) >> 1, px_hi = (x + pg.pbw) >> 1;
#pragma unroll
  for (int a = 1; a >= 0; --a) {
    const int py = py_hi - a;
    const int oy = y - (2 * py - pg.pbh);
    if (py < 0 || py >= pg.Hp || oy > 2) continue;
#pragma unroll
    for (int b = 1; b >= 0; --b) {
      const int px = px_hi - b;
      const int ox = x - (2 * px - pg.pbw);
      if (px < 0 || px >= pg.Wp || ox > 2) continue;
      const int64_t o = ((static_cast<int64_t>(n) * pg.Hp + py) * pg.Wp + px) * C + 4 * ch;
      const uint32_t codes = *reinterpret_cast<const uint32_t*>(pg.arg + o);
      const f4 gv = *reinterpret_cast<const f4*>(dP + o);
      const uint32_t want = static_cast<uint32_t>(oy * 3 + ox);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (((codes >> (8 * r)) & 0xFFu) == want) acc[r] += gv[r];
    }
  }
  return acc;
}

template <int CINP, int SRC, int MAXC = kMaxC>
struct Stager {
  static constexpr int CH = CINP / 4;
  f4 v[MAXC];
  // loads tile rows [0, rows) x [0, Wl) of the padded, D-dilated image of
  // source image n starting at source row j0 (see stage_image)
  __device__ __forceinline__ void load(const void* __restrict__ src, int n, int Hs, int Ws,
                                       int Cs, int j0, int pl, int D, int Wl, int total,
                                       bool relu, const PoolGeom& pg) {
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int e = threadIdx.x + k * kThreads;
      f4 x = {0.f, 0.f, 0.f, 0.f};
      if (e < total) {
        const int ch = e % CH;
        const int pix = e / CH;
        const int r = pix / Wl;
        const int c = pix - r * Wl;
        int j = j0 + r, i = c - pl;
        bool ok = j >= 0 && i >= 0;
        if (D > 1) {
          ok = ok && (j % D) == 0 && (i % D) == 0;
          j /= D;
          i /= D;
        }
        ok = ok && j < Hs && i < Ws;
        if (ok) {
          const int64_t pixel = (static_cast<int64_t>(n) * Hs + j) * Ws + i;
          if constexpr (SRC == kSrcU8) {
            const uint8_t* p = static_cast<const uint8_t*>(src) + pixel * Cs;
            x[0] = static_cast<float>(p[0]) / 255.f;
            if (Cs > 1) x[1] = static_cast<float>(p[1]) / 255.f;
            if (Cs > 2) x[2] = static_cast<float>(p[2]) / 255.f;
            if (Cs > 3) x[3] = static_cast<float>(p[3]) / 255.f;
          } else if constexpr (SRC == kSrcPoolGrad) {
            if (4 * ch < Cs) x = pool_grad_gather(static_cast<const float*>(src), pg, n, j, i, Cs, ch);
          } else if (4 * ch < Cs) {
            x = *reinterpret_cast<const f4*>(static_cast<const float*>(src) + pixel * Cs +
                                             4 * ch);
            if (relu) {
              x[0] = fmaxf(x[0], 0.f); x[1] = fmaxf(x[1], 0.f);
              x[2] = fmaxf(x[2], 0.f); x[3] = fmaxf(x[3], 0.f);
            }
          }
        }
      }
      v[k] = x;
    }
  }
  __device__ __forceinline__ void commit(float* x_s, int pitch, int total) const {
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int e = threadIdx.x + k * kThreads;
      if (e < total) {
        const int ch = e % CH, pix = e / CH;
        *reinterpret_cast<f4*>(x_s + pix * pitch + 4 * ch) = v[k];
      }
    }
  }
};

// Register prefetch of a contiguous [P pixels][CG of Cout channels] slice of
// dY (a tile of full rows) for the weight-gradient kernel.
template <int CG, int MAXD, bool GATHER>
struct DyStager {
  static constexpr int CH = CG / 4;
  f4 v[MAXD];
  // rows [oy0, oy0 + total / (Wo * CH)) of image n, channels co0 .. co0+CG;
  // GATHER: dy is the pooled gradient dP (see pool_grad_gather)
  __device__ __forceinline__ void load(const float* __restrict__ dy, int n, int oy0, int Ho,
                                       int Wo, int cout, int co0, int total,
                                       const PoolGeom& pg) {
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
      const int e = threadIdx.x + k * kThreads;
      f4 x = {0.f, 0.f, 0.f, 0.f};
      if (e < total) {
        const int ch = e % CH, p = e / CH;
        if constexpr (GATHER) {
          const int y = oy0 + p / Wo, xx = p - (p / Wo) * Wo;
          x = pool_grad_gather(dy, pg, n, y, xx, cout, co0 / 4 + ch);
        } else {
          x = *reinterpret_cast<const f4*>(
              dy + ((static_cast<int64_t>(n) * Ho + oy0) * Wo + p) * cout + co0 + 4 * ch);
        }
      }
      v[k] = x;
    }
  }
  __device__ __forceinline__ void commit(float* d_s, int pitch, int total) const {
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
      const int e = threadIdx.x + k * kThreads;
      if (e < total) {
        const int ch = e % CH, p = e / CH;
        *reinterpret_cast<f4*>(d_s + p * pitch + 4 * ch) = v[k];
      }
    }
  }
};
// x / d for 0 <= x < 2^20 and 1 <= d <= 2^10 via fp32: (x + 0.5) / d is at
// least 0.5 / d away from an integer, far above the fp32 rounding error of
// (x + 0.5) * rcp(d), so the truncation is exact (a 32-bit integer division
// is ~20 VALU instructions; this is 3).  rd = 1.f / d, computed once.
__device__ __forceinline__ int fdiv(int x, float rd) {
  return static_cast<int>((static_cast<float>(x) + 0.5f) * rd);
}

// compile-time loop: f(std::integral_constant<int, i>) for i = 0 .. N-1
template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int kMaxD = 8;  // staged dY chunks per thread per tile (taller tiles: more MFMA work per prefetch)

template <int CINP, int COUT_T, int K, int S, int SRC, bool FLIP>
__global__ __launch_bounds__(kThreads, 2) void conv_fwd_kernel(ConvArgs a, int R,
                                                               int tiles_per_img,
                                                               int ntiles) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int PP = fwd_pitch(CINP);
  constexpr int NH = COUT_T / 16;
  constexpr int VPL = CINP >= 16 ? 4 : CINP / 4;
  constexpr int NB = CINP >= 16 ? CINP / 16 : 1;
  constexpr int KK = K * K;
  static_assert(CINP == 4 || CINP == 8 || CINP % 16 == 0, "CINP");
  const int Wl = (a.Wo - 1) * S + K;
  const int rows = (R - 1) * S + K;
  const int total = rows * Wl * (CINP / 4);
  // weights as MFMA A fragments: [tap][b][g][co][VPL] (16-B lane reads,
  // consecutive lanes consecutive: conflict-free without padding)
  float* w_s = smem;
  float* x_s = smem + KK * CINP * COUT_T;  // [rows][Wl][PP]
  const int co0 = blockIdx.y * COUT_T;
  auto wput = [&](int tap, int o, int i, float v) {
    const int b = i / 16, rem = i - 16 * (i / 16);
    const int g = rem / VPL, v_ = rem - (rem / VPL) * VPL;
    w_s[(((tap * NB + b) * 4 + g) * COUT_T + o) * VPL + v_] = v;
  };
  if (!FLIP) {
    for (int e = threadIdx.x; e < KK * COUT_T * CINP; e += kThreads) {
      const int o = e % COUT_T, i = (e / COUT_T) % CINP, tap = e / (COUT_T * CINP);
      float v = 0.f;
      if (i < a.wcin) v = a.w[(static_cast<int64_t>(tap) * a.wcin + i) * a.wcout + co0 + o];
      wput(tap, o, i, v);
    }
  } else {
    // w_s[tap][o][i] = W[KK-1-tap][o][i]: o = input channel of the forward
    // conv (= dgrad output), i = its output channel (= dY channel)
    for (int e = threadIdx.x; e < KK * COUT_T * CINP; e += kThreads) {
      const int i = e % CINP, o = (e / CINP) % COUT_T, tap = e / (CINP * COUT_T);
      float v = 0.f;
      if (i < a.wcout)
        v = a.w[(static_cast<int64_t>(KK - 1 - tap) * a.wcin + co0 + o) * a.wcout + i];
      wput(tap, o, i, v);
    }
  }
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  float bias[NH][4];
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      bias[h][r] = a.bias != nullptr ? a.bias[co0 + 16 * h + 4 * g + r] : 0.f;
  const float* wl = w_s + (g * COUT_T + c16) * VPL;
  const float rwo = 1.f / static_cast<float>(a.Wo);

  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  Stager<CINP, SRC, fwd_maxc(CINP)> st;
  auto prefetch = [&](int t) {
    const int n = t / tiles_per_img;
    const int oy0 = (t - n * tiles_per_img) * R;
    st.load(a.src, n, a.Hs, a.Ws, a.Cs, oy0 * S - a.pt, a.pl, a.D, Wl, total,
            a.relu_in != 0, a.pool);
  };
  prefetch(tile);
  for (;;) {
    __syncthreads();  // the previous tile's LDS reads are done
    st.commit(x_s, PP, total);
    __syncthreads();
    const int cur = tile;
    tile += gridDim.x;
    // unconditional (the last tile re-stages itself, unused): a conditional
    // prefetch leaves a join at the loop back-edge
    prefetch(tile < ntiles ? tile : cur);  // in flight during the MFMAs below
    const int n = cur / tiles_per_img;
    const int oy0 = (cur - n * tiles_per_img) * R;
    const int P = min(R, a.Ho - oy0) * a.Wo;
    const int ngroups = (P + 15) >> 4;
    f4 acc[kGmax][NH];
    // groups wave + 4 i, two at a time (independent MFMA chains)
    auto mma = [&](auto NGc, int i0) {
      constexpr int NG = decltype(NGc)::value;
      int xb[NG];
#pragma unroll
      for (int gi = 0; gi < NG; ++gi) {
        const int p = (wave + 4 * (i0 + gi)) * 16 + c16;
        const int pp = p < P ? p : 0;
        const int oy = fdiv(pp, rwo), ox = pp - oy * a.Wo;
        xb[gi] = (oy * S * Wl + ox * S) * PP + VPL * g;
#pragma unroll
        for (int h = 0; h < NH; ++h) acc[i0 + gi][h] = f4{0.f, 0.f, 0.f, 0.f};
      }
      // software-pipelined over the KK * NB (tap, channel-block) steps: the
      // next step's operand reads are issued ahead of this step's MFMAs
      constexpr int STEPS = KK * NB;
      float av[2][NH][VPL], bv[2][NG][VPL];
      auto load_step = [&](int st, int buf) {
        const int tap = st / NB, b = st - (st / NB) * NB;
        const int ky = tap / K, kx = tap - (tap / K) * K;
        const int toff = (ky * Wl + kx) * PP;
#pragma unroll
        for (int h = 0; h < NH; ++h)
          lds_get<VPL>(wl + (((tap * NB + b) * 4) * COUT_T + 16 * h) * VPL, av[buf][h]);
#pragma unroll
        for (int gi = 0; gi < NG; ++gi)
          lds_get<VPL>(x_s + xb[gi] + toff + 16 * b, bv[buf][gi]);
      };
      load_step(0, 0);
#pragma unroll
      for (int st = 0; st < STEPS; ++st) {
        const int cur = st & 1;
        if (st + 1 < STEPS) load_step(st + 1, cur ^ 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int v = 0; v < VPL; ++v)
#pragma unroll
          for (int gi = 0; gi < NG; ++gi)
#pragma unroll
            for (int h = 0; h < NH; ++h)
              acc[i0 + gi][h] = mfma4(av[cur][h][v], bv[cur][gi][v], acc[i0 + gi][h]);
      }
    };
#pragma unroll
    for (int i = 0; i < kGmax; i += 2) {
      if (wave + 4 * i >= ngroups) break;
      if (wave + 4 * (i + 1) < ngroups)
        mma(std::integral_constant<int, 2>{}, i);
      else
        mma(std::integral_constant<int, 1>{}, i);
    }
    // epilogue (after all MFMAs of the tile)
    const int os = a.ostr > 0 ? a.ostr : 1;
    const int Hf = a.Hf > 0 ? a.Hf : a.Ho, Wf = a.Wf > 0 ? a.Wf : a.Wo;
#pragma unroll
    for (int i = 0; i < kGmax; ++i) {
      const int p = (wave + 4 * i) * 16 + c16;
      if (p >= P) continue;
      const int oy = fdiv(p, rwo), ox = p - oy * a.Wo;
      const int64_t pix = (static_cast<int64_t>(n) * Hf + (oy0 + oy) * os + a.ooy) * Wf +
                          ox * os + a.oox;
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        int64_t o = pix * a.Cout + co0 + 16 * h + 4 * g;
        if (a.phase_c > 0) {
          // phase-stacked dgrad: this 16-channel block is one phase's slice
          const int co = co0 + 16 * h;
          const int k = co / a.phase_c, ry = k / os, rx = k - (k / os) * os;
          const int yy = os * (oy0 + oy + a.ooy) + ry - a.pt_ph;
          const int xx = os * (ox + a.oox) + rx - a.pl_ph;
          if (yy < 0 || yy >= Hf || xx < 0 || xx >= Wf) continue;
          o = ((static_cast<int64_t>(n) * Hf + yy) * Wf + xx) * a.phase_c + (co - k * a.phase_c) +
              4 * g;
        }
        f4 v = acc[i][h];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bias[h][r];
        if (a.mask != nullptr) {
          const f4 m = *reinterpret_cast<const f4*>(a.mask + o);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = m[r] > 0.f ? v[r] : 0.f;
        }
        if (a.add != nullptr) {
          const f4 s = *reinterpret_cast<const f4*>(a.add + o);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += s[r];
        }
        if (a.relu_out) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        *reinterpret_cast<f4*>(a.out + o) = v;
      }
    }
    if (tile >= ntiles) break;
  }
}

// ------------------------------------------------------- fused conv + pool
// Stage head of the deep torso: conv3x3/1 SAME + bias, then the 3x3/2 SAME
// max-pool, in one persistent kernel.  A tile is R pooled rows of one image:
// its 2R+1 conv rows are computed into LDS (one row recomputed per tile
// boundary) and pooled from there, so the pre-pool map (4x the pooled size)
// never touches HBM.  Argmax codes as maxpool_fwd_kernel (first maximal tap).
template <int CINP, int COUT, int SRC>
__global__ __launch_bounds__(kThreads, 2) void conv_pool_fwd_kernel(
    ConvArgs a, int R, int tiles_per_img, int ntiles, int pbh, int pbw, int Hp, int Wp,
    float* __restrict__ pooled, uint8_t* __restrict__ parg) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int K = 3, KK = 9;
  constexpr int PP = fwd_pitch(CINP);
  constexpr int NH = COUT / 16;
  constexpr int VPL = CINP >= 16 ? 4 : CINP / 4;
  constexpr int NB = CINP >= 16 ? CINP / 16 : 1;
  constexpr int YP = COUT + 4;
  constexpr int C4 = COUT / 4;
  const int H = a.Ho, W = a.Wo;
  const int Wl = W + 2;
  const int CR = 2 * R + 1;
  const int rows = CR + 2;
  const int total = rows * Wl * (CINP / 4);
  float* w_s = smem;
  float* x_s = w_s + KK * CINP * COUT;
  // conv rows in LDS with a -inf column on each side (column c at c + 1) and
  // rows outside the image stored as -inf: the pool phase needs no bounds
  // masks and reads every tap at an immediate offset from a per-row base
  const int YW = W + 2;
  float* y_s = x_s + rows * Wl * PP;
  for (int e = threadIdx.x; e < CR * 2 * (YP / 4); e += kThreads) {
    const int q4 = e % (YP / 4), t = e / (YP / 4);
    const int col = (t & 1) ? W + 1 : 0;
    *reinterpret_cast<f4*>(y_s + ((t >> 1) * YW + col) * YP + 4 * q4) =
        f4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  }
  for (int e = threadIdx.x; e < KK * COUT * CINP; e += kThreads) {
    const int o = e % COUT, i = (e / COUT) % CINP, tap = e / (COUT * CINP);
    float v = 0.f;
    if (i < a.wcin) v = a.w[(static_cast<int64_t>(tap) * a.wcin + i) * a.wcout + o];
    const int b = i / 16, rem = i - 16 * (i / 16);
    const int g = rem / VPL, v_ = rem - (rem / VPL) * VPL;
    w_s[(((tap * NB + b) * 4 + g) * COUT + o) * VPL + v_] = v;
  }
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  float bias[NH][4];
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[h][r] = a.bias[16 * h + 4 * g + r];
  const float* wl = w_s + (g * COUT + c16) * VPL;
  const float rw = 1.f / static_cast<float>(W), rwp = 1.f / static_cast<float>(Hp > 0 ? Wp : 1);

  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  Stager<CINP, SRC> st;
  auto prefetch = [&](int t) {
    const int n = t / tiles_per_img;
    const int pi0 = (t - n * tiles_per_img) * R;
    st.load(a.src, n, a.Hs, a.Ws, a.Cs, 2 * pi0 - pbh - 1, 1, 1, Wl, total, false, a.pool);
  };
  prefetch(tile);
  const int P = CR * W;
  const int ngroups = (P + 15) >> 4;
  for (;;) {
    __syncthreads();  // previous tile: conv reads of x_s and pool reads of y_s done
    st.commit(x_s, PP, total);
    __syncthreads();
    const int cur = tile;
    tile += gridDim.x;
    prefetch(tile < ntiles ? tile : cur);  // unconditional: see conv_fwd_kernel
    const int n = cur / tiles_per_img;
    const int pi0 = (cur - n * tiles_per_img) * R;
    const int cr0 = 2 * pi0 - pbh;  // image row of the tile's conv row 0
    auto mma = [&](auto NGc, int g0) {
      constexpr int NG = decltype(NGc)::value;
      f4 acc[NG][NH];
      int xb[NG], q[NG];
      bool inimg[NG];
#pragma unroll
      for (int gi = 0; gi < NG; ++gi) {
        const int p = (g0 + 4 * gi) * 16 + c16;
        const int pp = p < P ? p : 0;
        const int oy = fdiv(pp, rw), ox = pp - oy * W;
        q[gi] = p < P ? (oy * YW + ox + 1) * YP : -1;
        inimg[gi] = cr0 + oy >= 0 && cr0 + oy < H;
        xb[gi] = (oy * Wl + ox) * PP + VPL * g;
#pragma unroll
        for (int h = 0; h < NH; ++h) acc[gi][h] = f4{0.f, 0.f, 0.f, 0.f};
      }
      constexpr int STEPS = KK * NB;
      float av[2][NH][VPL], bv[2][NG][VPL];
      auto load_step = [&](int st, int buf) {
        const int tap = st / NB, b = st - (st / NB) * NB;
        const int ky = tap / K, kx = tap - (tap / K) * K;
        const int toff = (ky * Wl + kx) * PP;
#pragma unroll
        for (int h = 0; h < NH; ++h)
          lds_get<VPL>(wl + (((tap * NB + b) * 4) * COUT + 16 * h) * VPL, av[buf][h]);
#pragma unroll
        for (int gi = 0; gi < NG; ++gi)
          lds_get<VPL>(x_s + xb[gi] + toff + 16 * b, bv[buf][gi]);
      };
      load_step(0, 0);
#pragma unroll
      for (int st = 0; st < STEPS; ++st) {
        const int cur = st & 1;
        if (st + 1 < STEPS) load_step(st + 1, cur ^ 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int v = 0; v < VPL; ++v)
#pragma unroll
          for (int gi = 0; gi < NG; ++gi)
#pragma unroll
            for (int h = 0; h < NH; ++h)
              acc[gi][h] = mfma4(av[cur][h][v], bv[cur][gi][v], acc[gi][h]);
      }
#pragma unroll
      for (int gi = 0; gi < NG; ++gi) {
        if (q[gi] < 0) continue;
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          f4 v = acc[gi][h];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = inimg[gi] ? v[r] + bias[h][r] : -INFINITY;
          *reinterpret_cast<f4*>(y_s + q[gi] + 16 * h + 4 * g) = v;
        }
      }
    };
    int grp = wave;
    if constexpr (CINP == 4) {
      // one MFMA per (tap, group): four groups in flight per wave cover the
      // LDS latency of the next tap's operands (two left the pipe idle)
      for (; grp + 12 < ngroups; grp += 16) mma(std::integral_constant<int, 4>{}, grp);
    }
    for (; grp + 4 < ngroups; grp += 8) mma(std::integral_constant<int, 2>{}, grp);
    if (grp < ngroups) mma(std::integral_constant<int, 1>{}, grp);
    __syncthreads();
    // pool the tile's conv rows: out-of-image taps read the -inf border /
    // rows, which never win the strict first-max compare
    const int Rv = min(R, Hp - pi0);
    const int nel = Rv * Wp * C4;
    for (int e = threadIdx.x; e < nel; e += kThreads) {
      const int c4 = e % C4;  // C4 is a power of two
      const int t = e / C4;
      const int pr = fdiv(t, rwp), pc = t - pr * Wp;
      // tap (0, 0): in-tile conv row 2 pr, column 2 pc - pbw (+1 border)
      const float* yb = y_s + ((2 * pr) * YW + 2 * pc - pbw + 1) * YP + 4 * c4;
      float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      int code[4] = {0, 0, 0, 0};
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const float* yr = yb + dy * YW * YP;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const f4 v = *reinterpret_cast<const f4*>(yr + dx * YP);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool gt = v[r] > best[r];
            best[r] = gt ? v[r] : best[r];
            code[r] = gt ? dy * 3 + dx : code[r];
          }
        }
      }
      const int64_t o = ((static_cast<int64_t>(n) * Hp + pi0 + pr) * Wp + pc) * COUT + 4 * c4;
      *reinterpret_cast<f4*>(pooled + o) = f4{best[0], best[1], best[2], best[3]};
      *reinterpret_cast<uint32_t*>(parg + o) =
          static_cast<uint32_t>(code[0]) | (static_cast<uint32_t>(code[1]) << 8) |
          (static_cast<uint32_t>(code[2]) << 16) | (static_cast<uint32_t>(code[3]) << 24);
    }
    if (tile >= ntiles) break;
  }
}

// ------------------------------------------------------------ weight grads
template <int CINP, int K, int S, int SRC, int NTT, int WSM, bool GATHER>
__global__ __launch_bounds__(kThreads) void conv_wgrad_kernel(WgradArgs a, int R,
                                                              int tiles_per_img,
                                                              int ntiles,
                                                              float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int M = K * K * CINP;
  // rows m < M: (tap, ci) of the image; row M: the bias ones-row (in the
  // last image tile's padding when M % 16 != 0, else one extra tile)
  constexpr int MT = (M + 16) / 16;
  constexpr int MTW = (MT + WSM - 1) / WSM;
  constexpr int PG = 4 / WSM;
  constexpr int XP = wg_pitch(CINP);
  constexpr int CG = NTT * 16;
  constexpr int DP = (CG % 32 == 0) ? CG + 16 : CG;
  const int Wl = (a.Wo - 1) * S + K;
  const int rows = (R - 1) * S + K;
  float* x_s = smem;
  float* d_s = smem + rows * Wl * XP;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int mg = wave % WSM, pg = wave / WSM;
  const int co0 = blockIdx.y * CG;
  int moff[MTW];
  float kconst[MTW];
  bool kimg[MTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    const int mb = mg + WSM * i;
    const int m = 16 * mb + c16;
    moff[i] = 0;
    kimg[i] = false;
    kconst[i] = 0.f;
    if (m < M) {
      const int tap = m / CINP, ci = m - (m / CINP) * CINP;
      const int ky = tap / K, kx = tap - (tap / K) * K;
      moff[i] = (ky * Wl + kx) * XP + ci;
      kimg[i] = true;
    } else if (m == M) {
      kconst[i] = 1.f;  // row M: sum of dY (bias gradient)
    }
  }
  f4 acc[MTW][NTT];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int nb = 0; nb < NTT; ++nb) acc[i][nb] = f4{0.f, 0.f, 0.f, 0.f};

  // persistent walk with the next tile's x / dY chunks prefetched into
  // registers while the current one computes
  Stager<CINP, SRC> sx;
  DyStager<CG, kMaxD, GATHER> sd;
  const int xtotal = rows * Wl * (CINP / 4);
  auto prefetch = [&](int t) {
    const int n = t / tiles_per_img;
    const int oy0 = (t - n * tiles_per_img) * R;
    sx.load(a.src, n, a.H, a.W, a.Cin, oy0 * S - a.pt, a.pl, 1, Wl, xtotal, a.relu_in != 0,
            a.pool);
    sd.load(a.dy, n, oy0, a.Ho, a.Wo, a.Cout, co0, min(R, a.Ho - oy0) * a.Wo * (CG / 4),
            a.pool);
  };
  int tile = blockIdx.x;
  if (tile < ntiles) prefetch(tile);
  while (tile < ntiles) {
    const int n = tile / tiles_per_img;
    const int oy0 = (tile - n * tiles_per_img) * R;
    const int Rv = min(R, a.Ho - oy0);
    const int P = Rv * a.Wo;
    __syncthreads();  // the previous tile's reads are done
    sx.commit(x_s, XP, xtotal);
    sd.commit(d_s, DP, P * (CG / 4));
    __syncthreads();
    const int cur_t = tile;
    tile += gridDim.x;
    prefetch(tile < ntiles ? tile : cur_t);  // unconditional: see conv_fwd_kernel
    const int nq = (P + 3) >> 2;
    if constexpr (CINP % 16 == 0 && WSM == 1) {
      // 16-channel-multiple inputs, one wave row set (res16 391 vs 438 us,
      // conv2 648 vs 715; the WSM = 2 res32 wgrad measured slower with it,
      // 342 vs 317 us, and keeps the generic loop): row block mb (16 rows m = 16 mb + c16) is
      // one tap and 16 consecutive input channels, so with the wave's block
      // set known at compile time (MG) every A-operand read is a per-ky lane
      // base plus an IMMEDIATE offset (no per-read address VALU), the
      // bias-row block is a per-lane constant, blocks past the last are
      // skipped, the pixel walk is branch-free and the two operand buffers
      // alternate without copies (valu/mfma 6.1 in rocprof before)
      auto run = [&](auto MGc) {
        constexpr int MG = decltype(MGc)::value;
        const int WlXP = Wl * XP;
        const int step = 4 * PG;
        const int dcy = step / a.Wo, dcx = step - (step / a.Wo) * a.Wo;
        int cy = (4 * pg + g) / a.Wo;
        int cx = (4 * pg + g) - cy * a.Wo;
        const float bias_row = c16 == 0 ? 1.f : 0.f;
        float a0[MTW], b0[NTT], a1[MTW], b1[NTT];
        auto load = [&](int qd, float (&av)[MTW], float (&bv)[NTT]) {
          const int p = 4 * qd + g;
          const bool valid = p < P;
          const int lb = valid ? (cy * S * Wl + cx * S) * XP + c16 : c16;
          const float* d = d_s + (valid ? p : 0) * DP + c16;
#pragma unroll
          for (int nb = 0; nb < NTT; ++nb) bv[nb] = valid ? d[16 * nb] : 0.f;
          int rb[K];
#pragma unroll
          for (int ky = 0; ky < K; ++ky) rb[ky] = lb + ky * WlXP;
          sfor<MTW>([&](auto Ic) {
            constexpr int i = decltype(Ic)::value;
            constexpr int mb = MG + WSM * i;
            if constexpr (16 * mb + 15 < M) {
              constexpr int tap = 16 * mb / CINP, ci0 = 16 * mb % CINP;
              av[i] = x_s[rb[tap / K] + (tap % K) * XP + ci0];
            } else if constexpr (16 * mb == M) {
              av[i] = bias_row;
            } else {
              av[i] = 0.f;
            }
          });
          cx += dcx;
          cy += dcy;
          const bool wrap = cx >= a.Wo;
          cx = wrap ? cx - a.Wo : cx;
          cy = wrap ? cy + 1 : cy;
        };
        auto mma = [&](const float (&av)[MTW], const float (&bv)[NTT]) {
          sfor<MTW>([&](auto Ic) {
            constexpr int i = decltype(Ic)::value;
            if constexpr (MG + WSM * i < MT) {
#pragma unroll
              for (int nb = 0; nb < NTT; ++nb) acc[i][nb] = mfma4(av[i], bv[nb], acc[i][nb]);
            }
          });
        };
        int qd = pg;
        if (qd < nq) load(qd, a0, b0);
        while (qd < nq) {
          if (qd + PG < nq) load(qd + PG, a1, b1);
          __builtin_amdgcn_sched_barrier(0);
          mma(a0, b0);
          qd += PG;
          if (qd >= nq) break;
          if (qd + PG < nq) load(qd + PG, a0, b0);
          __builtin_amdgcn_sched_barrier(0);
          mma(a1, b1);
          qd += PG;
        }
      };
      run(std::integral_constant<int, 0>{});
      continue;
    }
    // software-pipelined: quad qd+PG's operand reads are issued ahead of
    // quad qd's MFMAs.  The lane's pixel p = 4 qd + g advances by 4 PG per
    // quad: its (oy, ox) is stepped incrementally (no integer division in
    // the loop), and the row blocks that lie inside the image for every
    // wave need no bias-row select (compile-time).
    float av[MTW], bv[NTT];
    const int step = 4 * PG;
    int cy = 0, cx = 4 * pg + g;  // (oy, ox) of the next quad to load
    while (cx >= a.Wo) {
      cx -= a.Wo;
      ++cy;
    }
    auto load_quad = [&](int qd) {
      const int p = 4 * qd + g;
      const bool valid = p < P;
      const int pp = valid ? p : 0;
      const int xb = valid ? (cy * S * Wl + cx * S) * XP : 0;
#pragma unroll
      for (int nb = 0; nb < NTT; ++nb) {
        const float d = d_s[pp * DP + 16 * nb + c16];
        bv[nb] = valid ? d : 0.f;
      }
#pragma unroll
      for (int i = 0; i < MTW; ++i) {
        const float x = x_s[xb + moff[i]];
        // block i of every wave (mb <= WSM - 1 + WSM i) inside the image:
        // no select (folded at compile time after unrolling)
        av[i] = (16 * (WSM - 1 + WSM * i) + 15 < M) ? x : (kimg[i] ? x : kconst[i]);
      }
      cx += step;
      while (cx >= a.Wo) {
        cx -= a.Wo;
        ++cy;
      }
    };
    if (pg < nq) load_quad(pg);
    for (int qd = pg; qd < nq; qd += PG) {
      float ac[MTW], bc[NTT];
#pragma unroll
      for (int i = 0; i < MTW; ++i) ac[i] = av[i];
#pragma unroll
      for (int nb = 0; nb < NTT; ++nb) bc[nb] = bv[nb];
      if (qd + PG < nq) load_quad(qd + PG);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int nb = 0; nb < NTT; ++nb) acc[i][nb] = mfma4(ac[i], bc[nb], acc[i][nb]);
    }
  }

  float* dst = part + (static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * (MT * 16 * CG);
  if constexpr (PG == 1) {
#pragma unroll
    for (int i = 0; i < MTW; ++i) {
      const int mb = mg + WSM * i;
      if (mb >= MT) continue;
#pragma unroll
      for (int nb = 0; nb < NTT; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(16 * mb + 4 * g + r) * CG + 16 * nb + c16] = acc[i][nb][r];
    }
  } else {
    // the PG pixel groups' partial sums, added in a fixed order in LDS
    float* red = smem;  // [MT*16][CG]
    __syncthreads();
    for (int k = 0; k < PG; ++k) {
      if (pg == k) {
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
          const int mb = mg + WSM * i;
          if (mb >= MT) continue;
#pragma unroll
          for (int nb = 0; nb < NTT; ++nb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int idx = (16 * mb + 4 * g + r) * CG + 16 * nb + c16;
              red[idx] = (k == 0 ? 0.f : red[idx]) + acc[i][nb][r];
            }
        }
      }
      __syncthreads();
    }
    for (int e = threadIdx.x; e < MT * 16 * CG; e += kThreads) dst[e] = red[e];
  }
}

// Sums the G per-workgroup partials of every (row, co) in a fixed order and
// accumulates into dW (HWIO) / db.  64 elements per block, the slots split
// over the block's 4 waves (8 loads in flight per thread), the 4 wave sums
// combined in LDS in wave order: deterministic.
// Fixed-order sum of the per-workgroup weight-gradient slots: block = 16
// outputs x 16 slot groups (enough blocks to fill the GPU for the small
// 16/32-channel layers); slot group sg adds slots sg, sg+16, ... through 8
// independent accumulators, and the 16 groups are combined in LDS in a fixed
// tree order, so every run gives the same bits.
__device__ __forceinline__ void wgrad_reduce_body(
    const float* __restrict__ part, int G, int ngrp, int MT16, int CG, int CINP, int M,
    int Cin, int Cout, float* __restrict__ dw, float* __restrict__ db, int bid) {
  __shared__ float red[16][17];
  const int per = MT16 * CG;
  const int l = threadIdx.x & 15;
  const int e = bid * 16 + l;
  const int sg = threadIdx.x >> 4;
  const bool live = e < ngrp * per;
  const int ng = live ? e / per : 0, rem = live ? e - ng * per : 0;
  const int m = rem / CG, c = rem - (rem / CG) * CG;
  const bool want = live && ((m < M && (m % CINP) < Cin) || (db != nullptr && m == M));
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (want) {
    const float* p = part + static_cast<int64_t>(ng) * G * per + rem;
    for (int k = sg; k < G; k += 128) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int kk = k + 16 * u;
        if (kk < G) acc[u] += p[static_cast<int64_t>(kk) * per];
      }
    }
  }
  red[sg][l] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) +
               ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (sg != 0 || !want) return;
  float t[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    t[q] = (red[4 * q][l] + red[4 * q + 1][l]) + (red[4 * q + 2][l] + red[4 * q + 3][l]);
  const float s = (t[0] + t[1]) + (t[2] + t[3]);
  const int co = ng * CG + c;
  if (m < M) {
    const int tap = m / CINP, ci = m - (m / CINP) * CINP;
    dw[(static_cast<int64_t>(tap) * Cin + ci) * Cout + co] += s;
  } else {
    db[co] += s;
  }
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(
    const float* __restrict__ part, int G, int ngrp, int MT16, int CG, int CINP, int M,
    int Cin, int Cout, float* __restrict__ dw, float* __restrict__ db) {
  wgrad_reduce_body(part, G, ngrp, MT16, CG, CINP, M, Cin, Cout, dw, db, blockIdx.x);
}

// ------------------------------------------------- stage-head wgrad (scatter)
// Weight / bias gradient of a stage-head conv3x3/1 SAME (4 input channels,
// 16 output channels: the deep torso's first conv) straight from the pooled
// gradient dP and the max-pool's argmax codes.  The pre-pool gradient is
// dP routed to ONE position per (pooled pixel, channel), so
//   dW[ky,kx,ci,co] = sum_{n,py,px} dP[n,py,px,co] * X[n, y*+ky-1, x*+kx-1, ci]
// with (y*, x*) the argmax position of window (py, px) for channel co: a
// quarter of the dense pre-pool reduction's terms, and the dense pre-pool
// gradient (72x96x16 fp32 per frame, 4x the pooled map) is never written or
// read.  The patch depends on co, so this is VALU work (fp32 FMA, exact)
// with the input tile in LDS: thread = (pooled-pixel slot, co), 36 + 1
// accumulators.  Per-workgroup partials in the wgrad slot layout
// ([48 rows = tap*4 + ci, row 36 = bias][16 co]), summed by
// wgrad_reduce_kernel in slot order: bitwise reproducible.
constexpr int kPwRows = 2;  // pooled rows per tile
// LDS row pitch (16-B pixels) of the input tile: >= W + 2 and 5 mod 16.  A
// ds_read_b128 quarter-wave (16 lanes: two adjacent pooled pixels x 8 co)
// reads inside a 3-row x 5-column window; with the row pitch 5 mod 16 its 15
// positions fall in 15 distinct 16-B bank slots, so lanes either share an
// address (broadcast) or a slot never (the W + 2 pitch, 2 mod 16, measured
// 4.6 bank conflicts per LDS instruction in rocprof).
__host__ __device__ constexpr int pw_pitch(int W) { return W + 2 + ((5 - (W + 2)) % 16 + 16) % 16; }
static_assert(pw_pitch(96) == 101 && pw_pitch(84) == 101 && pw_pitch(3) == 5, "pw pitch");
// x: the fp32 4-channel image, or (u8_cs > 0) the uint8 frames themselves
// with u8_cs <= 4 channels, scaled by 1/255 on the way into LDS (the same
// tf.to_float(frame) / 255 as the forward, experiment.py:153-155)
// U8: the image is uint8 with u8_cs channels (x / 255 at staging), else the
// 4-channel fp32 image.  Compile-time: the runtime source switch cost the
// fp32 path 226 -> 334 us per call.
template <bool U8>
__global__ __launch_bounds__(kThreads) void pool_wgrad_kernel(
    const void* __restrict__ xsrc, int u8_cs, const float* __restrict__ dP,
    const uint8_t* __restrict__ arg, int H, int W, int Hp, int Wp, int pbh, int pbw,
    int tiles_per_img, int ntiles, float* __restrict__ part) {
  const f4* __restrict__ x = static_cast<const f4*>(xsrc);
  const uint8_t* __restrict__ xu = static_cast<const uint8_t*>(xsrc);
  extern __shared__ __attribute__((aligned(16))) f4 xs[];  // [2*kPwRows+3][W+2]
  const int co = threadIdx.x & 15, ps = threadIdx.x >> 4;
  const int Wl = pw_pitch(W);
  if constexpr (U8) {
    // exact x / 255 (the fp32 quotient the frame conversion produces)
    float* lut = reinterpret_cast<float*>(
        reinterpret_cast<uint32_t*>(xs + (2 * kPwRows + 3) * Wl) + (2 * kPwRows + 3) * 64 * 4);
    for (int i = threadIdx.x; i < 256; i += kThreads)
      lut[i] = static_cast<float>(static_cast<double>(i) / 255.0);
  }
  float acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[t][c] = 0.f;
  float accb = 0.f;
  constexpr int kPer = (kPwRows * 64 + 15) / 16;  // pooled pixels per thread (Wp <= 64)
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / tiles_per_img;
    const int py0 = (tile - n * tiles_per_img) * kPwRows;
    const int rp = min(kPwRows, Hp - py0);
    const int ybase = 2 * py0 - pbh - 1;  // image row of LDS row 0
    const int rows = 2 * rp + 3;
    const int np = rp * Wp;
    // this tile's pooled gradient and codes: loads in flight with the staging
    float g[kPer];
    uint32_t code[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int p = ps + 16 * k;
      g[k] = 0.f;
      code[k] = 0;
      if (p < np) {
        const int64_t o = (static_cast<int64_t>(n) * Hp + py0) * Wp * 16 + p * 16 + co;
        g[k] = dP[o];
        code[k] = arg[o];
      }
    }
    __syncthreads();  // the previous tile's LDS reads are done
    if constexpr (U8) {
      // the tile's frame rows as raw bytes (coalesced dword loads: a row is
      // W * u8_cs bytes, a multiple of 4 - the launcher checks), then each
      // LDS pixel expanded from them through the exact x / 255 table
      uint32_t* raw = reinterpret_cast<uint32_t*>(xs + (2 * kPwRows + 3) * Wl);
      const float* lut = reinterpret_cast<const float*>(raw + (2 * kPwRows + 3) * 64 * 4);
      const int rowd = W * u8_cs / 4;
      const uint32_t* src = reinterpret_cast<const uint32_t*>(xu);
      for (int d = threadIdx.x; d < rows * rowd; d += kThreads) {
        const int r = d / rowd, k = d - r * rowd;
        const int yy = ybase + r;
        uint32_t v = 0u;
        if (yy >= 0 && yy < H) v = src[(static_cast<int64_t>(n) * H + yy) * rowd + k];
        raw[r * rowd + k] = v;
      }
      __syncthreads();
      const uint8_t* rb = reinterpret_cast<const uint8_t*>(raw);
      for (int e = threadIdx.x; e < rows * Wl; e += kThreads) {
        const int r = e / Wl, c = e - r * Wl;
        const int xx = c - 1;
        f4 v = {0.f, 0.f, 0.f, 0.f};
        if (xx >= 0 && xx < W) {
          const uint8_t* q = rb + (r * W + xx) * u8_cs;
          v[0] = lut[q[0]];
          if (u8_cs > 1) v[1] = lut[q[1]];
          if (u8_cs > 2) v[2] = lut[q[2]];
          if (u8_cs > 3) v[3] = lut[q[3]];
        }
        xs[e] = v;
      }
    } else {
      for (int e = threadIdx.x; e < rows * Wl; e += kThreads) {
        const int r = e / Wl, c = e - r * Wl;
        const int yy = ybase + r, xx = c - 1;
        f4 v = {0.f, 0.f, 0.f, 0.f};
        if (yy >= 0 && yy < H && xx >= 0 && xx < W)
          v = x[(static_cast<int64_t>(n) * H + yy) * W + xx];
        xs[e] = v;
      }
    }
    __syncthreads();
    int pyl = 0, px = ps;  // (row, col) of pooled pixel p = ps + 16 k
    while (px >= Wp) {
      px -= Wp;
      ++pyl;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      if (ps + 16 * k < np) {
        const int dy = (code[k] * 11) >> 5;  // code / 3 for code <= 8
        const int dx = code[k] - 3 * dy;
        // LDS position of tap (0, 0): row 2 pyl + dy, col 2 px - pbw + dx
        // (the argmax never lies in the pool's padding; clamp for safety)
        const int base = max(0, (2 * pyl + dy) * Wl + 2 * px - pbw + dx);
        const float gv = g[k];
        accb += gv;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const f4 v = xs[base + ky * Wl + kx];
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[3 * ky + kx][c] = fmaf(gv, v[c], acc[3 * ky + kx][c]);
          }
      }
      px += 16;
      while (px >= Wp) {
        px -= Wp;
        ++pyl;
      }
    }
  }
  // sum the 16 pixel slots of each co in a fixed order: lanes co, co+16,
  // co+32, co+48 of a wave by butterfly, then the 4 waves through LDS
  __syncthreads();
  float* red = reinterpret_cast<float*>(xs);  // [4 waves][37][16]
  const int wave = threadIdx.x >> 6;
  auto wsum = [&](float v) {
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    return v;
  };
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float v = wsum(acc[t][c]);
      if ((threadIdx.x & 63) < 16) red[(wave * 37 + 4 * t + c) * 16 + co] = v;
    }
  {
    const float v = wsum(accb);
    if ((threadIdx.x & 63) < 16) red[(wave * 37 + 36) * 16 + co] = v;
  }
  __syncthreads();
  float* dst = part + static_cast<int64_t>(blockIdx.x) * (48 * 16);
  for (int e = threadIdx.x; e < 37 * 16; e += kThreads)
    dst[e] = (red[e] + red[37 * 16 + e]) + (red[2 * 37 * 16 + e] + red[3 * 37 * 16 + e]);
}

// The same fixed-order slot sum for small layers (total < 4096 outputs: the
// stage-0 scatter wgrad's 768, res16's 2560): block = 4 outputs x 64 slot
// groups, so the launch still fills the GPU (the 16 x 16 blocks gave the
// stage-0 reduction 48 workgroups and 38 us).
__device__ __forceinline__ void wgrad_reduce_narrow_body(
    const float* __restrict__ part, int G, int ngrp, int MT16, int CG, int CINP, int M,
    int Cin, int Cout, float* __restrict__ dw, float* __restrict__ db, int bid) {
  constexpr int OPB = 4, SG = 256 / OPB;
  __shared__ float red[SG][OPB + 1];
  const int per = MT16 * CG;
  const int l = threadIdx.x % OPB;
  const int e = bid * OPB + l;
  const int sg = threadIdx.x / OPB;
  const bool live = e < ngrp * per;
  const int ng = live ? e / per : 0, rem = live ? e - ng * per : 0;
  const int m = rem / CG, c = rem - (rem / CG) * CG;
  const bool want = live && ((m < M && (m % CINP) < Cin) || (db != nullptr && m == M));
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (want) {
    const float* p = part + static_cast<int64_t>(ng) * G * per + rem;
    for (int k = sg; k < G; k += 4 * SG) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kk = k + SG * u;
        if (kk < G) acc[u] += p[static_cast<int64_t>(kk) * per];
      }
    }
  }
  red[sg][l] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (sg != 0 || !want) return;
  float t[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < SG; q += 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] += red[q + j][l];
  }
  const float sum = (t[0] + t[1]) + (t[2] + t[3]);
  const int co = ng * CG + c;
  if (m < M) {
    const int tap = m / CINP, ci = m - (m / CINP) * CINP;
    dw[(static_cast<int64_t>(tap) * Cin + ci) * Cout + co] += sum;
  } else {
    db[co] += sum;
  }
}

__global__ __launch_bounds__(256) void wgrad_reduce_narrow_kernel(
    const float* __restrict__ part, int G, int ngrp, int MT16, int CG, int CINP, int M,
    int Cin, int Cout, float* __restrict__ dw, float* __restrict__ db) {
  wgrad_reduce_narrow_body(part, G, ngrp, MT16, CG, CINP, M, Cin, Cout, dw, db, blockIdx.x);
}

// One queued slot sum (deferred mode) and a batch of them for one launch:
// block b of the launch works for the job whose [first, first + blocks)
// range holds b (<= kMaxJobs jobs: a short scan of kernel arguments).
struct WgJob {
  const float* part;
  float* dw;
  float* db;
  int G, ngrp, MT16, CG, CINP, M, Cin, Cout;
  int narrow, blocks;
};
constexpr int kMaxJobs = 16;
struct WgJobs {
  WgJob job[kMaxJobs];
  int first[kMaxJobs + 1];
  int n;
};

__global__ __launch_bounds__(256) void wgrad_reduce_multi_kernel(WgJobs js) {
  int j = 0;
  while (j + 1 < js.n && static_cast<int>(blockIdx.x) >= js.first[j + 1]) ++j;
  const WgJob& q = js.job[j];
  const int bid = blockIdx.x - js.first[j];
  if (q.narrow)
    wgrad_reduce_narrow_body(q.part, q.G, q.ngrp, q.MT16, q.CG, q.CINP, q.M, q.Cin, q.Cout,
                             q.dw, q.db, bid);
  else
    wgrad_reduce_body(q.part, q.G, q.ngrp, q.MT16, q.CG, q.CINP, q.M, q.Cin, q.Cout, q.dw,
                      q.db, bid);
}

thread_local bool t_wg_defer = false;
thread_local std::vector<WgJob> t_wg_jobs;

// launches the fixed-order slot sum (the narrow form for small layers), or
// queues it in deferred mode
void wgrad_reduce(const float* part, int G, int ngrp, int MT16, int CG, int CINP, int M, int Cin,
                  int Cout, float* dw, float* db, hipStream_t s) {
  const int total = ngrp * MT16 * CG;
  if (t_wg_defer) {
    WgJob q{part, dw, db, G, ngrp, MT16, CG, CINP, M, Cin, Cout, total < 4096 ? 1 : 0,
            total < 4096 ? (total + 3) / 4 : (total + 15) / 16};
    t_wg_jobs.push_back(q);
    return;
  }
  if (total < 4096) {
    hipLaunchKernelGGL(wgrad_reduce_narrow_kernel, dim3((total + 3) / 4), dim3(256), 0, s, part,
                       G, ngrp, MT16, CG, CINP, M, Cin, Cout, dw, db);
  } else {
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((total + 15) / 16), dim3(256), 0, s, part, G,
                       ngrp, MT16, CG, CINP, M, Cin, Cout, dw, db);
  }
}

// ------------------------------------------------------------------ pooling
// Max-pool 3x3/2 (TF SAME) with first-max argmax codes.  Thread = 4 channels
// of one pooled pixel, threads laid out over (output row (n, py), element)
// flat; 32-bit index math (a 64-bit div/mod per element made the first
// version VALU bound), 64-bit row bases.  c4_shift = log2(C / 4).
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(
    const float* __restrict__ x, float* __restrict__ y, uint8_t* __restrict__ arg, int N,
    int H, int W, int C, int Hp, int Wp, int pb_h, int pb_w, int c4_shift) {
  // flat (row, element) index: rows narrower than a workgroup share one
  // (one workgroup per row left 25-62 % of the lanes idle at 12-24 columns)
  const unsigned rc = static_cast<unsigned>(Wp) << c4_shift;
  const unsigned flat = blockIdx.x * 256u + threadIdx.x;
  if (flat >= static_cast<unsigned>(N) * Hp * rc) return;
  const int row = static_cast<int>(flat / rc);  // n * Hp + py
  const int e = static_cast<int>(flat - static_cast<unsigned>(row) * rc);
  const int n = row / Hp, py = row - n * Hp;
  const int c4 = e & ((1 << c4_shift) - 1);
  const int px = e >> c4_shift;
  const float* img = x + static_cast<int64_t>(n) * H * W * C + 4 * c4;
  float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int code[4] = {0, 0, 0, 0};
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int yy = 2 * py - pb_h + dy;
    if (yy < 0 || yy >= H) continue;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int xx = 2 * px - pb_w + dx;
      if (xx < 0 || xx >= W) continue;
      const f4 v = *reinterpret_cast<const f4*>(img + (yy * W + xx) * C);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (v[r] > best[r]) {  // strict: the first maximal tap wins
          best[r] = v[r];
          code[r] = dy * 3 + dx;
        }
      }
    }
  }
  const int64_t o = static_cast<int64_t>(row) * Wp * C + 4 * e;
  *reinterpret_cast<f4*>(y + o) = f4{best[0], best[1], best[2], best[3]};
  *reinterpret_cast<uint32_t*>(arg + o) =
      static_cast<uint32_t>(code[0]) | (static_cast<uint32_t>(code[1]) << 8) |
      (static_cast<uint32_t>(code[2]) << 16) | (static_cast<uint32_t>(code[3]) << 24);
}

// Pool gradient for even H, W and pad-before 0 (the deep torso's 36x48 and
// 18x24 pools): thread = (pooled block (i, j), 4 channels) owning the 2x2
// pre-pool cells (2i + a, 2j + b).  Those cells can only be the argmax of
// windows (i-1, j-1), (i-1, j), (i, j-1), (i, j); each is loaded once (4
// dP + 4 code loads instead of 9 of each for the four cells separately) and
// the sums run in ascending (py, px) order: bitwise maxpool_bwd_kernel.
// Codes: window (py, px) tap (oy, ox) = oy * 3 + ox.
__global__ __launch_bounds__(256) void maxpool_bwd_blk_kernel(
    const float* __restrict__ dy, const uint8_t* __restrict__ arg, float* __restrict__ dx,
    int N, int Hp, int Wp, int C, int c4_shift) {
  const unsigned total = static_cast<unsigned>(N) * Hp * (static_cast<unsigned>(Wp) << c4_shift);
  const unsigned flat = blockIdx.x * 256u + threadIdx.x;
  if (flat >= total) return;
  const int c4 = static_cast<int>(flat & ((1u << c4_shift) - 1));
  const unsigned pix = flat >> c4_shift;  // (n, i, j)
  const int j = static_cast<int>(pix % static_cast<unsigned>(Wp));
  const unsigned ni = pix / static_cast<unsigned>(Wp);
  const int i = static_cast<int>(ni % static_cast<unsigned>(Hp));
  const int n = static_cast<int>(ni / static_cast<unsigned>(Hp));
  const int W = 2 * Wp;
  const int64_t pbase = static_cast<int64_t>(n) * Hp * Wp * C + 4 * c4;
  // windows: 0 = (i-1, j-1), 1 = (i-1, j), 2 = (i, j-1), 3 = (i, j)
  f4 g[4];
  uint32_t cd[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int py = i - 1 + (w >> 1), px = j - 1 + (w & 1);
    const bool in = py >= 0 && px >= 0;
    const int64_t o = pbase + static_cast<int64_t>(in ? py * Wp + px : 0) * C;
    g[w] = in ? *reinterpret_cast<const f4*>(dy + o) : f4{0.f, 0.f, 0.f, 0.f};
    cd[w] = in ? *reinterpret_cast<const uint32_t*>(arg + o) : 0xFFFFFFFFu;
  }
  auto add = [&](f4& acc, int w, uint32_t want) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (((cd[w] >> (8 * r)) & 0xFFu) == want) acc[r] += g[w][r];
  };
  f4 c00 = {0.f, 0.f, 0.f, 0.f}, c01 = c00, c10 = c00, c11 = c00;
  add(c00, 0, 8); add(c00, 1, 6); add(c00, 2, 2); add(c00, 3, 0);
  add(c01, 1, 7); add(c01, 3, 1);
  add(c10, 2, 5); add(c10, 3, 3);
  add(c11, 3, 4);
  float* row0 = dx + ((static_cast<int64_t>(n) * 2 * Hp + 2 * i) * W + 2 * j) * C + 4 * c4;
  float* row1 = row0 + static_cast<int64_t>(W) * C;
  *reinterpret_cast<f4*>(row0) = c00;
  *reinterpret_cast<f4*>(row0 + C) = c01;
  *reinterpret_cast<f4*>(row1) = c10;
  *reinterpret_cast<f4*>(row1 + C) = c11;
}

// Pool gradient gather: one grid row = one pre-pool row (n, y); thread = 4
// channels of one pixel (a flat layout as in maxpool_fwd measured slower here:
// 0.37 -> 0.41 ms/step), summing the (<= 4) windows whose argmax is this
// pixel in ascending (py, px) order (bitwise the sums of pool_grad_gather).
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(
    const float* __restrict__ dy, const uint8_t* __restrict__ arg, float* __restrict__ dx,
    int N, int H, int W, int C, int Hp, int Wp, int pb_h, int pb_w, int c4_shift) {
  const int row = blockIdx.x;  // n * H + y
  const int e = blockIdx.y * 256 + threadIdx.x;
  if (e >= (W << c4_shift)) return;
  const int n = row / H, y = row - n * H;
  const int c4 = e & ((1 << c4_shift) - 1);
  const int x = e >> c4_shift;
  const int64_t pbase = static_cast<int64_t>(n) * Hp * Wp * C + 4 * c4;
  const float* dP = dy + pbase;
  const uint8_t* ag = arg + pbase;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const int py_hi = (y + pb_h) >> 1, px_hi = (x + pb_w) >> 1;
#pragma unroll
  for (int a = 1; a >= 0; --a) {
    const int py = py_hi - a;
    const int oy = y - (2 * py - pb_h);
    if (py < 0 || py >= Hp || oy < 0 || oy > 2) continue;
#pragma unroll
    for (int b = 1; b >= 0; --b) {
      const int px = px_hi - b;
      const int ox = x - (2 * px - pb_w);
      if (px < 0 || px >= Wp || ox < 0 || ox > 2) continue;
      const int o = (py * Wp + px) * C;
      const uint32_t codes = *reinterpret_cast<const uint32_t*>(ag + o);
      const f4 g = *reinterpret_cast<const f4*>(dP + o);
      const uint32_t want = static_cast<uint32_t>(oy * 3 + ox);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (((codes >> (8 * r)) & 0xFFu) == want) acc[r] += g[r];
    }
  }
  *reinterpret_cast<f4*>(dx + static_cast<int64_t>(row) * W * C + 4 * e) = acc;
}

// uint8 frames [P, Cs<=4] -> [P, 4] fp32 x / 255 (tf.to_float(frame) / 255,
// reference experiment.py:153-155), zero-padded to 4 channels: the torso's
// first conv then stages one 16-B load per pixel instead of byte loads and
// divisions in every tile (and its weight gradient reuses the same image).
// uint8 frames [P pixels][Cs] -> the fp32 x / 255 image [P][4] (zero pad
// channels).  x / 255 comes from a 256-entry table of the correctly rounded
// quotients (computed in double: equal to the fp32 IEEE division for every
// byte), so the image is bitwise torch's / the reference's to_float / 255
// (experiment.py:153); the compiler's default fp32 division on gfx950 is
// not correctly rounded.
__global__ __launch_bounds__(256) void frames_f32_kernel(const uint8_t* __restrict__ x,
                                                         f4* __restrict__ y, int64_t P,
                                                         int Cs) {
  __shared__ float lut[256];
  lut[threadIdx.x] = static_cast<float>(static_cast<double>(threadIdx.x) / 255.0);
  __syncthreads();
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < P; i += stride) {
    const uint8_t* p = x + i * Cs;
    f4 v = {0.f, 0.f, 0.f, 0.f};
    v[0] = lut[p[0]];
    if (Cs > 1) v[1] = lut[p[1]];
    if (Cs > 2) v[2] = lut[p[2]];
    if (Cs > 3) v[3] = lut[p[3]];
    y[i] = v;
  }
}

// Same conversion, 1024 pixels per workgroup step: the tile's Cs * 1024
// bytes come in as coalesced dword loads (3 per thread for RGB) through LDS,
// then thread i writes pixels i + 256 k (k < 4), so each wave stores 1 KB
// contiguously.  (Per-pixel byte loads were the one-pixel kernel's limit;
// four pixels per thread straight from registers made the stores 64 B
// apart across the wave.)  Needs a 4-byte aligned source.
__global__ __launch_bounds__(256) void frames_f32_tile_kernel(const uint8_t* __restrict__ x,
                                                              f4* __restrict__ y, int64_t P,
                                                              int Cs) {
  __shared__ float lut[256];
  __shared__ uint32_t raw[1024];  // Cs * 1024 bytes, Cs <= 4
  lut[threadIdx.x] = static_cast<float>(static_cast<double>(threadIdx.x) / 255.0);
  const int64_t ntiles = (P + 1023) / 1024;
  const uint8_t* rb = reinterpret_cast<const uint8_t*>(raw);
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t p0 = t * 1024;
    const int np = static_cast<int>(P - p0 < 1024 ? P - p0 : 1024);
    const int nbytes = np * Cs;
    const uint8_t* src = x + p0 * Cs;
    __syncthreads();  // previous tile's LDS reads (and the table) done
    for (int d = threadIdx.x; 4 * d < nbytes; d += 256) {
      uint32_t v;
      if (4 * d + 4 <= nbytes) {
        v = reinterpret_cast<const uint32_t*>(src)[d];
      } else {
        v = 0;
        for (int b = 0; 4 * d + b < nbytes; ++b) v |= static_cast<uint32_t>(src[4 * d + b]) << (8 * b);
      }
      raw[d] = v;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = threadIdx.x + 256 * k;
      if (i < np) {
        const uint8_t* q = rb + i * Cs;
        f4 v = {0.f, 0.f, 0.f, 0.f};
        v[0] = lut[q[0]];
        if (Cs > 1) v[1] = lut[q[1]];
        if (Cs > 2) v[2] = lut[q[2]];
        if (Cs > 3) v[3] = lut[q[3]];
        y[p0 + i] = v;
      }
    }
  }
}

__global__ __launch_bounds__(256) void relu_mask_kernel(f4* __restrict__ dy,
                                                        const f4* __restrict__ ref,
                                                        int64_t n4) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n4; i += stride) {
    f4 v = dy[i];
    const f4 r = ref[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = r[k] > 0.f ? v[k] : 0.f;
    dy[i] = v;
  }
}

// ------------------------------------------------------------------ launch
template <typename Kern>
void allow_lds(Kern k, size_t bytes) {
  if (bytes > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             static_cast<int>(bytes));
    if (e != hipSuccess) (void)hipGetLastError();  // the launch reports it
  }
}

template <int CINP, int COUT_T, int K, int S, int SRC, bool FLIP>
bool run_conv(const ConvArgs& a, hipStream_t s) {
  constexpr int PP = fwd_pitch(CINP);
  const int Wl = (a.Wo - 1) * S + K;
  const size_t wbytes = static_cast<size_t>(4) * K * K * COUT_T * CINP;
  auto bytes = [&](int R) {
    return wbytes + static_cast<size_t>(4) * ((R - 1) * S + K) * Wl * PP;
  };
  const size_t budget = bytes(1) <= kLdsSoft ? kLdsSoft : kLdsHard;
  // tile height: fits LDS, the per-thread staging registers and kGmax groups
  // per wave; among those the one with the least busiest-wave work summed
  // over all tiles (+ a per-tile staging overhead)
  int best = 0;
  double best_cost = 1e30;
  for (int R = 1; R <= a.Ho; ++R) {
    const int rows = (R - 1) * S + K;
    if (bytes(R) > budget || rows * Wl * (CINP / 4) > fwd_maxc(CINP) * kThreads ||
        (R * a.Wo + 15) / 16 > 4 * kGmax)
      break;
    const int nt = (a.Ho + R - 1) / R;
    double cost = 0;
    for (int t = 0; t < nt; ++t) {
      const int rv = std::min(R, a.Ho - t * R);
      cost += ((rv * a.Wo + 15) / 16 + 3) / 4 + 0.4;
    }
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = R;
    }
  }
  if (best == 0) return false;
  const int R = best;
  const int nt = (a.Ho + R - 1) / R;
  const int ntiles = a.N * nt;
  const int gy = a.Cout / COUT_T;
  // 16-in/16-out layers gain from a third resident workgroup per CU (res16
  // fwd/dgrad 313 -> 284-292 us); 16->32 loses (518 -> 659 us)
  static const int occ_env = sa::measure_knob("SA_F32_FWD_OCC", 0);
  const int occ_cap = occ_env ? occ_env : (CINP <= 16 && COUT_T <= 16 ? 3 : 2);
  const int per_cu = occupancy(bytes(R), occ_cap);
  const int G = std::max(1, std::min(ntiles, conv_cus() * per_cu / gy));
  auto kern = conv_fwd_kernel<CINP, COUT_T, K, S, SRC, FLIP>;
  allow_lds(kern, bytes(R));
  hipLaunchKernelGGL(kern, dim3(G, gy), dim3(kThreads), bytes(R), s, a, R, nt, ntiles);
  return true;
}

template <int CINP, int COUT, int SRC>
bool run_conv_pool(const ConvArgs& a, int pbh, int pbw, float* pooled, uint8_t* arg,
                   hipStream_t s) {
  constexpr int PP = fwd_pitch(CINP);
  const int W = a.Wo, Wl = W + 2;
  const int Hp = (a.Ho + 1) / 2, Wp = (a.Wo + 1) / 2;
  auto bytes = [&](int R) {
    return static_cast<size_t>(4) *
           (9 * CINP * COUT + (2 * R + 3) * Wl * PP + (2 * R + 1) * (W + 2) * (COUT + 4));
  };
  const size_t budget = bytes(2) <= kLdsSoft ? kLdsSoft : kLdsHard;
  // pooled rows per tile cap: 2 for the 4-channel stage head (51.7 KB of LDS,
  // three workgroups per CU: 16.57 -> 16.46 ms/step against 3 rows, two)
  static const int rcap = sa::measure_knob("SA_F32_POOL_R", CINP == 4 ? 2 : 1 << 20);
  int R = 0;
  for (int r = 1; r <= std::min(Hp, rcap); ++r) {
    if (bytes(r) > budget || (2 * r + 3) * Wl * (CINP / 4) > kMaxC * kThreads) break;
    R = r;
  }
  if (R == 0) return false;
  const int nt = (Hp + R - 1) / R;
  R = (Hp + nt - 1) / nt;
  const int ntiles = a.N * nt;
  static const int occ_cap = sa::measure_knob("SA_F32_POOL_OCC", 3);
  const int per_cu = occupancy(bytes(R), occ_cap);
  const int G = std::max(1, std::min(ntiles, conv_cus() * per_cu));
  auto kern = conv_pool_fwd_kernel<CINP, COUT, SRC>;
  allow_lds(kern, bytes(R));
  hipLaunchKernelGGL(kern, dim3(G), dim3(kThreads), bytes(R), s, a, R, nt, ntiles, pbh, pbw,
                     Hp, Wp, pooled, arg);
  return true;
}

// output-channel tile: 32 when the weight slice stays small, else 16
int cout_tile(int cinp, int cout, int K) {
  static const int force = sa::measure_knob("SA_F32_COUT_T", 0);  // sweeps: 16 forces 16
  if (force == 16) return 16;
  if (cout % 32 == 0 && 4ll * K * K * 32 * cinp <= 48 * 1024) return 32;
  return 16;
}

template <int CINP, int K, int S, int SRC, int NTT, int WSM, bool GATHER>
bool run_wgrad(const WgradArgs& a, float* ws, hipStream_t s) {
  constexpr int M = K * K * CINP;
  constexpr int MT = (M + 16) / 16;
  constexpr int XP = wg_pitch(CINP);
  constexpr int CG = NTT * 16;
  constexpr int DP = (CG % 32 == 0) ? CG + 16 : CG;
  constexpr int PG = 4 / WSM;
  const int Wl = (a.Wo - 1) * S + K;
  const size_t red = PG > 1 ? static_cast<size_t>(4) * MT * 16 * CG : 0;
  auto bytes = [&](int R) {
    return std::max(red, static_cast<size_t>(4) * (((R - 1) * S + K) * Wl * XP + R * a.Wo * DP));
  };
  const size_t budget = bytes(1) <= kLdsSoft ? kLdsSoft : kLdsHard;
  // tallest tile that fits LDS and the per-thread prefetch registers
  int Rmax = 0;
  for (int R = 1; R <= a.Ho; ++R) {
    if (bytes(R) > budget || ((R - 1) * S + K) * Wl * (CINP / 4) > kMaxC * kThreads ||
        R * a.Wo * (CG / 4) > kMaxD * kThreads)
      break;
    Rmax = R;
  }
  if (Rmax == 0) return false;
  const int nt = (a.Ho + Rmax - 1) / Rmax;
  const int R = (a.Ho + nt - 1) / nt;
  const int ntiles = a.N * nt;
  const int ngrp = a.Cout / CG;
  const int G = static_cast<int>(
      std::min<int64_t>(ntiles, wgrad_slots(K, CINP, a.Cout)));
  auto kern = conv_wgrad_kernel<CINP, K, S, SRC, NTT, WSM, GATHER>;
  allow_lds(kern, bytes(R));
  hipLaunchKernelGGL(kern, dim3(G, ngrp), dim3(kThreads), bytes(R), s, a, R, nt, ntiles, ws);
  wgrad_reduce(ws, G, ngrp, MT * 16, CG, CINP, M, a.dw_cin > 0 ? a.dw_cin : a.Cin, a.Cout,
               a.dw, a.db, s);
  return true;
}

}  // namespace

void wgrad_reduce_slots(const float* part, int G, int rows16, int Cout, int Cin, float* dw,
                        float* db, hipStream_t s) {
  wgrad_reduce(part, G, 1, rows16, Cout, Cin, 9 * Cin, Cin, Cout, dw, db, s);
}

// Scatter-form stage-head wgrad from (dP, argmax) (pool_wgrad_kernel): on
// unless SA_F32_POOL_SCATTER=0 (then the dense-gather MFMA wgrad runs).
void wgrad_set_defer(bool on) { t_wg_defer = on; }

int wgrad_flush(hipStream_t s) {
  const int n = static_cast<int>(t_wg_jobs.size());
  for (int i0 = 0; i0 < n; i0 += kMaxJobs) {
    WgJobs js{};
    js.n = std::min(kMaxJobs, n - i0);
    int blocks = 0;
    for (int k = 0; k < js.n; ++k) {
      js.job[k] = t_wg_jobs[i0 + k];
      js.first[k] = blocks;
      blocks += js.job[k].blocks;
    }
    js.first[js.n] = blocks;
    hipLaunchKernelGGL(wgrad_reduce_multi_kernel, dim3(blocks), dim3(256), 0, s, js);
  }
  t_wg_jobs.clear();
  return n;
}

static bool pool_scatter_on() {
  static const bool on = sa::env_knob("SA_F32_POOL_SCATTER", 1) != 0;
  return on;
}
static bool pool_scatter_shape(int K, int S, int cinp, int cout) {
  return K == 3 && S == 1 && cinp == 4 && cout == 16;
}
// workgroups of a pool_wgrad launch (<= tiles): the resident count, 5 per CU
// at its 96 VGPRs (2-row tiles: 298 -> 228 us against 4-row tiles at 138
// VGPRs and 2048 slots)
constexpr int kPwSlots = 1280;

// Workgroup slots of a wgrad launch: the partials stay <= 8M floats, with at
// least 128 slots (before the tile-count cap) so the reduction fills the GPU.
int64_t wgrad_slots(int K, int cinp, int cout) {
  static const int cap = sa::measure_knob("SA_F32_WG_SLOTS", 512);
  const int64_t rows = ((K * K * cinp + 16) / 16) * 16;
  return std::max<int64_t>(128, std::min<int64_t>(cap, (8ll << 20) / (rows * cout)));
}

int64_t wgrad_workspace_floats(int K, int Cin, int Cout) {
  const int cinp = Cin <= 4 ? 4 : Cin;
  const int64_t rows = ((K * K * cinp + 16) / 16) * 16;
  int64_t n = wgrad_slots(K, cinp, Cout) * rows * Cout;
  if (pool_scatter_shape(K, 1, cinp, Cout)) n = std::max<int64_t>(n, int64_t{kPwSlots} * 48 * 16);
  return n;
}

bool conv_launch(const ConvArgs& a, int K, int S, int src, bool flip, hipStream_t s) {
  const int cinp = src == kSrcU8 ? 4 : a.Cs;
  if (src == kSrcU8 && (a.Cs < 1 || a.Cs > 4)) return false;
  if (src != kSrcU8 && a.Cs % 4 != 0) return false;
  if (src == kSrcPoolGrad && (a.pool.arg == nullptr || a.D != 1)) return false;
  if (K == 3 && S == 1 && src == kSrcF32 && wino_enabled() && wino_conv_launch(a, flip, s))
    return true;
  const int ct = cout_tile(cinp, a.Cout, K);
  if (a.Cout % ct != 0) return false;
#define SA_CONV_CASE(CINP, CT, KK, SS, SRC, FL)                                          \
  if (cinp == CINP && ct == CT && K == KK && S == SS && src == SRC && flip == FL)        \
    return run_conv<CINP, CT, KK, SS, SRC, FL>(a, s);
  // forward: deep ResNet (3x3/1; uint8 stage-1 input), shallow torso
  SA_CONV_CASE(4, 16, 3, 1, kSrcU8, false)
  SA_CONV_CASE(4, 16, 3, 1, kSrcF32, false)
  SA_CONV_CASE(4, 32, 8, 4, kSrcF32, false)
  SA_CONV_CASE(16, 16, 3, 1, kSrcF32, false)
  SA_CONV_CASE(16, 32, 3, 1, kSrcF32, false)
  SA_CONV_CASE(32, 32, 3, 1, kSrcF32, false)
  SA_CONV_CASE(32, 16, 3, 1, kSrcF32, false)  // SA_F32_COUT_T=16 sweeps
  SA_CONV_CASE(4, 32, 8, 4, kSrcU8, false)
  SA_CONV_CASE(32, 32, 4, 2, kSrcF32, false)
  SA_CONV_CASE(32, 16, 4, 2, kSrcF32, false)
  SA_CONV_CASE(64, 16, 3, 2, kSrcF32, false)
  SA_CONV_CASE(64, 32, 3, 2, kSrcF32, false)
  // data gradients (stride-1 correlation over the dilated dY)
  SA_CONV_CASE(16, 16, 3, 1, kSrcF32, true)
  SA_CONV_CASE(32, 16, 3, 1, kSrcF32, true)
  SA_CONV_CASE(32, 32, 3, 1, kSrcF32, true)
  SA_CONV_CASE(64, 16, 4, 1, kSrcF32, true)
  SA_CONV_CASE(128, 16, 3, 1, kSrcF32, true)
  // phase-decomposed dgrad of the shallow torso's stride-2 convs: one 2x2
  // sub-kernel per output phase over the undilated dY
  SA_CONV_CASE(64, 32, 2, 1, kSrcF32, true)
  SA_CONV_CASE(128, 16, 2, 1, kSrcF32, true)
  // data gradient of a stage-head conv straight from the pooled gradient
  SA_CONV_CASE(32, 16, 3, 1, kSrcPoolGrad, true)
  SA_CONV_CASE(32, 32, 3, 1, kSrcPoolGrad, true)
#undef SA_CONV_CASE
  return false;
}

static bool run_pool_wgrad(const WgradArgs& a, float* ws, int u8_cs, hipStream_t s) {
  const PoolGeom& pg = a.pool;
  // pooled 3x3/2 SAME geometry of the (stride-1) conv output, Wp <= 64
  if (pg.Hp != (a.Ho + 1) / 2 || pg.Wp != (a.Wo + 1) / 2 || pg.Wp > 64 || a.Ho != a.H ||
      a.Wo != a.W || a.pt != 1 || a.pl != 1 || a.relu_in || pg.pbh < 0 || pg.pbh > 1 ||
      pg.pbw < 0 || pg.pbw > 1)
    return false;
  const int tpi = (pg.Hp + kPwRows - 1) / kPwRows;
  const int ntiles = a.N * tpi;
  static const int slots = std::max(1, std::min(kPwSlots, sa::measure_knob("SA_F32_PW_SLOTS", kPwSlots)));
  const int G = std::min(ntiles, slots);
  size_t lds = std::max<size_t>(sizeof(float) * 4 * (2 * kPwRows + 3) * pw_pitch(a.W),
                                sizeof(float) * 4 * 37 * 16);
  if (u8_cs > 0) {
    // raw byte rows (W * u8_cs <= 256 dwords per row) + the 256-entry table
    // after the f4 image; rows must be whole dwords
    if ((a.W * u8_cs) % 4 != 0 || a.W * u8_cs > 1024) return false;
    lds = std::max<size_t>(lds, sizeof(float) * 4 * (2 * kPwRows + 3) * pw_pitch(a.W) +
                                    sizeof(uint32_t) * (2 * kPwRows + 3) * 256 +
                                    sizeof(float) * 256);
    allow_lds(pool_wgrad_kernel<true>, lds);
    hipLaunchKernelGGL(pool_wgrad_kernel<true>, dim3(G), dim3(kThreads), lds, s, a.src,
                       u8_cs, a.dy, pg.arg, a.H, a.W, pg.Hp, pg.Wp, pg.pbh, pg.pbw, tpi,
                       ntiles, ws);
  } else {
    allow_lds(pool_wgrad_kernel<false>, lds);
    hipLaunchKernelGGL(pool_wgrad_kernel<false>, dim3(G), dim3(kThreads), lds, s, a.src,
                       u8_cs, a.dy, pg.arg, a.H, a.W, pg.Hp, pg.Wp, pg.pbh, pg.pbw, tpi,
                       ntiles, ws);
  }
  wgrad_reduce(ws, G, 1, 48, 16, 4, 36, a.dw_cin > 0 ? a.dw_cin : a.Cin, a.Cout, a.dw, a.db, s);
  return true;
}

bool wgrad_launch(const WgradArgs& a, int K, int S, int src, float* ws, hipStream_t s) {
  if (K == 3 && S == 1 && src == kSrcF32 && wino_wgrad_enabled() && wino_wgrad_launch(a, ws, s))
    return true;
  const int cinp = src == kSrcU8 ? 4 : a.Cin;
  if (src == kSrcU8 && (a.Cin < 1 || a.Cin > 4)) return false;
  if (src == kSrcF32 && a.Cin % 4 != 0) return false;
  const bool gather = a.pool.arg != nullptr;
  if (gather && (src == kSrcF32 || src == kSrcU8) && pool_scatter_on() &&
      pool_scatter_shape(K, S, cinp, a.Cout) &&
      run_pool_wgrad(a, ws, src == kSrcU8 ? a.Cin : 0, s))
    return true;
#define SA_WG_CASE(CINP, KK, SS, SRC, COUT, NTT, WSM)                                     \
  if (cinp == CINP && K == KK && S == SS && src == SRC && a.Cout == COUT) {               \
    if (gather) return run_wgrad<CINP, KK, SS, SRC, NTT, WSM, true>(a, ws, s);            \
    return run_wgrad<CINP, KK, SS, SRC, NTT, WSM, false>(a, ws, s);                       \
  }
  SA_WG_CASE(4, 3, 1, kSrcU8, 16, 1, 1)
  SA_WG_CASE(4, 3, 1, kSrcF32, 16, 1, 1)
  SA_WG_CASE(4, 8, 4, kSrcF32, 32, 2, 2)
  SA_WG_CASE(4, 3, 1, kSrcU8, 32, 2, 1)
  SA_WG_CASE(16, 3, 1, kSrcF32, 16, 1, 1)
  SA_WG_CASE(16, 3, 1, kSrcF32, 32, 2, 1)
  SA_WG_CASE(32, 3, 1, kSrcF32, 32, 2, 2)
  SA_WG_CASE(4, 8, 4, kSrcU8, 32, 2, 2)
  SA_WG_CASE(32, 4, 2, kSrcF32, 64, 4, 4)
  SA_WG_CASE(64, 3, 2, kSrcF32, 128, 4, 4)
#undef SA_WG_CASE
  return false;
}

bool conv_pool_fwd_launch(const ConvArgs& a, int src, int pbh, int pbw, float* pooled,
                          uint8_t* arg, hipStream_t s) {
  if (src == kSrcU8 && a.Cs <= 4 && a.Cout == 16) return run_conv_pool<4, 16, kSrcU8>(a, pbh, pbw, pooled, arg, s);
  if (src == kSrcF32 && a.Cs == 4 && a.Cout == 16) return run_conv_pool<4, 16, kSrcF32>(a, pbh, pbw, pooled, arg, s);
  if (src == kSrcF32 && a.Cs == 16 && a.Cout == 32) return run_conv_pool<16, 32, kSrcF32>(a, pbh, pbw, pooled, arg, s);
  if (src == kSrcF32 && a.Cs == 32 && a.Cout == 32) return run_conv_pool<32, 32, kSrcF32>(a, pbh, pbw, pooled, arg, s);
  return false;
}

static int c4_shift_of(int C) {
  const int c4 = C / 4;
  int sh = 0;
  while ((1 << sh) < c4) ++sh;
  return (C % 4 == 0 && (1 << sh) == c4) ? sh : -1;
}

bool maxpool_fwd_launch(const float* x, float* y, uint8_t* arg, int N, int H, int W, int C,
                        int Hp, int Wp, int pb_h, int pb_w, hipStream_t s) {
  const int sh = c4_shift_of(C);
  if (sh < 0) return false;
  const uint64_t total = static_cast<uint64_t>(N) * Hp * (static_cast<unsigned>(Wp) << sh);
  if (total >= (1ull << 32)) return false;
  const dim3 grid(static_cast<unsigned>((total + 255) / 256));
  hipLaunchKernelGGL(maxpool_fwd_kernel, grid, dim3(256), 0, s, x, y, arg, N, H, W, C, Hp,
                     Wp, pb_h, pb_w, sh);
  return true;
}

bool maxpool_bwd_launch(const float* dy, const uint8_t* arg, float* dx, int N, int H, int W,
                        int C, int Hp, int Wp, int pb_h, int pb_w, hipStream_t s) {
  const int sh = c4_shift_of(C);
  if (sh < 0) return false;
  static const bool blk = sa::env_knob("SA_F32_POOL_BWD_BLK", 1) != 0;
  if (blk && pb_h == 0 && pb_w == 0 && H == 2 * Hp && W == 2 * Wp) {
    const int64_t total = static_cast<int64_t>(N) * Hp * (static_cast<int64_t>(Wp) << sh);
    if (total < (int64_t{1} << 31)) {
      hipLaunchKernelGGL(maxpool_bwd_blk_kernel, dim3(static_cast<unsigned>((total + 255) / 256)),
                         dim3(256), 0, s, dy, arg, dx, N, Hp, Wp, C, sh);
      return true;
    }
  }
  const dim3 grid(static_cast<unsigned>(N) * H, ((W << sh) + 255) / 256);
  hipLaunchKernelGGL(maxpool_bwd_kernel, grid, dim3(256), 0, s, dy, arg, dx, N, H, W, C, Hp,
                     Wp, pb_h, pb_w, sh);
  return true;
}

void frames_f32_launch(const uint8_t* x, float* y, int64_t P, int Cs, hipStream_t s) {
  static const bool tiled = sa::env_knob("SA_FRAMES_TILE", 1) != 0;  // 0: one pixel per thread
  if (tiled && (reinterpret_cast<uintptr_t>(x) & 3) == 0 && Cs >= 1 && Cs <= 4) {
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((P + 1023) / 1024, 8192));
    hipLaunchKernelGGL(frames_f32_tile_kernel, dim3(blocks), dim3(256), 0, s, x,
                       reinterpret_cast<f4*>(y), P, Cs);
    return;
  }
  int64_t blocks = std::min<int64_t>((P + 255) / 256, 8192);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(frames_f32_kernel, dim3(blocks), dim3(256), 0, s, x,
                     reinterpret_cast<f4*>(y), P, Cs);
}

void relu_mask_launch(float* dy, const float* ref, int64_t n, hipStream_t s) {
  const int64_t n4 = n / 4;
  int64_t blocks = std::min<int64_t>((n4 + 255) / 256, 4096);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(relu_mask_kernel, dim3(blocks), dim3(256), 0, s,
                     reinterpret_cast<f4*>(dy), reinterpret_cast<const f4*>(ref), n4);
}

}  // namespace cf32
}  // namespace sa
