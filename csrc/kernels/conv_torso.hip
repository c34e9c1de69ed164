// IMPALA deep-ResNet torso on gfx950: NHWC bf16 implicit-GEMM 3x3 convs on
// MFMA with every elementwise op of the reference graph fused in (SURVEY
// K1-K5', reference experiment.py:153-176 with TF-SAME padding):
//
//   conv1_pool_fwd  : uint8 frame (x/255 folded into W) -> conv3x3(3->16)+b ->
//                     maxpool 3x3/2 SAME; writes pooled bf16 + argmax (u8).
//                     The full-resolution conv output never touches HBM.
//   conv_pool_fwd   : conv3x3(Cin->Cout)+b -> maxpool (stages 2, 3).
//   res_conv_fwd    : relu-on-load -> conv3x3(C->C)+b [+ residual] [+ relu].
//   res_conv_bwd    : ONE pass per tile for dgrad AND wgrad AND bias grad:
//                     dx = [skip +] dgrad(dy) * (act > 0);
//                     dW += relu(act)^T dy (tr-read MFMA), db += sum dy.
//   pool_conv_bwd   : dY gathered from (dP, argmax) straight into LDS (never
//                     materialised), then dgrad + wgrad + bias grad.
//   conv1_pool_bwd  : the same for the uint8 first layer (wgrad only).
//
// Tiling: a workgroup (4 waves) owns R full-width rows of one image; pixels of
// the tile are linearised and processed in 16-pixel MFMA groups (a group may
// span rows).  Inputs are staged with a 1-pixel zero halo in LDS; D^T = W^T X^T
// puts 4 consecutive output channels of one pixel in each lane (8-byte NHWC
// stores).  Weight gradients accumulate in MFMA registers across all tiles a
// persistent workgroup visits and are flushed once with float atomics.
#include "conv_common.h"
#include "conv_launchers.h"

namespace sa {
namespace conv {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int GPW = 4;  // 16-pixel groups per wave per chunk

// ----------------------------------------------------------------- forward
// Per-wave implicit GEMM over a chunk of up to GPW groups. x_s: halo tile
// [rows][Wt+2][CIN]; output pixel q=(qr,qc) reads x_s[(qr+ky)*(Wt+2)+qc+kx].
// epi(q, co0, v[4]) is called for every valid (pixel, 4-channel slice).
template <int CIN, int COUT, typename Epi>
__device__ __forceinline__ void conv_tile_fwd(const bf16_t* x_s,
                                              const bf16_t* w_s, int Wt,
                                              int npix, Epi epi) {
  static_assert(CIN == 16 || CIN == 32, "CIN");
  constexpr int NH = COUT / 16;
  const int lane = lane_id();
  const int wave = wave_id();
  const int Wp = Wt + 2;
  const int ngroups = (npix + 15) / 16;
  for (int g0 = wave; g0 < ngroups; g0 += kWaves * GPW) {
    f4 acc[GPW][NH];
    int base[GPW];
#pragma unroll
    for (int gi = 0; gi < GPW; ++gi) {
#pragma unroll
      for (int h = 0; h < NH; ++h) acc[gi][h] = f4{0.f, 0.f, 0.f, 0.f};
      int q = (g0 + kWaves * gi) * 16 + (lane & 15);
      if (q >= npix) q = 0;
      const int qr = q / Wt, qc = q - (q / Wt) * Wt;
      base[gi] = (qr * Wp + qc) * CIN;
    }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap % 3;
      const int toff = (ky * Wp + kx) * CIN;
      if constexpr (CIN == 16) {
        s4 a[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h)
          a[h] = *reinterpret_cast<const s4*>(
              w_s + (tap * COUT + (lane & 15) + 16 * h) * CIN + 4 * (lane >> 4));
#pragma unroll
        for (int gi = 0; gi < GPW; ++gi) {
          if (g0 + kWaves * gi < ngroups) {
            const s4 b = *reinterpret_cast<const s4*>(x_s + base[gi] + toff +
                                                      4 * (lane >> 4));
#pragma unroll
            for (int h = 0; h < NH; ++h) acc[gi][h] = mfma16(a[h], b, acc[gi][h]);
          }
        }
      } else {
        bf8 a[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h)
          a[h] = *reinterpret_cast<const bf8*>(
              w_s + (tap * COUT + (lane & 15) + 16 * h) * CIN + 8 * (lane >> 4));
#pragma unroll
        for (int gi = 0; gi < GPW; ++gi) {
          if (g0 + kWaves * gi < ngroups) {
            const bf8 b = *reinterpret_cast<const bf8*>(x_s + base[gi] + toff +
                                                        8 * (lane >> 4));
#pragma unroll
            for (int h = 0; h < NH; ++h) acc[gi][h] = mfma32(a[h], b, acc[gi][h]);
          }
        }
      }
    }
#pragma unroll
    for (int gi = 0; gi < GPW; ++gi) {
      const int q = (g0 + kWaves * gi) * 16 + (lane & 15);
      if (g0 + kWaves * gi < ngroups && q < npix) {
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          float v[4] = {acc[gi][h][0], acc[gi][h][1], acc[gi][h][2], acc[gi][h][3]};
          epi(q, 16 * h + 4 * (lane >> 4), v);
        }
      }
    }
  }
}

__device__ __forceinline__ void store4(bf16_t* dst, const float v[4]) {
  uint2 o;
  o.x = static_cast<uint32_t>(f2bf(v[0])) | (static_cast<uint32_t>(f2bf(v[1])) << 16);
  o.y = static_cast<uint32_t>(f2bf(v[2])) | (static_cast<uint32_t>(f2bf(v[3])) << 16);
  *reinterpret_cast<uint2*>(dst) = o;
}
__device__ __forceinline__ void load4(const bf16_t* src, float v[4]) {
  const uint2 o = *reinterpret_cast<const uint2*>(src);
  v[0] = __uint_as_float(o.x << 16);
  v[1] = __uint_as_float(o.x & 0xFFFF0000u);
  v[2] = __uint_as_float(o.y << 16);
  v[3] = __uint_as_float(o.y & 0xFFFF0000u);
}

template <int C, bool RESID, bool POST_RELU>
__global__ __launch_bounds__(kThreads) void res_conv_fwd_kernel(
    const bf16_t* __restrict__ x, const float* __restrict__ w,
    const float* __restrict__ bias, const bf16_t* __restrict__ resid,
    bf16_t* __restrict__ y, int H, int W, int R) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* w_s = reinterpret_cast<bf16_t*>(smem);
  bf16_t* x_s = w_s + 9 * C * C;
  const int tiles_per_img = (H + R - 1) / R;
  const int n = blockIdx.x / tiles_per_img;
  const int r0 = (blockIdx.x - n * tiles_per_img) * R;
  const int Rv = min(R, H - r0);
  load_weights<C, C, true>(w, 1.f, w_s);
  load_halo_tile<C, true>(x, n, H, W, r0 - 1, Rv + 2, x_s);
  __syncthreads();
  const int64_t img0 = (static_cast<int64_t>(n) * H + r0) * W;
  conv_tile_fwd<C, C>(x_s, w_s, W, Rv * W, [&](int q, int co0, float v[4]) {
    const int64_t off = (img0 + q) * C + co0;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] += bias[co0 + i];
    if (RESID) {
      float r[4];
      load4(resid + off, r);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] += r[i];
    }
    if (POST_RELU) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], 0.f);
    }
    store4(y + off, v);
  });
}

// Max-pool 3x3/2 (TF SAME: pad_before pb, -inf padding) over a conv tile held
// in LDS y_s [Rc][W][COUT] whose row 0 is conv row cr0; writes pooled rows
// [i0, i0+Rpv).  8 channels per thread-iteration.
template <int COUT>
__device__ __forceinline__ void pool_tile(const bf16_t* y_s, int cr0, int H,
                                          int W, int Wo, int pb_h, int pb_w,
                                          int n, int Hp, int i0, int Rpv,
                                          bf16_t* __restrict__ pooled,
                                          uint8_t* __restrict__ argmax) {
  constexpr int CH = COUT / 8;
  const int total = Rpv * Wo * CH;
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    const int part = e % CH;
    const int pj = (e / CH) % Wo;
    const int pi = e / (CH * Wo);
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      best[c] = -INFINITY;
      arg[c] = 0;
    }
    const int crow0 = 2 * (i0 + pi) - pb_h;  // first conv row of the window
    const int ccol0 = 2 * pj - pb_w;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const int cr = crow0 + dy;
      if (cr < 0 || cr >= H) continue;
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int cc = ccol0 + dx;
        if (cc < 0 || cc >= W) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(
            y_s + ((cr - cr0) * W + cc) * COUT + part * 8);
        const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const float f = __uint_as_float((c & 1) ? (u[c >> 1] & 0xFFFF0000u)
                                                  : (u[c >> 1] << 16));
          if (f > best[c]) {
            best[c] = f;
            arg[c] = static_cast<uint8_t>(dy * 3 + dx);
          }
        }
      }
    }
    const int64_t o = ((static_cast<int64_t>(n) * Hp + i0 + pi) * Wo + pj) * COUT + part * 8;
    uint4 pv;
    pv.x = f2bf(best[0]) | (static_cast<uint32_t>(f2bf(best[1])) << 16);
    pv.y = f2bf(best[2]) | (static_cast<uint32_t>(f2bf(best[3])) << 16);
    pv.z = f2bf(best[4]) | (static_cast<uint32_t>(f2bf(best[5])) << 16);
    pv.w = f2bf(best[6]) | (static_cast<uint32_t>(f2bf(best[7])) << 16);
    *reinterpret_cast<uint4*>(pooled + o) = pv;
    uint2 av;
    av.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (static_cast<uint32_t>(arg[3]) << 24);
    av.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (static_cast<uint32_t>(arg[7]) << 24);
    *reinterpret_cast<uint2*>(argmax + o) = av;
  }
}

template <int CIN, int COUT>
__global__ __launch_bounds__(kThreads) void conv_pool_fwd_kernel(
    const bf16_t* __restrict__ x, const float* __restrict__ w,
    const float* __restrict__ bias, bf16_t* __restrict__ pooled,
    uint8_t* __restrict__ argmax, int H, int W, int Rp, int pb_h, int pb_w) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Hp = (H + 1) / 2, Wo = (W + 1) / 2;
  const int tiles_per_img = (Hp + Rp - 1) / Rp;
  const int n = blockIdx.x / tiles_per_img;
  const int i0 = (blockIdx.x - n * tiles_per_img) * Rp;
  const int Rpv = min(Rp, Hp - i0);
  const int cr0 = 2 * i0 - pb_h;
  const int Rc = 2 * Rpv + 1;
  bf16_t* w_s = reinterpret_cast<bf16_t*>(smem);
  bf16_t* x_s = w_s + 9 * CIN * COUT;
  bf16_t* y_s = x_s + (2 * Rp + 3) * (W + 2) * CIN;
  load_weights<CIN, COUT, true>(w, 1.f, w_s);
  load_halo_tile<CIN, false>(x, n, H, W, cr0 - 1, Rc + 2, x_s);
  __syncthreads();
  conv_tile_fwd<CIN, COUT>(x_s, w_s, W, Rc * W, [&](int q, int co0, float v[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] += bias[co0 + i];
    store4(y_s + q * COUT + co0, v);
  });
  __syncthreads();
  pool_tile<COUT>(y_s, cr0, H, W, Wo, pb_h, pb_w, n, Hp, i0, Rpv, pooled, argmax);
}

// First layer: uint8 RGB frame, K = 27 (tap*3+ci) padded to 32, one
// 16x16x32 MFMA per 16 pixels.  1/255 is folded into the bf16 weights; the
// raw byte values are exact in bf16.
__global__ __launch_bounds__(kThreads) void conv1_pool_fwd_kernel(
    const uint8_t* __restrict__ x, const float* __restrict__ w,
    const float* __restrict__ bias, bf16_t* __restrict__ pooled,
    uint8_t* __restrict__ argmax, int H, int W, int Rp, int pb_h, int pb_w) {
  constexpr int COUT = 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Hp = (H + 1) / 2, Wo = (W + 1) / 2;
  const int tiles_per_img = (Hp + Rp - 1) / Rp;
  const int n = blockIdx.x / tiles_per_img;
  const int i0 = (blockIdx.x - n * tiles_per_img) * Rp;
  const int Rpv = min(Rp, Hp - i0);
  const int cr0 = 2 * i0 - pb_h;
  const int Rc = 2 * Rpv + 1;
  const int Wp = W + 2;
  bf16_t* w_s = reinterpret_cast<bf16_t*>(smem);          // [16][32]
  bf16_t* y_s = w_s + COUT * 32;                           // [Rc][W][16]
  uint8_t* x_s = reinterpret_cast<uint8_t*>(y_s + (2 * Rp + 1) * W * COUT);
  for (int e = threadIdx.x; e < COUT * 32; e += blockDim.x) {
    const int co = e / 32, k = e % 32;
    w_s[e] = k < 27 ? f2bf(w[k * COUT + co] * (1.0f / 255.0f)) : 0;
  }
  load_halo_tile_u8(x, n, H, W, cr0 - 1, Rc + 2, x_s);
  __syncthreads();
  const int lane = lane_id();
  const int wave = wave_id();
  // per-lane k -> LDS byte offsets (relative to the output pixel's origin)
  int koff[8];
  bool kval[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * (lane >> 4) + j;
    kval[j] = k < 27;
    const int tap = k / 3, ci = k % 3;
    koff[j] = kval[j] ? ((tap / 3) * Wp + (tap % 3)) * 3 + ci : 0;
  }
  const bf8 a = *reinterpret_cast<const bf8*>(w_s + (lane & 15) * 32 + 8 * (lane >> 4));
  const int npix = Rc * W;
  const int ngroups = (npix + 15) / 16;
  for (int g = wave; g < ngroups; g += kWaves) {
    int q = g * 16 + (lane & 15);
    const bool valid = q < npix;
    if (!valid) q = 0;
    const int qr = q / W, qc = q - (q / W) * W;
    const uint8_t* px = x_s + (qr * Wp + qc) * 3;
    bf8 b;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      b[j] = kval[j] ? (__bf16)static_cast<float>(px[koff[j]]) : (__bf16)0.0f;
    f4 acc = mfma32(a, b, f4{0.f, 0.f, 0.f, 0.f});
    if (valid) {
      const int co0 = 4 * (lane >> 4);
      float v[4] = {acc[0] + bias[co0], acc[1] + bias[co0 + 1],
                    acc[2] + bias[co0 + 2], acc[3] + bias[co0 + 3]};
      store4(y_s + q * COUT + co0, v);
    }
  }
  __syncthreads();
  pool_tile<COUT>(y_s, cr0, H, W, Wo, pb_h, pb_w, n, Hp, i0, Rpv, pooled, argmax);
}

// ----------------------------------------------------------------- backward
// dgrad over the tile: dX[q][ci] = sum_tap W[tap][ci][co] dY[q - off][co]
// with dY in a halo tile d_s [rows][Wt+2][COUT] (output pixel q=(qr,qc) at
// halo (qr+1,qc+1); dY for tap (ky,kx) at (qr+2-ky, qc+2-kx)).
template <int CIN, int COUT, typename Epi>
__device__ __forceinline__ void conv_tile_dgrad(const bf16_t* d_s,
                                                const bf16_t* w_s, int Wt,
                                                int npix, Epi epi) {
  static_assert(COUT == 16 || COUT == 32, "COUT");
  constexpr int NH = CIN / 16;
  const int lane = lane_id();
  const int wave = wave_id();
  const int Wp = Wt + 2;
  const int ngroups = (npix + 15) / 16;
  for (int g0 = wave; g0 < ngroups; g0 += kWaves * GPW) {
    f4 acc[GPW][NH];
    int base[GPW];
#pragma unroll
    for (int gi = 0; gi < GPW; ++gi) {
#pragma unroll
      for (int h = 0; h < NH; ++h) acc[gi][h] = f4{0.f, 0.f, 0.f, 0.f};
      int q = (g0 + kWaves * gi) * 16 + (lane & 15);
      if (q >= npix) q = 0;
      const int qr = q / Wt, qc = q - (q / Wt) * Wt;
      base[gi] = (qr * Wp + qc) * COUT;  // + ((2-ky)*Wp + (2-kx))*COUT per tap
    }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap % 3;
      const int toff = ((2 - ky) * Wp + (2 - kx)) * COUT;
      if constexpr (COUT == 16) {
        s4 a[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h)
          a[h] = *reinterpret_cast<const s4*>(
              w_s + (tap * CIN + (lane & 15) + 16 * h) * COUT + 4 * (lane >> 4));
#pragma unroll
        for (int gi = 0; gi < GPW; ++gi) {
          if (g0 + kWaves * gi < ngroups) {
            const s4 b = *reinterpret_cast<const s4*>(d_s + base[gi] + toff +
                                                      4 * (lane >> 4));
#pragma unroll
            for (int h = 0; h < NH; ++h) acc[gi][h] = mfma16(a[h], b, acc[gi][h]);
          }
        }
      } else {
        bf8 a[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h)
          a[h] = *reinterpret_cast<const bf8*>(
              w_s + (tap * CIN + (lane & 15) + 16 * h) * COUT + 8 * (lane >> 4));
#pragma unroll
        for (int gi = 0; gi < GPW; ++gi) {
          if (g0 + kWaves * gi < ngroups) {
            const bf8 b = *reinterpret_cast<const bf8*>(d_s + base[gi] + toff +
                                                        8 * (lane >> 4));
#pragma unroll
            for (int h = 0; h < NH; ++h) acc[gi][h] = mfma32(a[h], b, acc[gi][h]);
          }
        }
      }
    }
#pragma unroll
    for (int gi = 0; gi < GPW; ++gi) {
      const int q = (g0 + kWaves * gi) * 16 + (lane & 15);
      if (g0 + kWaves * gi < ngroups && q < npix) {
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          float v[4] = {acc[gi][h][0], acc[gi][h][1], acc[gi][h][2], acc[gi][h][3]};
          epi(q, 16 * h + 4 * (lane >> 4), v);
        }
      }
    }
  }
}

// wgrad accumulators: wave w owns taps {w, w+4, w+8}; wave 1 (2 taps) also
// owns the bias pseudo-tap.  D[m=ci][n=co] per (tap, ci-half, co-half).
template <int CIN, int COUT>
struct WgradAcc {
  static constexpr int HC = CIN / 16, HO = COUT / 16;
  f4 w[3][HC][HO];
  f4 b[HO];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int c = 0; c < HC; ++c)
#pragma unroll
        for (int o = 0; o < HO; ++o) w[t][c][o] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int o = 0; o < HO; ++o) b[o] = f4{0.f, 0.f, 0.f, 0.f};
  }
};

// Accumulates dW += act^T dY over the tile's valid pixels.  a_s: halo tile of
// the (already relu'd if needed) conv input [rows][Wt+2][CIN]; d_s: halo tile
// of dY [rows][Wt+2][COUT]; zero_a / zero_d: offsets of an all-zero pixel.
template <int CIN, int COUT>
__device__ __forceinline__ void conv_tile_wgrad(const bf16_t* a_s,
                                                const bf16_t* d_s, int Wt,
                                                int npix, int zero_a,
                                                int zero_d,
                                                WgradAcc<CIN, COUT>& acc) {
  constexpr int HC = CIN / 16, HO = COUT / 16;
  const int lane = lane_id();
  const int wave = wave_id();
  const int Wp = Wt + 2;
  const int ngroups = (npix + 15) / 16;
  const int sub = lane & 15;
  const int qrow = sub >> 2;       // row of the 4x16 tr block
  const int pcol = (sub & 3) * 4;  // 4-element column chunk
  s4 ones;
  ones[0] = ones[1] = ones[2] = ones[3] = 0x3F80;  // bf16 1.0
  for (int g = 0; g < ngroups; ++g) {
    const int q = g * 16 + 4 * (lane >> 4) + qrow;
    const bool valid = q < npix;
    const int qr = valid ? q / Wt : 0;
    const int qc = valid ? q - qr * Wt : 0;
    const int pos = (qr + 1) * Wp + (qc + 1);
    s4 bd[HO];
#pragma unroll
    for (int o = 0; o < HO; ++o)
      bd[o] = lds_tr4(d_s + (valid ? pos * COUT : zero_d) + 16 * o + pcol);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int tap = wave + 4 * t;
      if (tap < 9) {
        const int ky = tap / 3, kx = tap % 3;
        const int apos = pos + (ky - 1) * Wp + (kx - 1);
#pragma unroll
        for (int c = 0; c < HC; ++c) {
          const s4 aa = lds_tr4(a_s + (valid ? apos * CIN : zero_a) + 16 * c + pcol);
#pragma unroll
          for (int o = 0; o < HO; ++o) acc.w[t][c][o] = mfma16(aa, bd[o], acc.w[t][c][o]);
        }
      }
    }
    if (wave == 1) {
#pragma unroll
      for (int o = 0; o < HO; ++o) acc.b[o] = mfma16(ones, bd[o], acc.b[o]);
    }
  }
}

template <int CIN, int COUT>
__device__ __forceinline__ void flush_wgrad(const WgradAcc<CIN, COUT>& acc,
                                            float scale, float* __restrict__ dw,
                                            float* __restrict__ db) {
  constexpr int HC = CIN / 16, HO = COUT / 16;
  const int lane = lane_id();
  const int wave = wave_id();
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int tap = wave + 4 * t;
    if (tap < 9) {
#pragma unroll
      for (int c = 0; c < HC; ++c)
#pragma unroll
        for (int o = 0; o < HO; ++o)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int ci = 16 * c + 4 * (lane >> 4) + i;
            const int co = 16 * o + (lane & 15);
            atomicAdd(dw + (tap * CIN + ci) * COUT + co, acc.w[t][c][o][i] * scale);
          }
    }
  }
  if (wave == 1 && (lane >> 4) == 0) {
#pragma unroll
    for (int o = 0; o < HO; ++o) atomicAdd(db + 16 * o + (lane & 15), acc.b[o][0]);
  }
}

template <int C, bool ADD_SKIP>
__global__ __launch_bounds__(kThreads) void res_conv_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ act,
    const bf16_t* __restrict__ skip, const float* __restrict__ w,
    bf16_t* __restrict__ dx, float* __restrict__ dw, float* __restrict__ db,
    int N, int H, int W, int R) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Wp = W + 2;
  const int tile_elems = (R + 2) * Wp * C;
  bf16_t* w_s = reinterpret_cast<bf16_t*>(smem);
  bf16_t* d_s = w_s + 9 * C * C;
  bf16_t* a_s = d_s + tile_elems + C;  // + one zero pixel each
  load_weights<C, C, false>(w, 1.f, w_s);
  for (int e = threadIdx.x; e < C; e += blockDim.x) {
    d_s[tile_elems + e] = 0;
    a_s[tile_elems + e] = 0;
  }
  WgradAcc<C, C> acc;
  acc.zero();
  const int tiles_per_img = (H + R - 1) / R;
  const int ntiles = N * tiles_per_img;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / tiles_per_img;
    const int r0 = (tile - n * tiles_per_img) * R;
    const int Rv = min(R, H - r0);
    __syncthreads();  // previous tile's LDS reads done
    load_halo_tile<C, false>(dy, n, H, W, r0 - 1, Rv + 2, d_s);
    load_halo_tile<C, true>(act, n, H, W, r0 - 1, Rv + 2, a_s);
    __syncthreads();
    const int npix = Rv * W;
    const int64_t img0 = (static_cast<int64_t>(n) * H + r0) * W;
    conv_tile_dgrad<C, C>(d_s, w_s, W, npix, [&](int q, int ci0, float v[4]) {
      const int qr = q / W, qc = q - (q / W) * W;
      float m[4];
      load4(a_s + ((qr + 1) * Wp + qc + 1) * C + ci0, m);
      const int64_t off = (img0 + q) * C + ci0;
      float s[4] = {0.f, 0.f, 0.f, 0.f};
      if (ADD_SKIP) load4(skip + off, s);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = s[i] + (m[i] > 0.f ? v[i] : 0.f);
      store4(dx + off, v);
    });
    conv_tile_wgrad<C, C>(a_s, d_s, W, npix, tile_elems, tile_elems, acc);
  }
  flush_wgrad<C, C>(acc, 1.f, dw, db);
}

// Gathers dY of the conv that feeds a max-pool, for the halo tile rows
// [cr0-1, cr0-1+rows) x cols [-1, W], from pooled grads dP and the argmax.
template <int COUT>
__device__ __forceinline__ void gather_pool_grad(
    const bf16_t* __restrict__ dP, const uint8_t* __restrict__ argmax, int n,
    int H, int W, int Hp, int Wo, int pb_h, int pb_w, int r_begin, int rows,
    bf16_t* d_s) {
  constexpr int CH = COUT / 8;
  const int Wp = W + 2;
  const int total = rows * Wp * CH;
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    const int part = e % CH;
    const int pix = e / CH;
    const int rr = pix / Wp;
    const int cc = pix - rr * Wp;
    const int r = r_begin + rr, c = cc - 1;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (r >= 0 && r < H && c >= 0 && c < W) {
      // windows i with 2i-pb <= r <= 2i-pb+2
      const int ilo = max(0, (r + pb_h - 1) / 2);  // ceil((r+pb-2)/2)
      const int ihi = min(Hp - 1, (r + pb_h) / 2);
      const int jlo = max(0, (c + pb_w - 1) / 2);
      const int jhi = min(Wo - 1, (c + pb_w) / 2);
      for (int i = ilo; i <= ihi; ++i) {
        const int dy = r - (2 * i - pb_h);
        for (int j = jlo; j <= jhi; ++j) {
          const int code = dy * 3 + (c - (2 * j - pb_w));
          const int64_t o = ((static_cast<int64_t>(n) * Hp + i) * Wo + j) * COUT + part * 8;
          const uint2 a = *reinterpret_cast<const uint2*>(argmax + o);
          const uint4 d = *reinterpret_cast<const uint4*>(dP + o);
          const uint32_t du[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t ab = ((k < 4 ? a.x : a.y) >> (8 * (k & 3))) & 0xFF;
            if (static_cast<int>(ab) == code)
              acc[k] += __uint_as_float((k & 1) ? (du[k >> 1] & 0xFFFF0000u)
                                                : (du[k >> 1] << 16));
          }
        }
      }
    }
    uint4 v;
    v.x = f2bf(acc[0]) | (static_cast<uint32_t>(f2bf(acc[1])) << 16);
    v.y = f2bf(acc[2]) | (static_cast<uint32_t>(f2bf(acc[3])) << 16);
    v.z = f2bf(acc[4]) | (static_cast<uint32_t>(f2bf(acc[5])) << 16);
    v.w = f2bf(acc[6]) | (static_cast<uint32_t>(f2bf(acc[7])) << 16);
    *reinterpret_cast<uint4*>(d_s + pix * COUT + part * 8) = v;
  }
}

template <int CIN, int COUT, bool NEED_DX>
__global__ __launch_bounds__(kThreads) void pool_conv_bwd_kernel(
    const bf16_t* __restrict__ dP, const uint8_t* __restrict__ argmax,
    const bf16_t* __restrict__ x, const float* __restrict__ w,
    bf16_t* __restrict__ dx, float* __restrict__ dw, float* __restrict__ db,
    int N, int H, int W, int R, int pb_h, int pb_w) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Wp = W + 2;
  const int Hp = (H + 1) / 2, Wo = (W + 1) / 2;
  const int d_elems = (R + 2) * Wp * COUT;
  const int x_elems = (R + 2) * Wp * CIN;
  bf16_t* w_s = reinterpret_cast<bf16_t*>(smem);
  bf16_t* d_s = w_s + 9 * CIN * COUT;
  bf16_t* x_s = d_s + d_elems + COUT;
  load_weights<CIN, COUT, false>(w, 1.f, w_s);
  for (int e = threadIdx.x; e < COUT; e += blockDim.x) d_s[d_elems + e] = 0;
  for (int e = threadIdx.x; e < CIN; e += blockDim.x) x_s[x_elems + e] = 0;
  WgradAcc<CIN, COUT> acc;
  acc.zero();
  const int tiles_per_img = (H + R - 1) / R;
  const int ntiles = N * tiles_per_img;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / tiles_per_img;
    const int r0 = (tile - n * tiles_per_img) * R;
    const int Rv = min(R, H - r0);
    __syncthreads();
    gather_pool_grad<COUT>(dP, argmax, n, H, W, Hp, Wo, pb_h, pb_w, r0 - 1,
                           Rv + 2, d_s);
    load_halo_tile<CIN, false>(x, n, H, W, r0 - 1, Rv + 2, x_s);
    __syncthreads();
    const int npix = Rv * W;
    if (NEED_DX) {
      const int64_t img0 = (static_cast<int64_t>(n) * H + r0) * W;
      conv_tile_dgrad<CIN, COUT>(d_s, w_s, W, npix, [&](int q, int ci0, float v[4]) {
        store4(dx + (img0 + q) * CIN + ci0, v);
      });
    }
    conv_tile_wgrad<CIN, COUT>(x_s, d_s, W, npix, x_elems, d_elems, acc);
  }
  flush_wgrad<CIN, COUT>(acc, 1.f, dw, db);
}

// First-layer weight gradient: dW[k=(tap,ci)][co] = sum_p x[p+off(tap)][ci]/255
// * dY[p][co]; K=27 rows as two 16-row MFMA m-tiles; A gathered from the u8
// halo tile, B = dY via transposed LDS reads.
__global__ __launch_bounds__(kThreads) void conv1_pool_bwd_kernel(
    const bf16_t* __restrict__ dP, const uint8_t* __restrict__ argmax,
    const uint8_t* __restrict__ x, float* __restrict__ dw,
    float* __restrict__ db, int N, int H, int W, int R, int pb_h, int pb_w) {
  constexpr int COUT = 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Wp = W + 2;
  const int Hp = (H + 1) / 2, Wo = (W + 1) / 2;
  const int d_elems = (R + 2) * Wp * COUT;
  bf16_t* d_s = reinterpret_cast<bf16_t*>(smem);
  uint8_t* x_s = reinterpret_cast<uint8_t*>(d_s + d_elems + COUT);
  for (int e = threadIdx.x; e < COUT; e += blockDim.x) d_s[d_elems + e] = 0;
  const int lane = lane_id();
  const int wave = wave_id();
  const int sub = lane & 15;
  // A row k (two m-tiles): offset of (tap, ci) relative to the pixel origin
  int koff[2];
  bool kval[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int k = sub + 16 * mt;
    kval[mt] = k < 27;
    const int tap = k / 3, ci = k % 3;
    koff[mt] = kval[mt] ? (((tap / 3) - 1) * Wp + ((tap % 3) - 1)) * 3 + ci : 0;
  }
  f4 accw[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  f4 accb = f4{0.f, 0.f, 0.f, 0.f};
  s4 ones;
  ones[0] = ones[1] = ones[2] = ones[3] = 0x3F80;
  const int tiles_per_img = (H + R - 1) / R;
  const int ntiles = N * tiles_per_img;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / tiles_per_img;
    const int r0 = (tile - n * tiles_per_img) * R;
    const int Rv = min(R, H - r0);
    __syncthreads();
    gather_pool_grad<COUT>(dP, argmax, n, H, W, Hp, Wo, pb_h, pb_w, r0 - 1,
                           Rv + 2, d_s);
    load_halo_tile_u8(x, n, H, W, r0 - 1, Rv + 2, x_s);
    __syncthreads();
    const int npix = Rv * W;
    const int ngroups = (npix + 15) / 16;
    for (int g = wave; g < ngroups; g += kWaves) {
      // B: dY rows (pixels 4(l>>4)+qrow of the group), channel columns
      const int qb = g * 16 + 4 * (lane >> 4) + (sub >> 2);
      const bool vb = qb < npix;
      const int qbr = vb ? qb / W : 0, qbc = vb ? qb - qbr * W : 0;
      const s4 bd = lds_tr4(d_s + (vb ? ((qbr + 1) * Wp + qbc + 1) * COUT : d_elems) +
                            (sub & 3) * 4);
      // A: rows k, columns = the 4 pixels 4(l>>4)+j of the group
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        s4 aa;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = g * 16 + 4 * (lane >> 4) + j;
          float v = 0.f;
          if (q < npix && kval[mt]) {
            const int qr = q / W, qc = q - (q / W) * W;
            v = static_cast<float>(x_s[((qr + 1) * Wp + qc + 1) * 3 + koff[mt]]);
          }
          aa[j] = static_cast<short>(f2bf(v));
        }
        accw[mt] = mfma16(aa, bd, accw[mt]);
      }
      accb = mfma16(ones, bd, accb);
    }
  }
  // flush: D[m=k][n=co] ; dw layout [k][co] (k = tap*3+ci, TF HWIO)
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = 16 * mt + 4 * (lane >> 4) + i;
      if (k < 27) atomicAdd(dw + k * COUT + sub, accw[mt][i] * (1.0f / 255.0f));
    }
  if ((lane >> 4) == 0) atomicAdd(db + sub, accb[0]);
}

int persistent_grid(int ntiles) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return ntiles < 2 * cus ? ntiles : 2 * cus;
}

template <typename K>
void set_smem(K kernel, size_t bytes) {
  if (bytes > 64 * 1024)
    hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                        hipFuncAttributeMaxDynamicSharedMemorySize,
                        static_cast<int>(bytes));
}

}  // namespace

// ----------------------------------------------------------------- launchers
int res_conv_rows(int H, int W) {
  int R = 192 / W;
  if (R < 1) R = 1;
  return R < H ? R : H;
}

void res_conv_fwd_launch(const void* x, const float* w, const float* b,
                         const void* resid, void* y, int N, int H, int W,
                         int C, bool post_relu, hipStream_t s) {
  const int R = res_conv_rows(H, W);
  const int grid = N * ((H + R - 1) / R);
  const size_t smem = (9 * C * C + (R + 2) * (W + 2) * C) * sizeof(bf16_t);
  auto X = static_cast<const bf16_t*>(x);
  auto RS = static_cast<const bf16_t*>(resid);
  auto Y = static_cast<bf16_t*>(y);
#define SA_RF(CC, RE, PR)                                                     \
  {                                                                           \
    auto k = res_conv_fwd_kernel<CC, RE, PR>;                                 \
    set_smem(k, smem);                                                        \
    hipLaunchKernelGGL(k, dim3(grid), dim3(kThreads), smem, s, X, w, b, RS,   \
                       Y, H, W, R);                                           \
  }
  const bool re = resid != nullptr;
  if (C == 16) {
    if (re && post_relu) SA_RF(16, true, true)
    else if (re) SA_RF(16, true, false)
    else SA_RF(16, false, false)
  } else {
    if (re && post_relu) SA_RF(32, true, true)
    else if (re) SA_RF(32, true, false)
    else SA_RF(32, false, false)
  }
#undef SA_RF
}

int pool_rows(int W, int CIN, int COUT, int Hp) {
  // ~480 conv pixels per tile, LDS <= 64 KB
  int Rp = (480 / W - 1) / 2;
  if (Rp < 1) Rp = 1;
  while (Rp > 1) {
    const size_t lds = (9 * CIN * COUT + (2 * Rp + 3) * (W + 2) * CIN +
                        (2 * Rp + 1) * W * COUT) * sizeof(bf16_t);
    if (lds <= 64 * 1024) break;
    --Rp;
  }
  return Rp < Hp ? Rp : Hp;
}

void conv_pool_fwd_launch(const void* x, const float* w, const float* b,
                          void* pooled, uint8_t* argmax, int N, int H, int W,
                          int CIN, int COUT, int pb_h, int pb_w, hipStream_t s) {
  const int Hp = (H + 1) / 2;
  const int Rp = pool_rows(W, CIN, COUT, Hp);
  const int grid = N * ((Hp + Rp - 1) / Rp);
  const size_t smem = (9 * CIN * COUT + (2 * Rp + 3) * (W + 2) * CIN +
                       (2 * Rp + 1) * W * COUT) * sizeof(bf16_t);
  auto X = static_cast<const bf16_t*>(x);
  auto P = static_cast<bf16_t*>(pooled);
#define SA_CP(CI, CO)                                                          \
  {                                                                            \
    auto k = conv_pool_fwd_kernel<CI, CO>;                                     \
    set_smem(k, smem);                                                         \
    hipLaunchKernelGGL(k, dim3(grid), dim3(kThreads), smem, s, X, w, b, P,     \
                       argmax, H, W, Rp, pb_h, pb_w);                          \
  }
  if (CIN == 16 && COUT == 32) SA_CP(16, 32)
  else if (CIN == 32 && COUT == 32) SA_CP(32, 32)
  else if (CIN == 16 && COUT == 16) SA_CP(16, 16)
  else if (CIN == 32 && COUT == 16) SA_CP(32, 16)
#undef SA_CP
}

void conv1_pool_fwd_launch(const uint8_t* x, const float* w, const float* b,
                           void* pooled, uint8_t* argmax, int N, int H, int W,
                           int pb_h, int pb_w, hipStream_t s) {
  const int Hp = (H + 1) / 2;
  int Rp = (480 / W - 1) / 2;
  if (Rp < 1) Rp = 1;
  if (Rp > Hp) Rp = Hp;
  const int grid = N * ((Hp + Rp - 1) / Rp);
  const size_t smem = (16 * 32 + (2 * Rp + 1) * W * 16) * sizeof(bf16_t) +
                      (2 * Rp + 3) * (W + 2) * 3;
  set_smem(conv1_pool_fwd_kernel, smem);
  hipLaunchKernelGGL(conv1_pool_fwd_kernel, dim3(grid), dim3(kThreads), smem,
                     s, x, w, b, static_cast<bf16_t*>(pooled), argmax, H, W,
                     Rp, pb_h, pb_w);
}

void res_conv_bwd_launch(const void* dy, const void* act, const void* skip,
                         const float* w, void* dx, float* dw, float* db, int N,
                         int H, int W, int C, hipStream_t s) {
  const int R = res_conv_rows(H, W);
  const int ntiles = N * ((H + R - 1) / R);
  const int grid = persistent_grid(ntiles);
  const size_t smem = (9 * C * C + 2 * ((R + 2) * (W + 2) * C + C)) * sizeof(bf16_t);
  auto DY = static_cast<const bf16_t*>(dy);
  auto A = static_cast<const bf16_t*>(act);
  auto SK = static_cast<const bf16_t*>(skip);
  auto DX = static_cast<bf16_t*>(dx);
#define SA_RB(CC, SKP)                                                         \
  {                                                                            \
    auto k = res_conv_bwd_kernel<CC, SKP>;                                     \
    set_smem(k, smem);                                                         \
    hipLaunchKernelGGL(k, dim3(grid), dim3(kThreads), smem, s, DY, A, SK, w,   \
                       DX, dw, db, N, H, W, R);                                \
  }
  if (C == 16) {
    if (skip) SA_RB(16, true) else SA_RB(16, false)
  } else {
    if (skip) SA_RB(32, true) else SA_RB(32, false)
  }
#undef SA_RB
}

void pool_conv_bwd_launch(const void* dP, const uint8_t* argmax, const void* x,
                          const float* w, void* dx, float* dw, float* db, int N,
                          int H, int W, int CIN, int COUT, int pb_h, int pb_w,
                          hipStream_t s) {
  // up to ~384 conv pixels per tile, LDS <= 60 KB
  int R = 384 / W;
  if (R < 1) R = 1;
  if (R > H) R = H;
  auto smem_of = [&](int r) {
    return (9 * CIN * COUT + (r + 2) * (W + 2) * (CIN + COUT) + CIN + COUT) *
           sizeof(bf16_t);
  };
  while (R > 1 && smem_of(R) > 60 * 1024) --R;
  const int ntiles = N * ((H + R - 1) / R);
  const int grid = persistent_grid(ntiles);
  const size_t smem = smem_of(R);
  auto DP = static_cast<const bf16_t*>(dP);
  auto X = static_cast<const bf16_t*>(x);
  auto DX = static_cast<bf16_t*>(dx);
#define SA_PB(CI, CO, NDX)                                                     \
  {                                                                            \
    auto k = pool_conv_bwd_kernel<CI, CO, NDX>;                                \
    set_smem(k, smem);                                                         \
    hipLaunchKernelGGL(k, dim3(grid), dim3(kThreads), smem, s, DP, argmax, X,  \
                       w, DX, dw, db, N, H, W, R, pb_h, pb_w);                 \
  }
  const bool ndx = dx != nullptr;
  if (CIN == 16 && COUT == 32) {
    if (ndx) SA_PB(16, 32, true) else SA_PB(16, 32, false)
  } else if (CIN == 32 && COUT == 32) {
    if (ndx) SA_PB(32, 32, true) else SA_PB(32, 32, false)
  } else if (CIN == 16 && COUT == 16) {
    if (ndx) SA_PB(16, 16, true) else SA_PB(16, 16, false)
  }
#undef SA_PB
}

void conv1_pool_bwd_launch(const void* dP, const uint8_t* argmax,
                           const uint8_t* x, float* dw, float* db, int N,
                           int H, int W, int pb_h, int pb_w, hipStream_t s) {
  int R = 384 / W;
  if (R < 1) R = 1;
  if (R > H) R = H;
  const int ntiles = N * ((H + R - 1) / R);
  const int grid = persistent_grid(ntiles);
  const size_t smem = ((R + 2) * (W + 2) * 16 + 16) * sizeof(bf16_t) +
                      (R + 2) * (W + 2) * 3;
  set_smem(conv1_pool_bwd_kernel, smem);
  hipLaunchKernelGGL(conv1_pool_bwd_kernel, dim3(grid), dim3(kThreads), smem,
                     s, static_cast<const bf16_t*>(dP), argmax, x, dw, db, N,
                     H, W, R, pb_h, pb_w);
}

}  // namespace conv
}  // namespace sa
