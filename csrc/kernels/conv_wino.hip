// Winograd F(2x2, 3x3) fp32 convolution for the deep torso's 3x3 / stride-1
// SAME convs (forward and data gradient), on v_mfma_f32_16x16x4_f32.
//
// Reference: experiment.py:156-176 (IMPALA ResNet: conv3x3/1 stage heads and
// residual convs, fp32).  The reference ran them through cuDNN in fp32,
// whose autotuner picks a Winograd algorithm for exactly these shapes; this
// is the MI355X-native equivalent: fp32 in / fp32 accumulate everywhere
// (no reduced-precision MFMA exists for f32 on gfx950), 2.25x fewer MFMA
// multiply-adds than the direct implicit GEMM of conv_f32.hip.
//
//   Y(2x2 tile) = A^T [ sum_ci (G g_ci,co G^T) .* (B^T d_ci B) ] A
//
// The 16 element-wise products (xi = 4a + b) are 16 small GEMMs over the
// input channels: M[xi][co][tile] = sum_ci U[xi][co][ci] V[xi][ci][tile].
// MFMA mapping (16x16x4 f32: A[i=l&15][k=l>>4], B[k][j=l&15],
// D[i=4(l>>4)+r][j=l&15]): i = output channel, j = tile, k = input channel.
//   * U = G g G^T is computed once per workgroup into LDS as MFMA A
//     fragments [xi][ci-block][g][co][4] (16-B lane reads, conflict-free);
//   * V = B^T d B is computed IN THE LANE that feeds it to the MFMA: lane
//     (tile j, channel quad g) reads its tile's 4x4 input patch for 4
//     channels (16 ds_read_b128) and transforms it in registers, so V never
//     touches LDS;
//   * the 16 M accumulators of a lane hold all 16 xi for 4 consecutive
//     output channels of ONE tile, so the output transform A^T M A, bias,
//     ReLU-mask, residual add, ReLU and the NHWC stores are in registers too.
//
// Work decomposition: tiles are numbered (image, tile row, tile column) over
// the whole batch; a persistent workgroup walks ranges of RT consecutive
// tiles (a range may cross images), stages the input rows its tiles need
// (shared halo rows, zero padding, optional ReLU on load) into LDS through a
// register prefetch issued one range ahead, and its waves take (16-tile
// group, output-channel slice) tasks.  Every range but the batch's last is
// full, so the waves stay balanced for any image size.
#include "conv_f32.h"

#include <algorithm>
#include <cstdlib>

namespace sa {
namespace cf32 {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kMaxParts = 4;  // images one range may touch

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// x / d for 0 <= x < 2^22, 1 <= d <= 2^10 (exact: (x + 0.5) / d lies at
// least 0.5 / d from an integer, far above the fp32 product's error)
__device__ __forceinline__ int fdivi(int x, float rd) {
  return static_cast<int>((static_cast<float>(x) + 0.5f) * rd);
}

struct WinoArgs {
  const float* src;   // [N, H, W, CIN]
  const float* w;     // HWIO [3, 3, wcin, wcout] (forward conv's weights)
  const float* bias;  // [COUT] or null
  const float* mask;  // [N, H, W, COUT] or null
  const float* add;   // [N, H, W, COUT] or null
  float* out;         // [N, H, W, COUT]
  int N, H, W;
  int TY, TX, NT, nranges;
  float rTX, rTY, rWl;
  int wcin, wcout, flip;
  int relu_in, relu_out;
  int maxrows;  // LDS row capacity (>= rows of every range)
  int ablate;  // measurement knob (SA_WINO_ABLATE): 1 no tasks, 2 no global
               // loads, 4 no LDS commit, 8 no stores
};

// Rows staged for a range: image part p (image n0 + p) contributes input
// rows 2 tya_p - 1 .. 2 tyb_p + 2 at LDS rows off_p ...; a tile (n, ty) of
// part p has its 4x4 patches at LDS row off_p + 2 (ty - tya_p).
struct RangeGeom {
  int t0, t1, n0;
  int off1, off2, off3, tya0, rows;
};

__device__ __forceinline__ RangeGeom range_geom(const WinoArgs& a, int r, int RT) {
  RangeGeom g;
  g.t0 = r * RT;
  g.t1 = min(g.t0 + RT, a.NT);
  const int R0 = fdivi(g.t0, a.rTX);
  const int R1 = fdivi(g.t1 - 1, a.rTX);
  g.n0 = fdivi(R0, a.rTY);
  const int n1 = fdivi(R1, a.rTY);
  g.tya0 = R0 - g.n0 * a.TY;
  int off[kMaxParts + 1];
  off[0] = 0;
#pragma unroll
  for (int p = 0; p < kMaxParts; ++p) {
    const int n = g.n0 + p;
    const int tya = p == 0 ? g.tya0 : 0;
    const int tyb = n == n1 ? R1 - n1 * a.TY : a.TY - 1;
    off[p + 1] = off[p] + (n <= n1 ? 2 * (tyb - tya) + 4 : 0);
  }
  g.off1 = off[1];
  g.off2 = off[2];
  g.off3 = off[3];
  g.rows = off[4];
  return g;
}

template <int CIN, int COUT, int NH, int NW, int RT, int MAXC, int WPS>
__global__ __launch_bounds__(64 * NW, WPS) void wino_conv_kernel(WinoArgs a) {
  constexpr int NTH = 64 * NW;
  constexpr int PP = CIN + 4;  // pixel pitch: 16-B units odd -> b128 patch reads conflict-free
  constexpr int C4 = CIN / 4;
  constexpr int LC4 = C4 == 4 ? 2 : 3;
  constexpr int NB = CIN / 16;
  constexpr int NS = COUT / (16 * NH);
  constexpr int NG = RT / 16;
  constexpr int NTASK = NG * NS;
  constexpr int USTR = NB * 4 * COUT * 4;  // floats per xi in U_s
  static_assert(CIN % 16 == 0 && COUT % (16 * NH) == 0 && RT % 16 == 0, "shape");
  static_assert(C4 == 4 || C4 == 8, "CIN");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* U_s = smem;                   // [16 xi][NB][4 g][COUT][4]
  float* x_s = smem + 16 * CIN * COUT;  // [rows][Wl][PP]

  // ---- weight transform U = G g G^T into LDS (once per workgroup)
  for (int e = threadIdx.x; e < CIN * COUT; e += NTH) {
    const int co = e % COUT, ci = e / COUT;
    float gk[3][3];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        float v = 0.f;
        if (!a.flip) {
          if (ci < a.wcin && co < a.wcout)
            v = a.w[((ky * 3 + kx) * a.wcin + ci) * a.wcout + co];
        } else {
          // data gradient: correlation of dY with W flipped in (ky, kx) and
          // transposed in (ci, co): ci = dY channel, co = dX channel
          if (co < a.wcin && ci < a.wcout)
            v = a.w[(((2 - ky) * 3 + (2 - kx)) * a.wcin + co) * a.wcout + ci];
        }
        gk[ky][kx] = v;
      }
    float t[4][3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      t[0][kx] = gk[0][kx];
      t[1][kx] = 0.5f * ((gk[0][kx] + gk[1][kx]) + gk[2][kx]);
      t[2][kx] = 0.5f * ((gk[0][kx] - gk[1][kx]) + gk[2][kx]);
      t[3][kx] = gk[2][kx];
    }
    const int b = ci >> 4, gq = (ci >> 2) & 3, v = ci & 3;
#pragma unroll
    for (int ra = 0; ra < 4; ++ra) {
      const float u[4] = {t[ra][0], 0.5f * ((t[ra][0] + t[ra][1]) + t[ra][2]),
                          0.5f * ((t[ra][0] - t[ra][1]) + t[ra][2]), t[ra][2]};
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
        U_s[(4 * ra + rb) * USTR + ((b * 4 + gq) * COUT + co) * 4 + v] = u[rb];
    }
  }

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int Wl = 2 * a.TX + 2;
  const int rowstr = Wl * PP;

  int r = blockIdx.x;
  if (r >= a.nranges) return;  // uniform: the whole workgroup leaves

  // ---- register prefetch of a range's input rows.  Thread k-slot e of a
  // range always stages LDS element e = (row L, column, channel quad): the
  // column / quad part of its global offset is fixed per thread, and the
  // per-range (image, row) part comes from a small row table in LDS (built
  // by the first `rows` threads), so a staged element costs a handful of
  // VALU.  Every load is issued unconditionally (invalid elements read a
  // dummy address and are zeroed at commit, where the ReLU-on-load is
  // applied too): a branch or a use right after a load makes the compiler
  // wait for it, serialising the prefetch.
  int* tab_s = reinterpret_cast<int*>(x_s + a.maxrows * Wl * PP);  // [maxrows]
  static_assert(MAXC <= 32, "stager mask");
  int sl_L[MAXC], sl_x[MAXC];
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int e = threadIdx.x + k * NTH;
    const int ch = e & (C4 - 1), pix = e >> LC4;
    const int L = pix / Wl, col = pix - L * Wl;
    sl_L[k] = L < a.maxrows ? L : -1;
    // -1: column in the zero padding
    sl_x[k] = (col >= 1 && col <= a.W) ? (col - 1) * CIN + 4 * ch : -1;
  }
  auto build_tab = [&](int rr) {
    const RangeGeom gm = range_geom(a, rr, RT);
    const int L = threadIdx.x;
    if (L < a.maxrows) {
      int v = -1;
      if (L < gm.rows) {
        const int p = (L >= gm.off1) + (L >= gm.off2) + (L >= gm.off3);
        const int offp = p == 0 ? 0 : (p == 1 ? gm.off1 : (p == 2 ? gm.off2 : gm.off3));
        const int y = 2 * (p == 0 ? gm.tya0 : 0) - 1 + (L - offp);
        if (y >= 0 && y < a.H) v = ((gm.n0 + p) * a.H + y) * a.W * CIN;
      }
      tab_s[L] = v;
    }
  };
  f4 stg[MAXC];
  uint32_t stg_ok = 0;
  auto prefetch = [&]() {  // reads tab_s
    uint32_t ok = 0;
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int rb = sl_L[k] >= 0 ? tab_s[sl_L[k]] : -1;
      const bool in = rb >= 0 && sl_x[k] >= 0 && !(a.ablate & 2);
      stg[k] = *reinterpret_cast<const f4*>(a.src + (in ? rb + sl_x[k] : 0));
      ok |= static_cast<uint32_t>(in) << k;
    }
    stg_ok = ok;
  };
  build_tab(r);
  __syncthreads();
  prefetch();

  for (;;) {
    __syncthreads();  // U_s written / the previous range's patch reads done
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      if (sl_L[k] >= 0 && !(a.ablate & 4)) {
        const int e = threadIdx.x + k * NTH;
        f4 v = stg[k];
        const bool in = (stg_ok >> k) & 1u;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float x = in ? v[q] : 0.f;
          v[q] = a.relu_in ? fmaxf(x, 0.f) : x;
        }
        *reinterpret_cast<f4*>(x_s + (e >> LC4) * PP + 4 * (e & (C4 - 1))) = v;
      }
    }
    const int cur = r;
    r += gridDim.x;
    if (r < a.nranges) build_tab(r);
    __syncthreads();
    if (r < a.nranges) prefetch();  // in flight under the MFMAs below
    const RangeGeom gm = range_geom(a, cur, RT);

    for (int task = (a.ablate & 1) ? NTASK : wave; task < NTASK; task += NW) {
      const int grp = task % NG, sl = task / NG;
      if (gm.t0 + 16 * grp >= gm.t1) continue;  // empty group (batch tail)
      const int co0 = sl * 16 * NH;
      int t = gm.t0 + 16 * grp + c16;
      const bool valid = t < gm.t1;
      if (!valid) t = gm.t0;
      const int R = fdivi(t, a.rTX), tx = t - R * a.TX;
      const int n = fdivi(R, a.rTY), ty = R - n * a.TY;
      const int p = n - gm.n0;
      const int offp = p == 0 ? 0 : (p == 1 ? gm.off1 : (p == 2 ? gm.off2 : gm.off3));
      const int base = offp + 2 * (ty - (p == 0 ? gm.tya0 : 0));
      const float* xp = x_s + (base * Wl + 2 * tx) * PP + 4 * g;
      const float* up = U_s + (g * COUT + co0 + c16) * 4;

      f4 acc[NH][16];
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int xi = 0; xi < 16; ++xi) acc[h][xi] = f4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
      for (int b = 0; b < NB; ++b) {
        // the lane's 4x4 input patch, 4 channels, and V = B^T d B
        f4 d[16];
#pragma unroll
        for (int dy = 0; dy < 4; ++dy)
#pragma unroll
          for (int dx = 0; dx < 4; ++dx)
            d[4 * dy + dx] =
                *reinterpret_cast<const f4*>(xp + dy * rowstr + dx * PP + 16 * b);
        f4 s[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          s[q] = d[q] - d[8 + q];
          s[4 + q] = d[4 + q] + d[8 + q];
          s[8 + q] = d[8 + q] - d[4 + q];
          s[12 + q] = d[4 + q] - d[12 + q];
        }
        f4 V[16];
#pragma unroll
        for (int ra = 0; ra < 4; ++ra) {
          V[4 * ra + 0] = s[4 * ra + 0] - s[4 * ra + 2];
          V[4 * ra + 1] = s[4 * ra + 1] + s[4 * ra + 2];
          V[4 * ra + 2] = s[4 * ra + 2] - s[4 * ra + 1];
          V[4 * ra + 3] = s[4 * ra + 1] - s[4 * ra + 3];
        }
        // 16 xi x 4 k-steps x NH slices; two xi chains interleaved (the
        // 16x16x4 f32 MFMA's dependent latency is 40 cycles, issue 32)
        const float* ub = up + b * 4 * COUT * 4;
#pragma unroll
        for (int xp2 = 0; xp2 < 8; ++xp2) {
          f4 ua[NH][2];
#pragma unroll
          for (int h = 0; h < NH; ++h)
#pragma unroll
            for (int q = 0; q < 2; ++q)
              ua[h][q] = *reinterpret_cast<const f4*>(ub + (2 * xp2 + q) * USTR + 64 * h);
#pragma unroll
          for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int q = 0; q < 2; ++q)
#pragma unroll
              for (int h = 0; h < NH; ++h)
                acc[h][2 * xp2 + q] =
                    mfma4(ua[h][q][v], V[2 * xp2 + q][v], acc[h][2 * xp2 + q]);
        }
      }

      // ---- output transform Y = A^T M A and the fused epilogue
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const int co = co0 + 16 * h + 4 * g;
        f4 bv = {0.f, 0.f, 0.f, 0.f};
        if (a.bias != nullptr) bv = *reinterpret_cast<const f4*>(a.bias + co);
        f4 tt[4][2];
#pragma unroll
        for (int ra = 0; ra < 4; ++ra) {
          tt[ra][0] = (acc[h][4 * ra] + acc[h][4 * ra + 1]) + acc[h][4 * ra + 2];
          tt[ra][1] = (acc[h][4 * ra + 1] - acc[h][4 * ra + 2]) - acc[h][4 * ra + 3];
        }
        f4 Y[4];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          Y[c] = (tt[0][c] + tt[1][c]) + tt[2][c];
          Y[2 + c] = (tt[1][c] - tt[2][c]) - tt[3][c];
        }
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
          for (int dx = 0; dx < 2; ++dx) {
            const int oy = 2 * ty + dy, ox = 2 * tx + dx;
            if (!valid || oy >= a.H || ox >= a.W || (a.ablate & 8)) continue;
            const int64_t o = ((static_cast<int64_t>(n) * a.H + oy) * a.W + ox) * COUT + co;
            f4 v = Y[2 * dy + dx] + bv;
            if (a.mask != nullptr) {
              const f4 m = *reinterpret_cast<const f4*>(a.mask + o);
#pragma unroll
              for (int k = 0; k < 4; ++k) v[k] = m[k] > 0.f ? v[k] : 0.f;
            }
            if (a.add != nullptr) v += *reinterpret_cast<const f4*>(a.add + o);
            if (a.relu_out) {
#pragma unroll
              for (int k = 0; k < 4; ++k) v[k] = fmaxf(v[k], 0.f);
            }
            *reinterpret_cast<f4*>(a.out + o) = v;
          }
      }
    }
    if (r >= a.nranges) break;
  }
}

template <typename Kern>
void allow_lds_w(Kern k, size_t bytes) {
  if (bytes > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             static_cast<int>(bytes));
    if (e != hipSuccess) (void)hipGetLastError();  // the launch reports it
  }
}

int env_int(const char* name, int def) {
  const char* e = std::getenv(name);
  return (e && *e) ? std::atoi(e) : def;
}

template <int CIN, int COUT, int NH, int NW, int RT, int MAXC, int WPS>
bool run_wino(const ConvArgs& c, bool flip, hipStream_t s) {
  const int H = c.Ho, W = c.Wo;
  const int TY = (H + 1) / 2, TX = (W + 1) / 2;
  const int64_t NT = static_cast<int64_t>(c.N) * TY * TX;
  if (NT >= (1 << 22) || TX > 1024 || TY > 1024) return false;
  const int per_img = TY * TX;
  const int maxparts = (RT - 1 + per_img - 1) / per_img + 1;
  if (maxparts > kMaxParts) return false;
  const int Wl = 2 * TX + 2;
  // staged rows <= 2 (tile rows spanned) + 2 (images touched)
  const int maxrows = 2 * ((RT - 1 + TX - 1) / TX + 1) + 2 * maxparts;
  if (static_cast<int64_t>(maxrows) * Wl * (CIN / 4) > static_cast<int64_t>(MAXC) * 64 * NW)
    return false;
  const size_t bytes = sizeof(float) * (16 * CIN * COUT +
                                        static_cast<size_t>(maxrows) * Wl * (CIN + 4) +
                                        maxrows);
  if (static_cast<int64_t>(c.N) * H * W * CIN >= (int64_t(1) << 31) || maxrows > 64 * NW)
    return false;
  if (bytes > 160 * 1024) return false;
  WinoArgs a{};
  a.src = static_cast<const float*>(c.src);
  a.w = c.w;
  a.bias = c.bias;
  a.mask = c.mask;
  a.add = c.add;
  a.out = c.out;
  a.N = c.N; a.H = H; a.W = W;
  a.TY = TY; a.TX = TX; a.NT = static_cast<int>(NT);
  a.nranges = static_cast<int>((NT + RT - 1) / RT);
  a.rTX = 1.f / static_cast<float>(TX);
  a.rTY = 1.f / static_cast<float>(TY);
  a.rWl = 1.f / static_cast<float>(Wl);
  a.wcin = c.wcin; a.wcout = c.wcout; a.flip = flip ? 1 : 0;
  a.relu_in = c.relu_in; a.relu_out = c.relu_out;
  a.maxrows = maxrows;
  static const int ablate = env_int("SA_WINO_ABLATE", 0);
  a.ablate = ablate;
  const int per_cu = std::max(1, std::min(WPS * 4 / NW, static_cast<int>((160 * 1024) / (bytes + 256))));
  static const int occ_env = env_int("SA_WINO_OCC", 0);
  const int occ = occ_env > 0 ? std::min(occ_env, per_cu) : per_cu;
  const int G = std::max(1, std::min(a.nranges, 256 * occ));
  auto kern = wino_conv_kernel<CIN, COUT, NH, NW, RT, MAXC, WPS>;
  allow_lds_w(kern, bytes);
  hipLaunchKernelGGL(kern, dim3(G), dim3(64 * NW), bytes, s, a);
  return true;
}

}  // namespace

bool wino_enabled() {
  static const bool on = env_int("SA_F32_WINO", 1) != 0;
  return on;
}

bool wino_conv_launch(const ConvArgs& c, bool flip, hipStream_t s) {
  // 3x3 / stride 1 / SAME, fp32 source, output = source dims, plain
  // placement (no phase / strided output, no pool-gradient source)
  if (c.D != 1 || c.pt != 1 || c.pl != 1 || c.Hs != c.Ho || c.Ws != c.Wo ||
      c.ostr > 0 || c.phase_c > 0 || c.pool.arg != nullptr)
    return false;
  const int cin = c.Cs, cout = c.Cout;
  // SA_WINO_CFG: alternative instances for measurement sweeps
  static const int cfg = env_int("SA_WINO_CFG", 0);
  if (cin == 16 && cout == 16) return run_wino<16, 16, 1, 4, 64, 10, 2>(c, flip, s);
  if (cin == 16 && cout == 32) {
    if (cfg == 1) return run_wino<16, 32, 2, 4, 64, 10, 1>(c, flip, s);
    return run_wino<16, 32, 1, 8, 64, 5, 2>(c, flip, s);
  }
  // 32 -> 16 (the stage-1 head's data gradient at 36x48): one workgroup of
  // four waves per CU (LDS) measured slower than the direct kernel
  // (674 vs 583 us), so it stays opt-in
  if (cin == 32 && cout == 16 && cfg == 2) return run_wino<32, 16, 1, 4, 64, 19, 1>(c, flip, s);
  if (cin == 32 && cout == 32) {
    if (cfg == 1) return run_wino<32, 32, 2, 4, 64, 15, 1>(c, flip, s);
    return run_wino<32, 32, 1, 8, 64, 8, 2>(c, flip, s);
  }
  return false;
}

}  // namespace cf32
}  // namespace sa
