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
#include "knobs.h"

#include <algorithm>
#include <cstdlib>

namespace sa {
namespace cf32 {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned gu32;

constexpr int kMaxParts = 4;  // images one range may touch

// Measurement knobs (SA_WINO_ABLATE / SA_FUSED_ABLATE: drop parts of a
// kernel's work to time the rest) exist only in builds with
// -DSA_MEASURE_KNOBS=1; in production builds every knob test folds to false,
// so no environment variable can remove a synchronisation or a store.
#ifndef SA_MEASURE_KNOBS
#define SA_MEASURE_KNOBS 0
#endif
__device__ __forceinline__ bool knob(int v, int bit) {
  return SA_MEASURE_KNOBS && (v & bit) != 0;
}

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Pricing builds only (-DSA_WINO_XMFMA=bits, never a production build): the
// MFMA at an odd (compile-time, unrolled) index becomes ONE VALU FMA on the
// same operands - half the matrix work, wrong results, everything else
// unchanged - to measure how much of a kernel the matrix pipe sets.  Bit 0:
// forward / data-gradient MFMAs, bit 1: weight-gradient MFMAs.
#ifndef SA_WINO_XMFMA
#define SA_WINO_XMFMA 0
#endif
template <int BIT>
__device__ __forceinline__ f4 mfma4x(float a, float b, f4 c, int idx) {
  if ((SA_WINO_XMFMA & BIT) && (idx & 1)) {
    c[0] = fmaf(a, b, c[0]);
    return c;
  }
  return mfma4(a, b, c);
}

// 16-B loads through a buffer descriptor: an offset at or past the buffer's
// end returns zeros (the hardware range check), so a stager's padding and
// out-of-image elements need no select when they are committed to LDS, and
// the per-lane address is a 32-bit byte offset.  Launchers refuse tensors
// of >= 4 GB.
constexpr uint32_t kOOB = 0xFFFFFFF0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const float* p, int64_t floats) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0,
                                           static_cast<int>(static_cast<uint32_t>(floats * 4)),
                                           0x00020000);
}
__device__ __forceinline__ f4 bload(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}
constexpr int64_t kMaxBufBytes = 0xFFFFFF00ll;

// Winograd transform add / subtract on float4 channel quads.  (A packed
// v_pk_add_f32 form was measured in round 4 and removed: the backend keeps
// <2 x float> arithmetic scalar, an inline-asm form read MFMA accumulators
// without the required wait states, and packed f32 beside MFMAs is an
// anti-lever on gfx950.)
__device__ __forceinline__ f4 tadd(f4 a, f4 b) { return a + b; }
__device__ __forceinline__ f4 tsub(f4 a, f4 b) { return a - b; }

// ReLU as one integer max on the bit pattern (negative floats, -0 and
// negative NaNs have the sign bit set: signed-int max with 0 gives +0);
// fmaxf(x, 0) is two instructions under IEEE mode (a canonicalising
// v_max_f32 x, x first)
__device__ __forceinline__ float relu0(float x) {
  return __int_as_float(max(__float_as_int(x), 0));
}

// Weight-gradient k-step: lane group g reads tile 4 st + kperm(g), order
// {0, 2, 1, 3}.  Adjacent tiles sit 2 pixels apart in LDS (8 banks for a
// 36-float pitch, 40 for 20), so the natural order put lane groups 0/1 (and
// 2/3), which one ds_read_b32 half-wave serves together, on overlapping
// banks; tiles 0 and 2 (1 and 3) are 16 banks apart at both pitches.  Which
// tile feeds which MFMA k slot does not change the sum over tiles.
__device__ __forceinline__ int kperm(int g) { return ((g & 1) << 1) | (g >> 1); }

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
               // loads, 4 no LDS commit, 8 no stores, 16 no weight transform
  int runs;    // 1: each workgroup walks a contiguous run of ranges (halo rows
               // shared with the previous range hit this CU's L2), 0: strided
  int prio;    // SA_WINO_PRIO=1: waves NW/2.. run at s_setprio 1 (static
               // priority for the second-dispatched half, MI355X_MICROARCH)
};

// Range walk of a persistent workgroup: a contiguous run [r, end) with step
// 1, or every gridDim.x-th range from blockIdx.x.
struct RangeWalk {
  int r, end, step;
};
__device__ __forceinline__ RangeWalk range_walk(int nranges, int runs) {
  RangeWalk w;
  if (runs) {
    w.r = static_cast<int>(static_cast<int64_t>(blockIdx.x) * nranges / gridDim.x);
    w.end = static_cast<int>((static_cast<int64_t>(blockIdx.x) + 1) * nranges / gridDim.x);
    w.step = 1;
  } else {
    w.r = blockIdx.x;
    w.end = nranges;
    w.step = gridDim.x;
  }
  return w;
}

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

// ---- tile-grid geometry: runtime or compile-time
// GH == 0: the map's H, W and the tile-grid divisors come from the kernel
// arguments (reciprocal index math, up to kMaxParts images per range, the
// row capacity `maxrows` an argument).  GH > 0: the map is GH x GW at
// compile time, so every divisor is a constant, the number of images a
// range can touch (MP) and the staged-row capacity fold to constants, the
// output-bounds tests of even maps vanish and offsets are 32-bit.  Both
// forms walk the same ranges in the same order with the same arithmetic
// (bitwise the same results, tests/test_conv_f32_gpu.py).
__host__ __device__ constexpr int wino_parts(int RT, int per_img) {
  return (RT - 1 + per_img - 1) / per_img + 1;
}
// LDS rows one range of RT tiles can need: 2 pixel rows per tile row it
// touches in each image part plus 2 halo rows per part.  Ranges start on
// tile-row boundaries when RT % TX == 0 (then they touch exactly RT / TX tile
// rows in total) and never straddle images when TY TX % RT == 0 (one part);
// otherwise a range may start mid-row (ceil((RT - 1) / TX) + 1 tile rows)
// and touch wino_parts images.  The host launchers and the compile-time
// geometry (TileGeo) both use this bound; the tight cases let the fused
// backward kernels stage the 72x128 frame's 36x64 / 18x32 maps in their
// register slots.
__host__ __device__ constexpr int wino_maxrows(int RT, int TX, int TY) {
  return 2 * (RT % TX == 0 ? RT / TX : (RT - 1 + TX - 1) / TX + 1) +
         2 * ((TY * TX) % RT == 0 ? 1 : wino_parts(RT, TY * TX));
}

// Staged-row pitch padding (compile-time geometry only).  A 16-tile patch
// read whose tiles wrap to the next tile row jumps by 2 Wl - 2 TX pixels
// instead of 0; at 5 (20-float pitch) or 9 (36-float pitch) 16-B units per
// pixel that jump lands the wrapped lanes on the 16-B bank groups of the
// unwrapped ones unless Wl - TX = 0 mod 8.  Padding each LDS row to that
// makes the wrap free: modelled b128 cycles per patch read 1.33 -> 1.00 at
// 36x48, 1.71 -> 1.03 at 42x42, 1.89 -> 1.11 at 18x24, 2.36 -> 1.12 at
// 21x21 (9x12 and 11x11 need no pad).  The stagers keep the unpadded
// element numbering; only the LDS address of a staged row moves.
// SA_WINO_LPAD bit 0: the forward kernel, 1: the fused 16-channel backward,
// 2: the fused32 backward (where its LDS budget allows).  Measured (in-step
// PMC, profiles/experiments.md round 5): the conflicts drop as modelled but
// the step time does not move, and the fused32 instances spill more with
// it, so only the forward (no spills either way) pads by default.
#ifndef SA_WINO_LPAD
#define SA_WINO_LPAD 1
#endif
constexpr bool wino_lpad_on(int bit) { return (SA_WINO_LPAD >> bit) & 1; }
__host__ __device__ constexpr int wino_lpad(int TX) {
  return (8 - (TX + 2) % 8) % 8;
}
// L * padc for a stager commit.  SA_WINO_LPAD_OPQ=1 recomputes it at every
// commit from an opaque copy of L (keeps the products out of the range
// loop's invariants; measured: more spills, not fewer)
#ifndef SA_WINO_LPAD_OPQ
#define SA_WINO_LPAD_OPQ 0
#endif
template <int PADC>
__device__ __forceinline__ int pad_pix(int L) {
  if constexpr (PADC == 0) {
    return 0;
  } else {
    if constexpr (SA_WINO_LPAD_OPQ) asm volatile("" : "+v"(L));
    return L * PADC;
  }
}
// LDS row pitch (pixels) of a kernel instance at tile-grid width TX
template <int GH, bool LP = true>
constexpr int wino_wl(int TX) {
  return 2 * TX + 2 + (GH > 0 && LP ? wino_lpad(TX) : 0);
}

template <int GH, int GW, int RT, bool LP = true>
struct TileGeo {
  static constexpr bool kCt = GH > 0;
  static constexpr int cTY = (GH + 1) / 2, cTX = (GW + 1) / 2;
  // images one range may touch
  static constexpr int MP = kCt ? wino_parts(RT, cTY * cTX) : kMaxParts;
  static constexpr int cMaxRows = kCt ? wino_maxrows(RT, cTX, cTY) : 0;
  // row padding (pixels): staged row L sits at LDS pixel L * WL, its
  // element e (unpadded numbering over WL0-pixel rows) at e + L * PADC
  static constexpr int PADC = kCt && LP ? wino_lpad(cTX) : 0;
  static_assert(MP <= kMaxParts, "range spans too many images");
  int H, W, TY, TX, NT, maxrows, WL0, WL;
  float rTX, rTY;
  __device__ __forceinline__ TileGeo(int H_, int W_, int TY_, int TX_, int NT_, float rTX_,
                                     float rTY_, int maxrows_)
      : H(kCt ? GH : H_), W(kCt ? GW : W_), TY(kCt ? cTY : TY_), TX(kCt ? cTX : TX_), NT(NT_),
        maxrows(kCt ? cMaxRows : maxrows_), WL0(2 * TX + 2), WL(2 * TX + 2 + PADC), rTX(rTX_),
        rTY(rTY_) {}
  // (t, R >= 0: unsigned constant division is a multiply-high and a shift)
  __device__ __forceinline__ int div_tx(int t) const {
    return kCt ? static_cast<int>(static_cast<unsigned>(t) / cTX) : fdivi(t, rTX);
  }
  __device__ __forceinline__ int div_ty(int R) const {
    return kCt ? static_cast<int>(static_cast<unsigned>(R) / cTY) : fdivi(R, rTY);
  }
  // output pixel (oy, ox) of a tile lies inside the map: always for even maps
  __device__ __forceinline__ bool in_y(int oy) const { return (kCt && GH % 2 == 0) || oy < H; }
  __device__ __forceinline__ bool in_x(int ox) const { return (kCt && GW % 2 == 0) || ox < W; }
  // image part of LDS row L / its first row
  __device__ __forceinline__ int part_of(const RangeGeom& g, int L) const {
    return (L >= g.off1) + (MP > 2 ? (L >= g.off2) : 0) + (MP > 3 ? (L >= g.off3) : 0);
  }
  __device__ __forceinline__ int part_off(const RangeGeom& g, int p) const {
    return p == 0 ? 0 : (p == 1 || MP <= 2 ? g.off1 : (p == 2 || MP <= 3 ? g.off2 : g.off3));
  }
  __device__ __forceinline__ RangeGeom range(int r) const {
    RangeGeom g;
    g.t0 = r * RT;
    g.t1 = min(g.t0 + RT, NT);
    const int R0 = div_tx(g.t0);
    const int R1 = div_tx(g.t1 - 1);
    g.n0 = div_ty(R0);
    const int n1 = div_ty(R1);
    g.tya0 = R0 - g.n0 * TY;
    int off[MP + 1];
    off[0] = 0;
#pragma unroll
    for (int p = 0; p < MP; ++p) {
      const int n = g.n0 + p;
      const int tya = p == 0 ? g.tya0 : 0;
      const int tyb = n == n1 ? R1 - n1 * TY : TY - 1;
      off[p + 1] = off[p] + (n <= n1 ? 2 * (tyb - tya) + 4 : 0);
    }
    g.off1 = off[1];
    g.off2 = MP > 2 ? off[2] : off[MP];
    g.off3 = MP > 3 ? off[3] : off[MP];
    g.rows = off[MP];
    return g;
  }
};

// FL: compile-time epilogue / stager flags (bit 0 ReLU on the input, 1 ReLU
// on the output, 2 mask, 3 residual add, 4 bias), or -1 = read them from
// the arguments (a runtime ReLU is a max + select per staged value)
template <int CIN, int COUT, int NH, int NW, int RT, int MAXC, int WPS, int FL = -1, int GH = 0,
          int GW = 0>
__global__ __launch_bounds__(64 * NW, WPS) void wino_conv_kernel(WinoArgs a) {
  constexpr int NTH = 64 * NW;
  const TileGeo<GH, GW, RT, wino_lpad_on(0)> G(a.H, a.W, a.TY, a.TX, a.NT, a.rTX, a.rTY,
                                                a.maxrows);
  const bool f_relu_in = FL < 0 ? a.relu_in != 0 : (FL & 1) != 0;
  const bool f_relu_out = FL < 0 ? a.relu_out != 0 : (FL & 2) != 0;
  const bool f_mask = FL < 0 ? a.mask != nullptr : (FL & 4) != 0;
  const bool f_add = FL < 0 ? a.add != nullptr : (FL & 8) != 0;
  const bool f_bias = FL < 0 ? a.bias != nullptr : (FL & 16) != 0;
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

  // ---- weight transform U = G g G^T into LDS (once per workgroup; the
  // measurement bit 16 skips it to time the rest)
  for (int e = threadIdx.x; e < (knob(a.ablate, 16) ? 0 : CIN * COUT); e += NTH) {
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
  const int Wl = G.WL;
  const int rowstr = Wl * PP;

  const RangeWalk rw = range_walk(a.nranges, a.runs);
  int r = rw.r;
  if (r >= rw.end) return;  // uniform: the whole workgroup leaves
  if (a.prio && __builtin_amdgcn_readfirstlane(wave) >= NW / 2) __builtin_amdgcn_s_setprio(1);

  // ---- register prefetch of a range's input rows.  Thread k-slot e of a
  // range always stages LDS element e = (row L, column, channel quad): the
  // column / quad part of its global offset is fixed per thread, and the
  // per-range (image, row) part comes from a small row table in LDS (built
  // by the first `rows` threads), so a staged element costs a handful of
  // VALU.  Every load is issued unconditionally (invalid elements read a
  // dummy address and are zeroed at commit, where the ReLU-on-load is
  // applied too): a branch or a use right after a load makes the compiler
  // wait for it, serialising the prefetch.
  int* tab_s = reinterpret_cast<int*>(x_s + G.maxrows * Wl * PP);  // [maxrows]
  static_assert(MAXC <= 32, "stager mask");
  int sl_L[MAXC], sl_x[MAXC];
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int e = threadIdx.x + k * NTH;
    const int ch = e & (C4 - 1), pix = e >> LC4;
    const int L = pix / G.WL0, col = pix - L * G.WL0;
    sl_L[k] = L < G.maxrows ? L : -1;
    // -1: column in the zero padding
    sl_x[k] = (col >= 1 && col <= G.W) ? (col - 1) * CIN + 4 * ch : -1;
  }
  auto build_tab = [&](int rr) {
    const RangeGeom gm = G.range(rr);
    const int L = threadIdx.x;
    if (L < G.maxrows) {
      int v = -1;
      if (L < gm.rows) {
        const int p = G.part_of(gm, L);
        const int offp = G.part_off(gm, p);
        const int y = 2 * (p == 0 ? gm.tya0 : 0) - 1 + (L - offp);
        if (y >= 0 && y < G.H) v = ((gm.n0 + p) * G.H + y) * G.W * CIN;
      }
      tab_s[L] = v;
    }
  };
  f4 stg[MAXC];
  const auto srcr = buf_rsrc(a.src, static_cast<int64_t>(a.N) * G.H * G.W * CIN);
  auto prefetch = [&]() __attribute__((always_inline)) {  // reads tab_s
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int rb = sl_L[k] >= 0 ? tab_s[sl_L[k]] : -1;
      const bool in = rb >= 0 && sl_x[k] >= 0 && !knob(a.ablate, 2);
      stg[k] = bload(srcr, in ? static_cast<uint32_t>(rb + sl_x[k]) * 4u : kOOB);
    }
  };
  build_tab(r);
  __syncthreads();
  prefetch();

  for (;;) {
    __syncthreads();  // U_s written / the previous range's patch reads done
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      if (sl_L[k] >= 0 && !knob(a.ablate, 4)) {
        const int e = threadIdx.x + k * NTH;
        f4 v = stg[k];  // zero where out of the image (range check)
        if (f_relu_in) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = relu0(v[q]);
        }
        *reinterpret_cast<f4*>(x_s + ((e >> LC4) + pad_pix<decltype(G)::PADC>(sl_L[k])) * PP + 4 * (e & (C4 - 1))) = v;
      }
    }
    const int cur = r;
    r += rw.step;
    // unconditional (the last range re-stages itself, unused): a
    // conditional prefetch leaves a join at the loop back-edge
    build_tab(r < rw.end ? r : cur);
    __syncthreads();
    prefetch();  // in flight under the MFMAs below
    const RangeGeom gm = G.range(cur);

    for (int task = knob(a.ablate, 1) ? NTASK : wave; task < NTASK; task += NW) {
      const int grp = task % NG, sl = task / NG;
      if (gm.t0 + 16 * grp >= gm.t1) continue;  // empty group (batch tail)
      const int co0 = sl * 16 * NH;
      int t = gm.t0 + 16 * grp + c16;
      const bool valid = t < gm.t1;
      if (!valid) t = gm.t0;
      const int R = G.div_tx(t), tx = t - R * G.TX;
      const int n = G.div_ty(R), ty = R - n * G.TY;
      const int p = n - gm.n0;
      const int offp = G.part_off(gm, p);
      const int base = offp + 2 * (ty - (p == 0 ? gm.tya0 : 0));
      const float* xp = x_s + (base * Wl + 2 * tx) * PP + 4 * g;
      const float* up = U_s + (g * COUT + co0 + c16) * 4;
      // epilogue operands (mask / residual) of the 4 outputs: global loads
      // issued before the MFMAs, so their latency hides under them - or,
      // at >= 3 waves per SIMD (register cap 168), after them (other waves
      // cover the latency)
      constexpr bool kLateEpi = WPS >= 3;
      f4 pm[NH][4], pa[NH][4];
      auto load_epi = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < NH; ++h)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int oy = 2 * ty + (q >> 1), ox = 2 * tx + (q & 1);
            const bool in = valid && G.in_y(oy) && G.in_x(ox);
            const int64_t o = in ? ((static_cast<int64_t>(n) * G.H + oy) * G.W + ox) * COUT +
                                       co0 + 16 * h + 4 * g
                                 : 0;
            pm[h][q] = (f_mask && in) ? *reinterpret_cast<const f4*>(a.mask + o)
                                      : f4{1.f, 1.f, 1.f, 1.f};
            pa[h][q] = (f_add && in) ? *reinterpret_cast<const f4*>(a.add + o)
                                     : f4{0.f, 0.f, 0.f, 0.f};
          }
      };
      if constexpr (!kLateEpi) load_epi();

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
          s[q] = tsub(d[q], d[8 + q]);
          s[4 + q] = tadd(d[4 + q], d[8 + q]);
          s[8 + q] = tsub(d[8 + q], d[4 + q]);
          s[12 + q] = tsub(d[4 + q], d[12 + q]);
        }
        f4 V[16];
#pragma unroll
        for (int ra = 0; ra < 4; ++ra) {
          V[4 * ra + 0] = tsub(s[4 * ra + 0], s[4 * ra + 2]);
          V[4 * ra + 1] = tadd(s[4 * ra + 1], s[4 * ra + 2]);
          V[4 * ra + 2] = tsub(s[4 * ra + 2], s[4 * ra + 1]);
          V[4 * ra + 3] = tsub(s[4 * ra + 1], s[4 * ra + 3]);
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
                    mfma4x<1>(ua[h][q][v], V[2 * xp2 + q][v], acc[h][2 * xp2 + q], v);
        }
      }

      // ---- output transform Y = A^T M A and the fused epilogue
      if constexpr (kLateEpi) load_epi();
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const int co = co0 + 16 * h + 4 * g;
        f4 bv = {0.f, 0.f, 0.f, 0.f};
        if (f_bias) bv = *reinterpret_cast<const f4*>(a.bias + co);
        f4 tt[4][2];
#pragma unroll
        for (int ra = 0; ra < 4; ++ra) {
          tt[ra][0] = tadd(tadd(acc[h][4 * ra], acc[h][4 * ra + 1]), acc[h][4 * ra + 2]);
          tt[ra][1] = tsub(tsub(acc[h][4 * ra + 1], acc[h][4 * ra + 2]), acc[h][4 * ra + 3]);
        }
        f4 Y[4];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          Y[c] = tadd(tadd(tt[0][c], tt[1][c]), tt[2][c]);
          Y[2 + c] = tsub(tsub(tt[1][c], tt[2][c]), tt[3][c]);
        }
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
          for (int dx = 0; dx < 2; ++dx) {
            const int oy = 2 * ty + dy, ox = 2 * tx + dx;
            if (!valid || !G.in_y(oy) || !G.in_x(ox) || knob(a.ablate, 8)) continue;
            const int64_t o = ((static_cast<int64_t>(n) * G.H + oy) * G.W + ox) * COUT + co;
            f4 v = Y[2 * dy + dx] + bv;
            const f4 m = pm[h][2 * dy + dx];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = m[k] > 0.f ? v[k] : 0.f;
            v += pa[h][2 * dy + dx];
            if (f_relu_out) {
#pragma unroll
              for (int k = 0; k < 4; ++k) v[k] = relu0(v[k]);
            }
            *reinterpret_cast<f4*>(a.out + o) = v;
          }
      }
    }
    if (r >= rw.end) break;
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


int g_wino_fault = 0;  // conv_wino_fault(): tests of the fail-loud hand-off

template <int CIN, int COUT, int NH, int NW, int RT, int MAXC, int WPS, int FL = -1, int GH = 0,
          int GW = 0>
bool run_wino_g(const ConvArgs& c, bool flip, hipStream_t s) {
  const int H = c.Ho, W = c.Wo;
  if (GH > 0 && (H != GH || W != GW)) return false;
  const int TY = (H + 1) / 2, TX = (W + 1) / 2;
  const int64_t NT = static_cast<int64_t>(c.N) * TY * TX;
  if (NT >= (1 << 22) || TX > 1024 || TY > 1024) return false;
  const int per_img = TY * TX;
  const int maxparts = (RT - 1 + per_img - 1) / per_img + 1;
  if (maxparts > kMaxParts) return false;
  const int Wl = 2 * TX + 2, WlP = wino_wl<GH, wino_lpad_on(0)>(TX);
  // staged rows <= 2 (tile rows spanned) + 2 (images touched); exactly
  // 2 RT / TX + 2 when every range is whole tile rows of one image
  const int maxrows = wino_maxrows(RT, TX, TY);
  if (static_cast<int64_t>(maxrows) * Wl * (CIN / 4) > static_cast<int64_t>(MAXC) * 64 * NW)
    return false;
  const size_t bytes = sizeof(float) * (16 * CIN * COUT +
                                        static_cast<size_t>(maxrows) * WlP * (CIN + 4) +
                                        maxrows);
  if (static_cast<int64_t>(c.N) * H * W * CIN * 4 > kMaxBufBytes || maxrows > 64 * NW)
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
  static const int ablate = measure_knob("SA_WINO_ABLATE", 0);
  a.ablate = ablate;
  static const int runs = measure_knob("SA_WINO_RUNS", 1);
  a.runs = runs;
  static const int prio = measure_knob("SA_WINO_PRIO", 0);
  a.prio = prio;
  const int per_cu = std::max(1, std::min(WPS * 4 / NW, static_cast<int>((160 * 1024) / (bytes + 256))));
  static const int occ_env = measure_knob("SA_WINO_OCC", 0);
  const int occ = occ_env > 0 ? std::min(occ_env, per_cu) : per_cu;
  const int G = std::max(1, std::min(a.nranges, conv_cus() * occ));
  auto kern = wino_conv_kernel<CIN, COUT, NH, NW, RT, MAXC, WPS, FL, GH, GW>;
  allow_lds_w(kern, bytes);
  hipLaunchKernelGGL(kern, dim3(G), dim3(64 * NW), bytes, s, a);
  return true;
}

// Compile-time-geometry switch of the fp32 Winograd kernels (TileGeo):
// SA_WINO_GEO=0 keeps every map on the runtime-geometry instances.
int g_wino_geo = -1;  // -1: not read yet; conv_wino_geo() sets it (tests)
bool wino_geo_enabled() {
  if (g_wino_geo < 0) g_wino_geo = env_knob("SA_WINO_GEO", 1) != 0 ? 1 : 0;
  return g_wino_geo != 0;
}
// per kernel family (SA_WINO_GEO_MASK, sweeps): bit 0 the forward, bit 1 the
// 16-channel fused backward, bit 2 the fused32 backward
bool wino_geo_family(int bit) {
  static const int mask = measure_knob("SA_WINO_GEO_MASK", 7);
  return wino_geo_enabled() && (mask & bit) != 0;
}

// The deep torso's maps get compile-time instances (only where that layer
// runs): the IMPALA / DMLab 72x96 ladder (36x48, 18x24, 9x12), the Atari
// 84x84 ladder (42x42, 21x21, 11x11) and the 72x128 Doom ladder (36x64,
// 18x32, 9x16); any other map runs the runtime-geometry kernel.  Per channel
// configuration: 16 -> 16 (res16) and 16 -> 32 (stage-1 head) at 36x48 /
// 42x42 / 36x64, 32 -> 32 (res32, stage-2 head) at 18x24, 9x12, 21x21,
// 11x11, 18x32, 9x16.
#define SA_GEO(h, w) \
  if (HH == (h) && WW == (w) && SA_CALL(h, w)) return true;
#define SA_WINO_GEO_DISPATCH(CI, CO, FAM)                                      \
  if (wino_geo_family(FAM)) {                                                  \
    if constexpr ((CI) == 16) { SA_GEO(36, 48) SA_GEO(42, 42) SA_GEO(36, 64) } \
    if constexpr ((CI) == 32 && (CO) == 32) {                                  \
      SA_GEO(18, 24) SA_GEO(9, 12) SA_GEO(21, 21) SA_GEO(11, 11)               \
      SA_GEO(18, 32) SA_GEO(9, 16)                                             \
    }                                                                          \
  }

// runtime geometry only (the opt-in experiment variants)
template <int CIN, int COUT, int NH, int NW, int RT, int MAXC, int WPS, int FL = -1>
bool run_wino(const ConvArgs& c, bool flip, hipStream_t s) {
  return run_wino_g<CIN, COUT, NH, NW, RT, MAXC, WPS, FL>(c, flip, s);
}

// compile-time geometry where the map has an instance, else runtime
template <int CIN, int COUT, int NH, int NW, int RT, int MAXC, int WPS>
bool run_wino_ct(const ConvArgs& c, bool flip, hipStream_t s) {
  const int HH = c.Ho, WW = c.Wo;
#define SA_CALL(h, w) run_wino_g<CIN, COUT, NH, NW, RT, MAXC, WPS, -1, h, w>(c, flip, s)
  SA_WINO_GEO_DISPATCH(CIN, COUT, 1)
#undef SA_CALL
  return run_wino_g<CIN, COUT, NH, NW, RT, MAXC, WPS>(c, flip, s);
}

// The deep torso's forward flag sets get compile-time instances: residual
// conv 1 (ReLU in + out, bias) = 19, conv 2 (skip add, bias [, ReLU out for
// the torso's last]) = 24 / 26, stage head (bias) = 16; anything else the
// runtime-flag instance
template <int CIN, int COUT, int NH, int NW, int RT, int MAXC, int WPS>
bool run_wino_fl(const ConvArgs& c, bool flip, hipStream_t s) {
  const int fl = (c.relu_in ? 1 : 0) | (c.relu_out ? 2 : 0) | (c.mask ? 4 : 0) |
                 (c.add ? 8 : 0) | (c.bias ? 16 : 0);
  // SA_WINO_FL: 1 = every instance (measured 10.85 vs 10.77 ms/step with
  // none: the 32-channel instances spilled), 2 = the 16-channel-input
  // instances only (no spill risk at 112 VGPRs), 0 = none
  // 3 (default): the compile-time-geometry 16 -> 16 instances with the two
  // residual flag sets compile-time too (conv 1 = 19, conv 2 = 24): full
  // fp32 step 9.546 / 9.547 -> 9.502 / 9.460 ms (geometry alone; one box)
  // 4 (default) adds the 32 -> 32 residual convs at 18x24: 9.474 / 9.449 /
  // 9.446 (3) -> 9.466 / 9.434 / 9.429 ms
  static const int on = measure_knob("SA_WINO_FL", 4);
  if constexpr (CIN == 16 && COUT == 16) {
    if (on >= 3 && !flip && wino_geo_enabled()) {
      const int HH = c.Ho, WW = c.Wo;
#define SA_CALL(h, w) run_wino_g<CIN, COUT, NH, NW, RT, MAXC, WPS, 19, h, w>(c, flip, s)
      if (fl == 19) { SA_GEO(36, 48) SA_GEO(42, 42) SA_GEO(36, 64) }
#undef SA_CALL
#define SA_CALL(h, w) run_wino_g<CIN, COUT, NH, NW, RT, MAXC, WPS, 24, h, w>(c, flip, s)
      if (fl == 24) { SA_GEO(36, 48) SA_GEO(42, 42) SA_GEO(36, 64) }
#undef SA_CALL
    }
  }
  // 4: also the 32 -> 32 residual convs at 18x24 (188 / 210 VGPRs, no
  // spills in the geometry instances)
  if constexpr (CIN == 32 && COUT == 32) {
    if (on >= 4 && !flip && wino_geo_enabled()) {
      const int HH = c.Ho, WW = c.Wo;
#define SA_CALL(h, w) run_wino_g<CIN, COUT, NH, NW, RT, MAXC, WPS, 19, h, w>(c, flip, s)
      // (the 19 instances of the odd maps spill 4-6 VGPRs: runtime flags there)
      if (fl == 19) { SA_GEO(18, 24) SA_GEO(18, 32) }
#undef SA_CALL
#define SA_CALL(h, w) run_wino_g<CIN, COUT, NH, NW, RT, MAXC, WPS, 24, h, w>(c, flip, s)
      if (fl == 24) {
        SA_GEO(18, 24) SA_GEO(9, 12) SA_GEO(21, 21) SA_GEO(11, 11) SA_GEO(18, 32) SA_GEO(9, 16)
      }
#undef SA_CALL
    }
  }
  if ((on == 1 || (on == 2 && CIN == 16)) && !flip) {
    if (fl == 19) return run_wino<CIN, COUT, NH, NW, RT, MAXC, WPS, 19>(c, flip, s);
    if (fl == 24) return run_wino<CIN, COUT, NH, NW, RT, MAXC, WPS, 24>(c, flip, s);
    if (fl == 26) return run_wino<CIN, COUT, NH, NW, RT, MAXC, WPS, 26>(c, flip, s);
    if (fl == 16) return run_wino<CIN, COUT, NH, NW, RT, MAXC, WPS, 16>(c, flip, s);
  }
  return run_wino_ct<CIN, COUT, NH, NW, RT, MAXC, WPS>(c, flip, s);
}

// ------------------------------------------------------- fused stage heads
// Deep-torso stage head (3x3/1 SAME conv + bias) with the following 3x3/2
// SAME max-pool and its argmax fused into the epilogue (reference
// experiment.py:160-163: conv -> max_pool), so the pre-pool map exists only
// in LDS: stage 0 (4-channel fp32 image -> 16, 72x96) and stage 1 (16 -> 32,
// 36x48).  Needs H % 4 == 0 and a pooled pad-before of 0 (even H, W).  Each
// range is the tile-row pair (2k, 2k+1) of one image (RT = W tiles: pixel
// rows 4k..4k+3), one 16-tile x 16-channel task per wave.  The epilogue writes
// Y + b into an LDS image of those 4 rows (aliasing the staged input rows,
// which every wave has finished reading); the pool phase (thread = pooled
// column x channel quad; one half of the workgroup per pooled row) then
// stores pooled row 2k (pixel rows 4k..4k+2) and keeps the rows-(4k+2, 4k+3)
// part of pooled row 2k+1 in registers until the next range - the same
// workgroup's, since each walks a contiguous run - adds pixel row 4k+4.  A
// run's first range (k > 0) leaves its top-row part in `side`, the run's last
// carry is stored as is, and wino_pool_fix_kernel merges those pairs
// afterwards.  Values and argmax codes are bitwise those of the Winograd conv
// + maxpool_fwd_kernel pair (strict >, taps in row-major window order: the
// first maximal tap wins).
//
// CIN == 4 (stage 0: RGB + a zero channel): the MFMA's k = 4 input channels
// are the lane groups g, so a lane transforms ONE channel of its tile's 4x4
// patch (scalar B^T d B) and each xi is one MFMA; CIN == 16 as
// wino_conv_kernel (4 channels per lane, 4 k-steps per xi).
struct WinoPoolArgs {
  WinoArgs c;
  float* pooled;     // [N, H/2, W/2, COUT]
  uint8_t* arg;      // [N, H/2, W/2, COUT] tap codes dy * 3 + dx
  f4* side_v;        // [G][W/2 * COUT/4] top-row parts of the run-start ranges
  uint32_t* side_c;  // [G][W/2 * COUT/4] their codes (4 x 8 bits)
};

template <int CIN_, int COUT_, int RT>
struct PoolGeo {
  static constexpr int CIN = CIN_, COUT = COUT_;
  static constexpr int W = RT;                      // one tile-row pair = RT tiles
  // 16-tile groups: the last one partly past the range when RT % 16 != 0
  // (the 84-wide Atari frame: 84 tiles in 6 groups, 12 lanes idle)
  static constexpr int NG = (RT + 15) / 16;
  static constexpr int NW = NG * (COUT / 16);       // one task per wave
  static constexpr int PP = CIN == 4 ? 4 : CIN + 4;  // staged pixel pitch (floats)
  static constexpr int IPP = COUT + 4;               // pre-pool image pixel pitch
  static constexpr int ROWS = 6;                     // staged input rows per range
  static constexpr int XREG = (ROWS * (W + 2) * PP > 4 * W * IPP) ? ROWS * (W + 2) * PP
                                                                   : 4 * W * IPP;
  static constexpr int MAXC = (ROWS * (W + 2) * (CIN / 4) + 64 * NW - 1) / (64 * NW);
  // pool-phase threads (two pooled rows x WP columns x CQ quads) and whether
  // each pooled row is whole waves (the conflict-free lane map needs it)
  static constexpr int PTH = (W / 2) * (COUT / 4);
  static constexpr bool kWaveRows = PTH % 64 == 0;
  static constexpr int WP = W / 2;                   // pooled width
  static constexpr int CQ = COUT / 4;                // channel quads
  static constexpr size_t bytes = sizeof(float) * (16 * CIN * COUT + XREG + ROWS);
};

__device__ __forceinline__ void pool_take(f4& best, int (&code)[4], const f4 v, int c) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (v[q] > best[q]) {  // strict: the first maximal tap wins
      best[q] = v[q];
      code[q] = c;
    }
}
__device__ __forceinline__ uint32_t pack_codes(const int (&code)[4]) {
  return static_cast<uint32_t>(code[0]) | (static_cast<uint32_t>(code[1]) << 8) |
         (static_cast<uint32_t>(code[2]) << 16) | (static_cast<uint32_t>(code[3]) << 24);
}

// Pool-phase lane -> (pooled column, channel quad) map of one wave (64 / CQ
// columns x CQ quads): every 16-lane group of a ds_read_b128 (gfx950 lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59},
// {36-43,48-51,60-63}) reads 16 distinct 16-B bank segments of the pre-pool
// image (pixel pitch IPP floats, pooled column pj -> pixel 2 pj): each
// segment s = (pj IPP / 2 + pq) mod 16 is taken by exactly one (pj, pq) per
// group.  The natural map (pq = lane % CQ) put 2-4 lanes of a group on one
// segment.
__host__ __device__ constexpr int b128_group(int l) {
  const int h = l & 31;
  const int g = (h < 4 || (h >= 12 && h < 16) || (h >= 20 && h < 28)) ? 0 : 1;
  return g + 2 * (l >> 5);
}
template <int CQ, int IPP>
struct PoolLaneMap {
  unsigned char pj[64] = {}, pq[64] = {};
  constexpr PoolLaneMap() {
    constexpr int NP = 64 / CQ;
    bool used[64] = {};
    for (int g = 0; g < 4; ++g) {
      int next = 0;  // next lane of group g to assign
      for (int seg = 0; seg < 16; ++seg) {
        int pick = -1;
        for (int c = 0; c < NP && pick < 0; ++c)
          for (int q = 0; q < CQ && pick < 0; ++q)
            if (!used[c * CQ + q] && (c * (IPP / 2) + q) % 16 == seg) pick = c * CQ + q;
        while (b128_group(next) != g) ++next;
        used[pick] = true;
        pj[next] = static_cast<unsigned char>(pick / CQ);
        pq[next] = static_cast<unsigned char>(pick % CQ);
        ++next;
      }
    }
  }
};
template <int CQ, int IPP>
constexpr bool pool_lane_map_ok() {
  constexpr PoolLaneMap<CQ, IPP> m{};
  bool seen[64] = {};
  for (int l = 0; l < 64; ++l) {
    const int id = m.pj[l] * CQ + m.pq[l];
    if (m.pj[l] >= 64 / CQ || seen[id]) return false;
    seen[id] = true;
  }
  return true;
}
static_assert(pool_lane_map_ok<8, 36>() && pool_lane_map_ok<4, 20>(), "pool lane map");

// OT: the map may have an odd number of tile rows (H % 4 == 2: the image's
// last range is one tile row); compiled only where such a map runs
template <int CIN, int COUT, int RT, bool OT = false>
__global__ __launch_bounds__((64 * PoolGeo<CIN, COUT, RT>::NW), 3) void wino_conv_pool_kernel(
    WinoPoolArgs pa) {
  using P = PoolGeo<CIN, COUT, RT>;
  constexpr int W = P::W, NW = P::NW, NTH = 64 * NW;
  constexpr int PP = P::PP, IPP = P::IPP, MAXC = P::MAXC, WP = P::WP, CQ = P::CQ;
  constexpr int C4 = CIN / 4, LC4 = C4 == 4 ? 2 : 0;
  constexpr int NG = P::NG;
  constexpr int Wl = W + 2, rowstr = Wl * PP;
  // CIN == 4 (stage 0): the staged rows are channel planes [4][ROWS][Wl] with
  // an odd plane stride, so a lane's scalar patch reads (16 tiles x 2 pixels
  // apart, channel g) hit 32 distinct banks; the interleaved [pixel][4]
  // layout put the 16 tiles of a half-wave on 4 banks (PMC: 5.0 bank-
  // conflict cycles per LDS instruction)
  constexpr int PS = (P::ROWS * Wl) | 1;
  static_assert(CIN != 4 || 4 * PS <= P::XREG, "planes fit the staging region");
  static_assert(CIN == 4 || CIN == 16, "CIN");
  static_assert(NW * 64 >= 2 * WP * CQ, "two pooled rows x WP columns x CQ quads fit the workgroup");
  static_assert(RT % 2 == 0 && MAXC <= 32, "shape");
  const WinoArgs& a = pa.c;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // U: CIN 16 [16 xi][4 g][COUT][4 v] (f4 A fragments), CIN 4 [16 xi][4 ci][COUT]
  float* U_s = smem;
  float* x_s = smem + 16 * CIN * COUT;  // staged rows [6][Wl][PP], then the image [4][W][IPP]
  float* img = x_s;
  int* tab_s = reinterpret_cast<int*>(x_s + P::XREG);  // [6]

  // U = G g G^T (forward weights HWIO [3][3][CIN][COUT])
  for (int e = threadIdx.x; e < CIN * COUT; e += NTH) {
    const int co = e % COUT, ci = e / COUT;
    float gk[3][3];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) gk[ky][kx] = a.w[((ky * 3 + kx) * CIN + ci) * COUT + co];
    float t[4][3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      t[0][kx] = gk[0][kx];
      t[1][kx] = 0.5f * ((gk[0][kx] + gk[1][kx]) + gk[2][kx]);
      t[2][kx] = 0.5f * ((gk[0][kx] - gk[1][kx]) + gk[2][kx]);
      t[3][kx] = gk[2][kx];
    }
#pragma unroll
    for (int ra = 0; ra < 4; ++ra) {
      const float u[4] = {t[ra][0], 0.5f * ((t[ra][0] + t[ra][1]) + t[ra][2]),
                          0.5f * ((t[ra][0] - t[ra][1]) + t[ra][2]), t[ra][2]};
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const int xi = 4 * ra + rb;
        if constexpr (CIN == 16)
          U_s[xi * (16 * COUT) + (((ci >> 2) & 3) * COUT + co) * 4 + (ci & 3)] = u[rb];
        else
          U_s[(xi * 4 + ci) * COUT + co] = u[rb];
      }
    }
  }

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const RangeWalk rw = range_walk(a.nranges, 1);
  int r = rw.r;
  if (r >= rw.end) return;  // uniform
  const int rfirst = r;
  // ranges (tile-row pairs) per image; an odd tile-row count (H % 4 == 2,
  // the 42-row Atari stage-1 map) leaves a last range of one tile row
  const int KP = OT ? (a.TY + 1) / 2 : a.TY / 2;
  const int Hp = a.H / 2;

  // staging: the generic kernel's register prefetch (row table in LDS)
  int sl_L[MAXC], sl_x[MAXC];
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int e = threadIdx.x + k * NTH;
    const int ch = e & (C4 - 1), pix = e >> LC4;
    const int L = pix / Wl, col = pix - L * Wl;
    sl_L[k] = L < P::ROWS ? L : -1;
    sl_x[k] = (col >= 1 && col <= W) ? (col - 1) * CIN + 4 * ch : -1;
  }
  auto build_tab = [&](int rr) {
    const int n = rr / KP, k = rr - n * KP;
    const int L = threadIdx.x;
    if (L < P::ROWS) {
      const int y = 4 * k - 1 + L;
      tab_s[L] = (y >= 0 && y < a.H) ? ((n * a.H + y) * W) * CIN : -1;
    }
  };
  f4 stg[MAXC];
  const auto srcr = buf_rsrc(a.src, static_cast<int64_t>(a.N) * a.H * W * CIN);
  auto prefetch = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int rb = sl_L[k] >= 0 ? tab_s[sl_L[k]] : -1;
      const bool in = rb >= 0 && sl_x[k] >= 0;
      stg[k] = bload(srcr, in ? static_cast<uint32_t>(rb + sl_x[k]) * 4u : kOOB);
    }
  };
  build_tab(r);
  __syncthreads();
  prefetch();

  // pool-phase thread: pooled column pj, channel quad pq; the first WP * CQ
  // threads own pooled row 2k (9 taps), the rest the odd row 2k+1 (its
  // carried part + 3 taps of the next range, then 6 taps): balanced
  // (rows of whole waves take the conflict-free lane map, other widths the
  // natural quad-fastest numbering; threads past the two rows idle)
  const int pt = threadIdx.x % (WP * CQ);
  constexpr PoolLaneMap<CQ, IPP> kMap{};
  const int pj = P::kWaveRows ? (pt >> 6) * (64 / CQ) + kMap.pj[pt & 63] : pt / CQ;
  const int pq = P::kWaveRows ? kMap.pq[pt & 63] : pt % CQ;
  const bool even_row = threadIdx.x < WP * CQ;
  const bool pool_thread = NW * 64 == 2 * WP * CQ || threadIdx.x < 2 * WP * CQ;
  constexpr float kNegInf = -__builtin_inff();
  f4 cv = {kNegInf, kNegInf, kNegInf, kNegInf};
  int cc[4] = {0, 0, 0, 0};
  bool cvalid = false;
  int64_t cdst = 0;  // pooled element offset of the carried window

  // this wave's task: 16-tile group grp, 16-channel slice sl
  const int grp = wave % NG, sl = wave / NG;
  const int co0 = sl * 16;
  // tile within the range = (row txl / (W/2), column); lanes past the range
  // (RT % 16 != 0) compute tile 0 again and store nothing; tiles of a
  // missing second tile row (odd TY) store -inf (pool padding)
  const bool tvalid = RT % 16 == 0 || 16 * grp + c16 < RT;
  const int txl = tvalid ? 16 * grp + c16 : 0;
  const int tyl = txl / (W / 2), tx = txl - tyl * (W / 2);
  // CIN 16: 4 channels 4g.. of each patch pixel; CIN 4: channel g
  const float* xp = CIN == 16 ? x_s + (2 * tyl * Wl + 2 * tx) * PP + 4 * g
                              : x_s + g * PS + 2 * tyl * Wl + 2 * tx;
  const float* up = CIN == 16 ? U_s + (g * COUT + co0 + c16) * 4 : U_s + g * COUT + co0 + c16;
  const f4 bv = *reinterpret_cast<const f4*>(a.bias + co0 + 4 * g);

  for (;;) {
    __syncthreads();  // U_s written / the previous range's pool reads are done
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      if (sl_L[k] >= 0) {
        const int e = threadIdx.x + k * NTH;
        if constexpr (CIN == 16) {
          *reinterpret_cast<f4*>(x_s + (e >> LC4) * PP + 4 * (e & (C4 - 1))) = stg[k];
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) x_s[q * PS + e] = stg[k][q];
        }
      }
    }
    const int cur = r;
    ++r;
    build_tab(r < rw.end ? r : cur);  // unconditional: see wino_conv_kernel
    __syncthreads();
    prefetch();  // in flight under the MFMAs below

    f4 acc[16];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) acc[xi] = f4{0.f, 0.f, 0.f, 0.f};
    if (!knob(a.ablate, 1)) {
      if constexpr (CIN == 16) {
        constexpr int USTR = 16 * COUT;  // floats per xi
        f4 d[16];
#pragma unroll
        for (int dy = 0; dy < 4; ++dy)
#pragma unroll
          for (int dx = 0; dx < 4; ++dx)
            d[4 * dy + dx] = *reinterpret_cast<const f4*>(xp + dy * rowstr + dx * PP);
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
#pragma unroll
        for (int xp2 = 0; xp2 < 8; ++xp2) {
          f4 ua[2];
#pragma unroll
          for (int q = 0; q < 2; ++q)
            ua[q] = *reinterpret_cast<const f4*>(up + (2 * xp2 + q) * USTR);
#pragma unroll
          for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int q = 0; q < 2; ++q)
              acc[2 * xp2 + q] = mfma4(ua[q][v], V[2 * xp2 + q][v], acc[2 * xp2 + q]);
        }
      } else {
        float d[16];
#pragma unroll
        for (int dy = 0; dy < 4; ++dy)
#pragma unroll
          for (int dx = 0; dx < 4; ++dx) d[4 * dy + dx] = xp[dy * Wl + dx];
        float s[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          s[q] = d[q] - d[8 + q];
          s[4 + q] = d[4 + q] + d[8 + q];
          s[8 + q] = d[8 + q] - d[4 + q];
          s[12 + q] = d[4 + q] - d[12 + q];
        }
        float V[16];
#pragma unroll
        for (int ra = 0; ra < 4; ++ra) {
          V[4 * ra + 0] = s[4 * ra + 0] - s[4 * ra + 2];
          V[4 * ra + 1] = s[4 * ra + 1] + s[4 * ra + 2];
          V[4 * ra + 2] = s[4 * ra + 2] - s[4 * ra + 1];
          V[4 * ra + 3] = s[4 * ra + 1] - s[4 * ra + 3];
        }
        float ua[16];
#pragma unroll
        for (int xi = 0; xi < 16; ++xi) ua[xi] = up[xi * 4 * COUT];
#pragma unroll
        for (int xi = 0; xi < 16; ++xi) acc[xi] = mfma4(ua[xi], V[xi], acc[xi]);
      }
    }
    __syncthreads();  // every wave's patch reads are done: x_s becomes the image

    // output transform Y = A^T M A + b into the pre-pool image
    {
      const int kk = cur - (cur / KP) * KP;  // this range's tile-row pair
      const bool row_ok = !OT || 2 * kk + tyl < a.TY;
      f4 tt[4][2];
#pragma unroll
      for (int ra = 0; ra < 4; ++ra) {
        tt[ra][0] = (acc[4 * ra] + acc[4 * ra + 1]) + acc[4 * ra + 2];
        tt[ra][1] = (acc[4 * ra + 1] - acc[4 * ra + 2]) - acc[4 * ra + 3];
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
        for (int dx = 0; dx < 2; ++dx)
          if (tvalid && !knob(a.ablate, 32))
            *reinterpret_cast<f4*>(img + ((2 * tyl + dy) * W + 2 * tx + dx) * IPP + co0 + 4 * g) =
                row_ok ? Y[2 * dy + dx] + bv : f4{kNegInf, kNegInf, kNegInf, kNegInf};
    }
    __syncthreads();

    // pool phase
    if (pool_thread && !knob(a.ablate, 16)) {
      const int n = cur / KP, k = cur - n * KP;
      auto tap = [&](int row, int dx) -> f4 {
        return *reinterpret_cast<const f4*>(img + (row * W + 2 * pj + dx) * IPP + 4 * pq);
      };
      const bool edge = 2 * pj + 2 >= W;  // the window's third column is padding
      const int64_t orow = static_cast<int64_t>(n) * Hp;
      // (a) pooled row 2k-1: the carried rows (4k-2, 4k-1) + pixel row 4k
      if (!even_row && (cvalid || (cur == rfirst && k > 0))) {
        f4 best = cv;
        int code[4] = {cc[0], cc[1], cc[2], cc[3]};
        if (!cvalid) {
          best = f4{kNegInf, kNegInf, kNegInf, kNegInf};
          code[0] = code[1] = code[2] = code[3] = 0;
        }
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
          if (dx < 2 || !edge) pool_take(best, code, tap(0, dx), 6 + dx);
        if (cvalid) {
          *reinterpret_cast<f4*>(pa.pooled + cdst) = best;
          *reinterpret_cast<uint32_t*>(pa.arg + cdst) = pack_codes(code);
        } else {  // the run's first range: the previous workgroup holds rows 4k-2, 4k-1
          // (indexed by (pj, pq): wino_pool_fix_kernel's thread numbering)
          pa.side_v[blockIdx.x * (WP * CQ) + pj * CQ + pq] = best;
          pa.side_c[blockIdx.x * (WP * CQ) + pj * CQ + pq] = pack_codes(code);
        }
      }
      // (b) pooled row 2k: pixel rows 4k .. 4k+2
      if (even_row) {
        f4 best = {kNegInf, kNegInf, kNegInf, kNegInf};
        int code[4] = {0, 0, 0, 0};
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
            if (dx < 2 || !edge) pool_take(best, code, tap(dy, dx), 3 * dy + dx);
        const int64_t o = ((orow + 2 * k) * WP + pj) * COUT + 4 * pq;
        *reinterpret_cast<f4*>(pa.pooled + o) = best;
        *reinterpret_cast<uint32_t*>(pa.arg + o) = pack_codes(code);
      }
      // (c) pooled row 2k+1: pixel rows 4k+2, 4k+3 here, 4k+4 in the next range
      // (none in an odd-TY image's last range)
      if (!even_row && (!OT || 2 * k + 1 < Hp)) {
        f4 best = {kNegInf, kNegInf, kNegInf, kNegInf};
        int code[4] = {0, 0, 0, 0};
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
            if (dx < 2 || !edge) pool_take(best, code, tap(2 + dy, dx), 3 * dy + dx);
        const int64_t o = ((orow + 2 * k + 1) * WP + pj) * COUT + 4 * pq;
        if (k == KP - 1 || r >= rw.end) {
          // the image's last pooled row (pixel row 4k+4 is padding), or the
          // run's last range (the next workgroup's side part is merged by
          // wino_pool_fix_kernel)
          *reinterpret_cast<f4*>(pa.pooled + o) = best;
          *reinterpret_cast<uint32_t*>(pa.arg + o) = pack_codes(code);
          cvalid = false;
        } else {
          cv = best;
          cc[0] = code[0]; cc[1] = code[1]; cc[2] = code[2]; cc[3] = code[3];
          cdst = o;
          cvalid = true;
        }
      }
    }
    if (r >= rw.end) break;
  }
}

// Merges the top-row parts left by each run's first range into the pooled
// row its predecessor workgroup stored without them (one workgroup per run).
__global__ __launch_bounds__(256) void wino_pool_fix_kernel(const f4* __restrict__ side_v,
                                                            const uint32_t* __restrict__ side_c,
                                                            float* __restrict__ pooled,
                                                            uint8_t* __restrict__ arg,
                                                            int nranges, int KP, int Hp, int WP,
                                                            int COUT) {
  const int b = blockIdx.x;
  const int r = static_cast<int>(static_cast<int64_t>(b) * nranges / gridDim.x);
  const int n = r / KP, k = r - n * KP;
  const int CQ = COUT / 4;
  if (k == 0 || static_cast<int>(threadIdx.x) >= WP * CQ) return;
  const int pj = threadIdx.x / CQ, pq = threadIdx.x - pj * CQ;
  const int64_t o = ((static_cast<int64_t>(n) * Hp + 2 * k - 1) * WP + pj) * COUT + 4 * pq;
  f4 best = *reinterpret_cast<const f4*>(pooled + o);
  const uint32_t c0 = *reinterpret_cast<const uint32_t*>(arg + o);
  int code[4] = {static_cast<int>(c0 & 0xFF), static_cast<int>((c0 >> 8) & 0xFF),
                 static_cast<int>((c0 >> 16) & 0xFF), static_cast<int>(c0 >> 24)};
  const f4 sv = side_v[b * (WP * CQ) + threadIdx.x];
  const uint32_t sc = side_c[b * (WP * CQ) + threadIdx.x];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (sv[q] > best[q]) {
      best[q] = sv[q];
      code[q] = static_cast<int>((sc >> (8 * q)) & 0xFF);
    }
  *reinterpret_cast<f4*>(pooled + o) = best;
  *reinterpret_cast<uint32_t*>(arg + o) = pack_codes(code);
}

template <int CIN, int COUT, int RT>
bool run_wino_pool(const float* x, const float* w, const float* b, float* pooled, uint8_t* arg,
                   float* side, int64_t side_floats, int N, int H, int W, hipStream_t s) {
  using P = PoolGeo<CIN, COUT, RT>;
  if (W != P::W || H % 2 != 0 || H < 4) return false;
  const int TY = H / 2, TX = W / 2;
  const int64_t NT = static_cast<int64_t>(N) * TY * TX;
  // integer range / tile index math throughout (no fdivi): int32 bounds only
  if (NT >= (int64_t{1} << 30) || static_cast<int64_t>(N) * H * W * CIN * 4 > kMaxBufBytes)
    return false;
  WinoArgs a{};
  a.src = x;
  a.w = w;
  a.bias = b;
  a.N = N; a.H = H; a.W = W;
  a.TY = TY; a.TX = TX; a.NT = static_cast<int>(NT);
  a.nranges = N * ((TY + 1) / 2);  // tile-row pairs; odd TY: a last single row
  a.rTX = 1.f / static_cast<float>(TX);
  a.rTY = 1.f / static_cast<float>(TY);
  a.wcin = CIN; a.wcout = COUT;
  a.maxrows = P::ROWS;
  a.runs = 1;
  static const int ablate = measure_knob("SA_WINO_ABLATE", 0);
  a.ablate = ablate;  // 1 no MFMA tasks, 16 no pool phase, 32 no image writes
  // workgroups per CU: LDS-bound, capped at 3 waves per SIMD unless
  // SA_WINO_POOL_OCC asks for another count (sweeps)
  static const int occ = measure_knob("SA_WINO_POOL_OCC", 0);
  const int lds_cu = static_cast<int>((160 * 1024) / (P::bytes + 256));
  const int per_cu = std::max(1, std::min(occ > 0 ? occ : 3 * 4 / P::NW, lds_cu));
  const int G = std::max(1, std::min(a.nranges, conv_cus() * per_cu));
  const int side_n = (W / 2) * P::CQ;
  if (static_cast<int64_t>(G) * side_n * 5 > side_floats) return false;
  WinoPoolArgs pa{};
  pa.c = a;
  pa.pooled = pooled;
  pa.arg = arg;
  pa.side_v = reinterpret_cast<f4*>(side);
  pa.side_c = reinterpret_cast<uint32_t*>(side + static_cast<int64_t>(G) * side_n * 4);
  // odd tile-row maps: the OT instance, compiled for the widths that have one
  constexpr bool kHasOT = RT == 42 || RT == 48;
  if (TY % 2 != 0 && !kHasOT) return false;
  auto kern = TY % 2 != 0 ? wino_conv_pool_kernel<CIN, COUT, RT, kHasOT>
                          : wino_conv_pool_kernel<CIN, COUT, RT>;
  allow_lds_w(kern, P::bytes);
  hipLaunchKernelGGL(kern, dim3(G), dim3(64 * P::NW), P::bytes, s, pa);
  hipLaunchKernelGGL(wino_pool_fix_kernel, dim3(G), dim3(256), 0, s, pa.side_v, pa.side_c,
                     pooled, arg, a.nranges, (TY + 1) / 2, TY, W / 2, COUT);
  return true;
}

// Stage-2 head (32 -> 32 at 18x24 -> 9x12): its 9 tile rows per image are
// odd, so tile-row pairs would straddle images; here a range is one WHOLE
// image (108 tiles, padded to 7 groups of 16), every pooled window lies
// inside it, and no carry or fix-up is needed.  The 20 staged input rows
// (75 KB) and U (64 KB) leave one workgroup per CU; 7 waves take the 14
// (group, 16-channel slice) tasks two each, hold each task's A^T M A in
// registers until every wave has read its patches, then write the image.
template <int CIN, int COUT, int H, int W>
struct PoolImgGeo {
  static constexpr int TY = H / 2, TX = W / 2, NTI = TY * TX;
  static constexpr int RT = (NTI + 15) / 16 * 16;
  static constexpr int NG = RT / 16, NS = COUT / 16, NTASK = NG * NS;
  static constexpr int NW = 8;                       // tasks: two per wave (0..5), one (6, 7)
  static constexpr int ROWS = H + 2, Wl = W + 2;
  static constexpr int PP = CIN + 4, IPP = COUT + 4;
  static constexpr int XREG = (ROWS * Wl * PP > H * W * IPP) ? ROWS * Wl * PP : H * W * IPP;
  // only the image interior is staged (the zero border is rewritten per image)
  static constexpr int MAXC = (H * W * (CIN / 4) + 64 * NW - 1) / (64 * NW);
  static constexpr size_t bytes = sizeof(float) * (16 * CIN * COUT + XREG + ROWS);
};

template <int CIN, int COUT, int H, int W>
__global__ __launch_bounds__(512, 1) void wino_conv_pool_img_kernel(WinoPoolArgs pa) {
  using P = PoolImgGeo<CIN, COUT, H, W>;
  constexpr int TX = P::TX, NTI = P::NTI, NG = P::NG, NTASK = P::NTASK, NW = P::NW;
  constexpr int NTH = 64 * NW, ROWS = P::ROWS, Wl = P::Wl, PP = P::PP, IPP = P::IPP;
  constexpr int MAXC = P::MAXC, C4 = CIN / 4, LC4 = C4 == 8 ? 3 : 2, NB = CIN / 16;
  constexpr int USTR = NB * 4 * COUT * 4, rowstr = Wl * PP;
  constexpr int Hp = H / 2, Wp = W / 2, CQ = COUT / 4;
  static_assert(NTH == 512 && NTASK <= 2 * NW && CIN % 16 == 0 && H % 2 == 0 && W % 2 == 0 &&
                MAXC <= 32, "shape");
  const WinoArgs& a = pa.c;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* U_s = smem;                    // [16 xi][NB][4 g][COUT][4]
  float* x_s = smem + 16 * CIN * COUT;  // staged rows [ROWS][Wl][PP], then the image [H][W][IPP]
  float* img = x_s;
  int* tab_s = reinterpret_cast<int*>(x_s + P::XREG);

  for (int e = threadIdx.x; e < CIN * COUT; e += NTH) {
    const int co = e % COUT, ci = e / COUT;
    float gk[3][3];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) gk[ky][kx] = a.w[((ky * 3 + kx) * CIN + ci) * COUT + co];
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
  const RangeWalk rw = range_walk(a.nranges, 1);  // a range = one image
  int r = rw.r;
  if (r >= rw.end) return;

  // staging slot k of a thread: image element e = (pixel, channel quad) of
  // the interior (its LDS place is row y + 1, column x + 1)
  auto build_tab = [&](int n) {
    if (threadIdx.x == 0) tab_s[0] = n * H * W * CIN;
  };
  f4 stg[MAXC];
  const auto srcr = buf_rsrc(a.src, static_cast<int64_t>(a.N) * H * W * CIN);
  auto prefetch = [&]() __attribute__((always_inline)) {
    const int base = tab_s[0];
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int e = threadIdx.x + k * NTH;
      stg[k] = bload(srcr, e < H * W * C4 ? static_cast<uint32_t>(base + 4 * e) * 4u : kOOB);
    }
  };
  build_tab(r);
  __syncthreads();
  prefetch();
  constexpr float kNegInf = -__builtin_inff();

  for (;;) {
    __syncthreads();  // U_s written / the previous image's pool reads are done
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int e = threadIdx.x + k * NTH;
      if (e < H * W * C4) {
        const int pix = e >> LC4, q = e & (C4 - 1);
        const int y = pix / W, x = pix - y * W;
        *reinterpret_cast<f4*>(x_s + ((y + 1) * Wl + x + 1) * PP + 4 * q) = stg[k];
      }
    }
    // the zero border (the previous image's pre-pool map overwrote it)
    for (int e = threadIdx.x; e < (2 * Wl + 2 * H) * C4; e += NTH) {
      const int q = e % C4, c = e / C4;
      const int pix = c < 2 * Wl ? (c < Wl ? c : (ROWS - 1) * Wl + c - Wl)
                                 : ((c - 2 * Wl) / 2 + 1) * Wl + ((c - 2 * Wl) & 1) * (Wl - 1);
      *reinterpret_cast<f4*>(x_s + pix * PP + 4 * q) = f4{0.f, 0.f, 0.f, 0.f};
    }
    const int n = r;
    ++r;
    build_tab(r < rw.end ? r : n);  // unconditional: see wino_conv_kernel
    __syncthreads();
    prefetch();

    f4 Yt[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int task = wave + NW * i;
      const int grp = task % NG, sl = task / NG;
      const int t0 = 16 * grp + c16;
      const int t = t0 < NTI ? t0 : 0;
      const int ty = t / TX, tx = t - ty * TX;
      const int co0 = sl * 16;
      const float* xp = x_s + (2 * ty * Wl + 2 * tx) * PP + 4 * g;
      const float* up = U_s + (g * COUT + co0 + c16) * 4;
      f4 acc[16];
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) acc[xi] = f4{0.f, 0.f, 0.f, 0.f};
      if (task < NTASK) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          f4 d[16];
#pragma unroll
          for (int dy = 0; dy < 4; ++dy)
#pragma unroll
            for (int dx = 0; dx < 4; ++dx)
              d[4 * dy + dx] = *reinterpret_cast<const f4*>(xp + dy * rowstr + dx * PP + 16 * b);
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
          const float* ub = up + b * 4 * COUT * 4;
#pragma unroll
          for (int xp2 = 0; xp2 < 8; ++xp2) {
            f4 ua[2];
#pragma unroll
            for (int q = 0; q < 2; ++q)
              ua[q] = *reinterpret_cast<const f4*>(ub + (2 * xp2 + q) * USTR);
#pragma unroll
            for (int v = 0; v < 4; ++v)
#pragma unroll
              for (int q = 0; q < 2; ++q)
                acc[2 * xp2 + q] = mfma4(ua[q][v], V[2 * xp2 + q][v], acc[2 * xp2 + q]);
          }
        }
      }
      f4 tt[4][2];
#pragma unroll
      for (int ra = 0; ra < 4; ++ra) {
        tt[ra][0] = (acc[4 * ra] + acc[4 * ra + 1]) + acc[4 * ra + 2];
        tt[ra][1] = (acc[4 * ra + 1] - acc[4 * ra + 2]) - acc[4 * ra + 3];
      }
      const f4 bv = *reinterpret_cast<const f4*>(a.bias + (co0 < COUT ? co0 : 0) + 4 * g);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        Yt[i][c] = (tt[0][c] + tt[1][c]) + tt[2][c] + bv;
        Yt[i][2 + c] = (tt[1][c] - tt[2][c]) - tt[3][c] + bv;
      }
    }
    __syncthreads();  // every wave's patch reads are done: x_s becomes the image
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int task = wave + NW * i;
      const int grp = task % NG, sl = task / NG;
      const int t = 16 * grp + c16;
      if (task < NTASK && t < NTI) {
        const int ty = t / TX, tx = t - ty * TX;
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
          for (int dx = 0; dx < 2; ++dx)
            *reinterpret_cast<f4*>(img + ((2 * ty + dy) * W + 2 * tx + dx) * IPP + sl * 16 + 4 * g) =
                Yt[i][2 * dy + dx];
      }
    }
    __syncthreads();
    // pool phase: every window of the image (pad-before 0, the bottom /
    // right tap row beyond the image is padding)
    // lanes permuted inside each 64-element chunk (8 pooled pixels x 8
    // quads) by the conflict-free pool lane map (wino_conv_pool_kernel)
    static_assert(CQ == 8, "lane map for 8 channel quads");
    constexpr PoolLaneMap<CQ, IPP> kMap{};
    const int lmap = kMap.pj[threadIdx.x & 63] * CQ + kMap.pq[threadIdx.x & 63];
    for (int e0 = threadIdx.x & ~63; e0 < Hp * Wp * CQ; e0 += NTH) {
      const int e = e0 + lmap;
      if (e >= Hp * Wp * CQ) continue;
      const int pr = e / (Wp * CQ), rem = e - pr * (Wp * CQ);
      const int pc = rem / CQ, pq = rem - pc * CQ;
      f4 best = {kNegInf, kNegInf, kNegInf, kNegInf};
      int code[4] = {0, 0, 0, 0};
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int y = 2 * pr + dy, x = 2 * pc + dx;
          if (y < H && x < W)
            pool_take(best, code,
                      *reinterpret_cast<const f4*>(img + (y * W + x) * IPP + 4 * pq), 3 * dy + dx);
        }
      const int64_t o = ((static_cast<int64_t>(n) * Hp + pr) * Wp + pc) * COUT + 4 * pq;
      *reinterpret_cast<f4*>(pa.pooled + o) = best;
      *reinterpret_cast<uint32_t*>(pa.arg + o) = pack_codes(code);
    }
    if (r >= rw.end) break;
  }
}

template <int CIN, int COUT, int H, int W>
bool run_wino_pool_img(const float* x, const float* w, const float* b, float* pooled,
                       uint8_t* arg, int N, int Hr, int Wr, hipStream_t s) {
  using P = PoolImgGeo<CIN, COUT, H, W>;
  if (Hr != H || Wr != W || static_cast<int64_t>(N) * H * W * CIN * 4 > kMaxBufBytes) return false;
  WinoArgs a{};
  a.src = x;
  a.w = w;
  a.bias = b;
  a.N = N; a.H = H; a.W = W;
  a.nranges = N;
  a.runs = 1;
  const int G = std::max(1, std::min(N, conv_cus()));
  auto kern = wino_conv_pool_img_kernel<CIN, COUT, H, W>;
  allow_lds_w(kern, P::bytes);
  WinoPoolArgs pa{};
  pa.c = a;
  pa.pooled = pooled;
  pa.arg = arg;
  hipLaunchKernelGGL(kern, dim3(G), dim3(64 * P::NW), P::bytes, s, pa);
  return true;
}


// ------------------------------------------------------------ weight grad
// Winograd F(2x2, 3x3) weight gradient.  With Z = A dY A^T (4x4 per 2x2 dY
// tile) and V = B^T d B (the forward's input transform),
//   dL/dU[xi][ci][co] = sum_tiles V[xi][tile][ci] Z[xi][tile][co]
//   dW[ci][co] = G^T (dL/dU) G,  db[co] = sum dY[co]
// (U = G g G^T is linear in g).  The 16 tile reductions are MFMA GEMMs with
// k = tile: A[i = ci][k] = V, B[k][j = co] = Z; lane (c16, g) computes V for
// its input channel and Z for its output channel of tile g, from the input
// and dY rows of the range staged in LDS.  Waves own xi rows (XR of the 4)
// and split the range's k-steps (4 tiles each) when they own all of them.
// Each workgroup finishes with G^T P G of its partial sums and writes them in
// the direct kernel's wgrad slot layout; the fixed-order slot reduction of
// conv_f32.hip sums the slots (deterministic).
struct WinoWgArgs {
  const float* x;   // [N, H, W, CIN]
  const float* dy;  // [N, H, W, COUT]
  float* part;      // slots [G][rows16][COUT]
  int N, H, W;
  int TY, TX, NT, nranges, maxrows, rows16;
  float rTX, rTY, rWl, rWd;
  int relu_in;
};

// input patch rows used by B^T rows a = XG*XR .. XG*XR + XR - 1
// (a = 0: d0 - d2, 1: d1 + d2, 2: d2 - d1, 3: d1 - d3)
__host__ __device__ constexpr bool wg_need_row(int XR, int XG, int dy) {
  return XR == 4 ? true
       : XR == 2 ? (XG == 0 ? dy <= 2 : dy >= 1)
       : (XG == 0 ? (dy == 0 || dy == 2)
          : XG == 3 ? (dy == 1 || dy == 3) : (dy == 1 || dy == 2));
}

template <int CIN, int COUT, int XR, int RT, int MAXCX, int MAXCD>
__global__ __launch_bounds__(256, 1) void wino_wgrad_kernel(WinoWgArgs a) {
  constexpr int NW = 4, NTH = 256;
  constexpr int PX = CIN + 8, PD = COUT + 8;  // 2*pitch = 16 mod 32 words
  constexpr int C4X = CIN / 4, C4D = COUT / 4;
  constexpr int LCX = C4X == 4 ? 2 : 3, LCD = C4D == 4 ? 2 : 3;
  constexpr int NBI = CIN / 16, NBO = COUT / 16;
  constexpr int NXG = 4 / XR;   // xi-row groups
  constexpr int KS = NW / NXG;  // waves sharing one group's k-steps
  constexpr int NSTEP = RT / 4;
  static_assert(XR == 1 || XR == 2 || XR == 4, "XR");
  static_assert(MAXCX <= 32 && MAXCD <= 32, "stager masks");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Wl = 2 * a.TX + 2, Wd = 2 * a.TX;
  float* x_s = smem;                          // [maxrows][Wl][PX]
  float* d_s = x_s + a.maxrows * Wl * PX;     // [maxrows][Wd][PD] (same rows)
  int* tab_s = reinterpret_cast<int*>(d_s + a.maxrows * Wd * PD);  // [maxrows]
  int* tile_s = tab_s + a.maxrows;                                  // [RT][2]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int xg = wave / KS, kq = wave - (wave / KS) * KS;

  int r = blockIdx.x;
  if (r >= a.nranges) return;

  // ---- staging slots (see wino_conv_kernel): X with a zero halo, dY on the
  // same LDS rows (the halo rows it does not need are staged and unused)
  int sx_L[MAXCX], sx_o[MAXCX], sd_L[MAXCD], sd_o[MAXCD];
#pragma unroll
  for (int k = 0; k < MAXCX; ++k) {
    const int e = threadIdx.x + k * NTH;
    const int ch = e & (C4X - 1), pix = e >> LCX;
    const int L = pix / Wl, col = pix - L * Wl;
    sx_L[k] = L < a.maxrows ? L : -1;
    sx_o[k] = (col >= 1 && col <= a.W) ? (col - 1) * CIN + 4 * ch : -1;
  }
#pragma unroll
  for (int k = 0; k < MAXCD; ++k) {
    const int e = threadIdx.x + k * NTH;
    const int ch = e & (C4D - 1), pix = e >> LCD;
    const int L = pix / Wd, col = pix - L * Wd;
    sd_L[k] = L < a.maxrows ? L : -1;
    sd_o[k] = col < a.W ? col * COUT + 4 * ch : -1;
  }
  // row table: global pixel index (n*H + y)*W of LDS row L, or -1
  auto row_of = [&](const RangeGeom& gm, int L) {
    int v = -1;
    if (L < gm.rows) {
      const int p = (L >= gm.off1) + (L >= gm.off2) + (L >= gm.off3);
      const int offp = p == 0 ? 0 : (p == 1 ? gm.off1 : (p == 2 ? gm.off2 : gm.off3));
      const int y = 2 * (p == 0 ? gm.tya0 : 0) - 1 + (L - offp);
      if (y >= 0 && y < a.H) v = ((gm.n0 + p) * a.H + y) * a.W;
    }
    return v;
  };
  auto geom = [&](int rr) {
    RangeGeom g2;
    WinoArgs t{};
    t.NT = a.NT; t.TX = a.TX; t.TY = a.TY; t.rTX = a.rTX; t.rTY = a.rTY;
    g2 = range_geom(t, rr, RT);
    return g2;
  };
  f4 stx[MAXCX], std_[MAXCD];
  uint32_t okx = 0, okd = 0;
  auto prefetch = [&]() {  // reads tab_s
    okx = 0;
    okd = 0;
#pragma unroll
    for (int k = 0; k < MAXCX; ++k) {
      const int rb = sx_L[k] >= 0 ? tab_s[sx_L[k]] : -1;
      const bool in = rb >= 0 && sx_o[k] >= 0;
      stx[k] = *reinterpret_cast<const f4*>(a.x + (in ? rb * CIN + sx_o[k] : 0));
      okx |= static_cast<uint32_t>(in) << k;
    }
#pragma unroll
    for (int k = 0; k < MAXCD; ++k) {
      const int rb = sd_L[k] >= 0 ? tab_s[sd_L[k]] : -1;
      const bool in = rb >= 0 && sd_o[k] >= 0;
      std_[k] = *reinterpret_cast<const f4*>(a.dy + (in ? rb * COUT + sd_o[k] : 0));
      okd |= static_cast<uint32_t>(in) << k;
    }
  };
  {
    const RangeGeom gm = geom(r);
    if (threadIdx.x < a.maxrows) tab_s[threadIdx.x] = row_of(gm, threadIdx.x);
  }
  __syncthreads();
  prefetch();

  f4 acc[XR][4][NBI][NBO];
#pragma unroll
  for (int i = 0; i < XR; ++i)
#pragma unroll
    for (int bc = 0; bc < 4; ++bc)
#pragma unroll
      for (int b = 0; b < NBI; ++b)
#pragma unroll
        for (int b2 = 0; b2 < NBO; ++b2) acc[i][bc][b][b2] = f4{0.f, 0.f, 0.f, 0.f};
  float dbacc[NBO];
#pragma unroll
  for (int b2 = 0; b2 < NBO; ++b2) dbacc[b2] = 0.f;

  const int rsx = Wl * PX, rsd = Wd * PD;
  for (;;) {
    __syncthreads();  // the previous range's LDS reads are done
#pragma unroll
    for (int k = 0; k < MAXCX; ++k) {
      if (sx_L[k] >= 0) {
        const int e = threadIdx.x + k * NTH;
        f4 v = stx[k];
        const bool in = (okx >> k) & 1u;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float t = in ? v[q] : 0.f;
          v[q] = a.relu_in ? relu0(t) : t;
        }
        *reinterpret_cast<f4*>(x_s + (e >> LCX) * PX + 4 * (e & (C4X - 1))) = v;
      }
    }
#pragma unroll
    for (int k = 0; k < MAXCD; ++k) {
      if (sd_L[k] >= 0) {
        const int e = threadIdx.x + k * NTH;
        f4 v = std_[k];
        const bool in = (okd >> k) & 1u;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = in ? v[q] : 0.f;
        *reinterpret_cast<f4*>(d_s + (e >> LCD) * PD + 4 * (e & (C4D - 1))) = v;
      }
    }
    const int cur = r;
    r += gridDim.x;
    {
      // tile table of the current range, row table of the next one
      const RangeGeom gm = geom(cur);
      for (int tt = threadIdx.x; tt < RT; tt += NTH) {
        const int t = gm.t0 + tt;
        int xb = -1, db = -1;
        if (t < gm.t1) {
          const int R = fdivi(t, a.rTX), tx = t - R * a.TX;
          const int n = fdivi(R, a.rTY), ty = R - n * a.TY;
          const int p = n - gm.n0;
          const int offp = p == 0 ? 0 : (p == 1 ? gm.off1 : (p == 2 ? gm.off2 : gm.off3));
          const int base = offp + 2 * (ty - (p == 0 ? gm.tya0 : 0));
          xb = (base * Wl + 2 * tx) * PX;
          db = ((base + 1) * Wd + 2 * tx) * PD;
        }
        tile_s[2 * tt] = xb;
        tile_s[2 * tt + 1] = db;
      }
      if (r < a.nranges) {
        const RangeGeom gn = geom(r);
        if (threadIdx.x < a.maxrows) tab_s[threadIdx.x] = row_of(gn, threadIdx.x);
      }
    }
    __syncthreads();
    if (r < a.nranges) prefetch();  // in flight under the MFMAs below

    auto run = [&](auto XGc) {
      constexpr int XG = decltype(XGc)::value;
      for (int st = kq; st < NSTEP; st += KS) {
        const int tt = 4 * st + kperm(g);
        int xb = tile_s[2 * tt], db = tile_s[2 * tt + 1];
        const bool valid = xb >= 0;
        xb = valid ? xb : 0;
        db = valid ? db : 0;
        // Z rows (this group's xi rows) for every output-channel block
        f4 zf[XR][NBO];  // zf[i][b2][bcol] = Z[a = XG*XR + i][bcol] for co
#pragma unroll
        for (int b2 = 0; b2 < NBO; ++b2) {
          const float* dp = d_s + db + 16 * b2 + c16;
          float y00 = dp[0], y01 = dp[PD], y10 = dp[rsd], y11 = dp[rsd + PD];
          if (!valid) y00 = y01 = y10 = y11 = 0.f;
          if constexpr (XG == 0) dbacc[b2] += (y00 + y01) + (y10 + y11);
#pragma unroll
          for (int i = 0; i < XR; ++i) {
            const int ar = XG * XR + i;
            float r0, r1;
            if (ar == 0) { r0 = y00; r1 = y01; }
            else if (ar == 1) { r0 = y00 + y10; r1 = y01 + y11; }
            else if (ar == 2) { r0 = y00 - y10; r1 = y01 - y11; }
            else { r0 = -y10; r1 = -y11; }
            zf[i][b2] = f4{r0, r0 + r1, r0 - r1, -r1};
          }
        }
#pragma unroll
        for (int b = 0; b < NBI; ++b) {
          const float* xp = x_s + xb + 16 * b + c16;
          // patch rows this group needs (B^T row a combines two rows)
          float d[4][4];
#pragma unroll
          for (int dy = 0; dy < 4; ++dy) {
            if (wg_need_row(XR, XG, dy)) {
#pragma unroll
              for (int dx = 0; dx < 4; ++dx) d[dy][dx] = xp[dy * rsx + dx * PX];
            } else {
#pragma unroll
              for (int dx = 0; dx < 4; ++dx) d[dy][dx] = 0.f;
            }
          }
#pragma unroll
          for (int i = 0; i < XR; ++i) {
            const int ar = XG * XR + i;
            float sq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              if (ar == 0) sq[q] = d[0][q] - d[2][q];
              else if (ar == 1) sq[q] = d[1][q] + d[2][q];
              else if (ar == 2) sq[q] = d[2][q] - d[1][q];
              else sq[q] = d[1][q] - d[3][q];
            }
            float V[4] = {sq[0] - sq[2], sq[1] + sq[2], sq[2] - sq[1], sq[1] - sq[3]};
            if (!valid) V[0] = V[1] = V[2] = V[3] = 0.f;
#pragma unroll
            for (int bc = 0; bc < 4; ++bc)
#pragma unroll
              for (int b2 = 0; b2 < NBO; ++b2)
                acc[i][bc][b][b2] = mfma4(V[bc], zf[i][b2][bc], acc[i][bc][b][b2]);
          }
        }
      }
    };
    if constexpr (NXG == 1) {
      run(std::integral_constant<int, 0>{});
    } else if constexpr (NXG == 2) {
      if (xg == 0) run(std::integral_constant<int, 0>{});
      else run(std::integral_constant<int, 1>{});
    } else {
      if (xg == 0) run(std::integral_constant<int, 0>{});
      else if (xg == 1) run(std::integral_constant<int, 1>{});
      else if (xg == 2) run(std::integral_constant<int, 2>{});
      else run(std::integral_constant<int, 3>{});
    }
    if (r >= a.nranges) break;
  }

  // ---- workgroup epilogue: P = sum over the KS waves of a group (fixed
  // order) in LDS, then dW = G^T P G per (ci, co) into this slot
  __syncthreads();
  float* P = smem;                      // [16][CIN][COUT]
  float* dB = smem + 16 * CIN * COUT;   // [COUT]
  for (int k = 0; k < KS; ++k) {
    if (kq == k) {
#pragma unroll
      for (int i = 0; i < XR; ++i)
#pragma unroll
        for (int bc = 0; bc < 4; ++bc)
#pragma unroll
          for (int b = 0; b < NBI; ++b)
#pragma unroll
            for (int b2 = 0; b2 < NBO; ++b2)
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const int xi = 4 * (xg * XR + i) + bc;
                const int ci = 16 * b + 4 * g + q, co = 16 * b2 + c16;
                float* pp = P + (xi * CIN + ci) * COUT + co;
                *pp = (k == 0 ? 0.f : *pp) + acc[i][bc][b][b2][q];
              }
      if (xg == 0) {
#pragma unroll
        for (int b2 = 0; b2 < NBO; ++b2) {
          float v = dbacc[b2];
          v += __shfl_xor(v, 16);
          v += __shfl_xor(v, 32);
          if (g == 0) dB[16 * b2 + c16] = (k == 0 ? 0.f : dB[16 * b2 + c16]) + v;
        }
      }
    }
    __syncthreads();
  }
  float* slot = a.part + static_cast<int64_t>(blockIdx.x) * a.rows16 * COUT;
  for (int e = threadIdx.x; e < CIN * COUT; e += NTH) {
    const int ci = e / COUT, co = e - (e / COUT) * COUT;
    float pm[4][4];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) pm[xi >> 2][xi & 3] = P[(xi * CIN + ci) * COUT + co];
    float t[3][4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      t[0][b] = pm[0][b] + 0.5f * (pm[1][b] + pm[2][b]);
      t[1][b] = 0.5f * (pm[1][b] - pm[2][b]);
      t[2][b] = 0.5f * (pm[1][b] + pm[2][b]) + pm[3][b];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float w0 = t[i][0] + 0.5f * (t[i][1] + t[i][2]);
      const float w1 = 0.5f * (t[i][1] - t[i][2]);
      const float w2 = 0.5f * (t[i][1] + t[i][2]) + t[i][3];
      slot[((3 * i + 0) * CIN + ci) * COUT + co] = w0;
      slot[((3 * i + 1) * CIN + ci) * COUT + co] = w1;
      slot[((3 * i + 2) * CIN + ci) * COUT + co] = w2;
    }
  }
  for (int co = threadIdx.x; co < COUT; co += NTH) slot[9 * CIN * COUT + co] = dB[co];
}

template <int CIN, int COUT, int XR, int RT, int MAXCX, int MAXCD>
bool run_wino_wgrad(const WgradArgs& c, float* ws, hipStream_t s) {
  const int H = c.H, W = c.W;
  const int TY = (H + 1) / 2, TX = (W + 1) / 2;
  const int64_t NT = static_cast<int64_t>(c.N) * TY * TX;
  if (NT >= (1 << 22) || TX > 1024 || TY > 1024) return false;
  const int per_img = TY * TX;
  const int maxparts = (RT - 1 + per_img - 1) / per_img + 1;
  if (maxparts > kMaxParts) return false;
  const int Wl = 2 * TX + 2, Wd = 2 * TX;
  const int maxrows = 2 * ((RT - 1 + TX - 1) / TX + 1) + 2 * maxparts;
  if (maxrows * Wl * (CIN / 4) > MAXCX * 256 || maxrows * Wd * (COUT / 4) > MAXCD * 256 ||
      maxrows > 256)
    return false;
  if (static_cast<int64_t>(c.N) * H * W >= (int64_t(1) << 31) / 32) return false;
  const size_t stage = sizeof(float) * (static_cast<size_t>(maxrows) * (Wl * (CIN + 8) +
                                                                        Wd * (COUT + 8))) +
                       sizeof(int) * (maxrows + 2 * RT);
  const size_t epi = sizeof(float) * (16 * CIN * COUT + COUT);
  const size_t bytes = std::max(stage, epi);
  if (bytes > 160 * 1024) return false;
  const int M = 9 * CIN;
  const int rows16 = ((M + 16) / 16) * 16;
  const int nranges = static_cast<int>((NT + RT - 1) / RT);
  // slots: one per resident workgroup (<= the direct kernel's workspace)
  const int64_t cap = wgrad_workspace_floats(3, CIN, COUT) / (static_cast<int64_t>(rows16) * COUT);
  const int G = static_cast<int>(std::min<int64_t>({nranges, conv_cus(), cap}));
  WinoWgArgs a{};
  a.x = static_cast<const float*>(c.src);
  a.dy = c.dy;
  a.part = ws;
  a.N = c.N; a.H = H; a.W = W;
  a.TY = TY; a.TX = TX; a.NT = static_cast<int>(NT); a.nranges = nranges;
  a.maxrows = maxrows; a.rows16 = rows16;
  a.rTX = 1.f / static_cast<float>(TX);
  a.rTY = 1.f / static_cast<float>(TY);
  a.relu_in = c.relu_in;
  auto kern = wino_wgrad_kernel<CIN, COUT, XR, RT, MAXCX, MAXCD>;
  allow_lds_w(kern, bytes);
  hipLaunchKernelGGL(kern, dim3(G), dim3(256), bytes, s, a);
  wgrad_reduce_slots(ws, G, rows16, COUT, CIN, c.dw, c.db, s);
  return true;
}


// ------------------------------------------------- fused data + weight grad
// One backward pass of a 3x3/1 SAME conv whose input x is also the ReLU
// mask of the data gradient (every residual conv of the deep torso:
// experiment.py:166-172, t = relu(conv(relu(x))), y = conv(t) + x):
//   dX = (dY (*) W_flipped^T) * (x > 0) [+ add]      Winograd, as above
//   dW += sum_p relu?(x)[p + tap] dY[p],  db += sum_p dY[p]   direct MFMA
// dY and x are staged ONCE per range (same rows, same halo) and serve the
// data gradient's source and mask and both weight-gradient operands - the
// separate dgrad + wgrad kernels read each of them twice from HBM (at the
// 36x48x16 stage every such pass is 357 MB per learner step).  Waves 0-3
// run the Winograd data-gradient tasks (16-tile groups) plus a few
// weight-gradient k-steps, waves 4-7 the rest of the weight gradient
// (k = one 2x2 tile = 4 pixels per MFMA).  Weight-gradient partials go to
// the wgrad slot layout (fixed-order reduction: deterministic).
struct WinoBwdArgs {
  const float* dy;   // [N, H, W, C] (the dgrad source)
  const float* w;    // forward weights HWIO [3, 3, C, C]
  const float* x;    // [N, H, W, C] forward input: dgrad mask + wgrad operand
  const float* add;  // [N, H, W, C] or null
  float* out;        // dX [N, H, W, C]
  float* part;       // wgrad slots [G][rows16][C]
  int N, H, W;
  int TY, TX, NT, nranges, maxrows, rows16;
  float rTX, rTY;
  int relu_x;        // wgrad operand = relu(x)
  int mask_x = 1;    // dX masked by (x > 0) (fused32 kernel; the 16-channel one always masks)
  int ablate = 0;    // measurement knob (SA_FUSED_ABLATE, SA_MEASURE_KNOBS builds only):
                     // 2 no dgrad, 4 no wgrad, 8 no global dY loads (fused32)
  int runs = 1;      // contiguous range runs (wino_bwd_fused_kernel; fused32 always)
  unsigned* err = nullptr;  // the device's sticky conv error word (rmsprop.hip guard)
  int fault = 0;     // fault injection: every hand-off wait reports a timeout
  int prio = 0;      // SA_FUSED_PRIO: s_setprio 1 for the weight-gradient waves
                     // (1) or the data-gradient waves (2)
};

// WWG: the weight gradient in Winograd form too (dL/dU = sum_tiles V(x) .*
// Z(dY), dW = G^T P G, as wino_wgrad_kernel): waves 0-3 run the dgrad groups
// only, waves 4-7 four k-steps of 4 tiles each, 256 instead of 576 weight-
// gradient MFMAs per range.  One workgroup per CU (LDS) either way, so the
// WWG instance may use up to 256 VGPRs.
// NW waves per workgroup (WWG only, else 8): NW / 2 data-gradient waves (one
// 16-tile group each) and NW / 2 weight-gradient waves splitting the range's
// RT / 4 k-steps evenly.  NW = 12 over 96-tile ranges (three waves per SIMD)
// does not fit: capped at 168 VGPRs the kernel spills 121 (it needs ~256 at
// two waves per SIMD), so only NW = 8 is instantiated.
template <int C, int RT, int MAXC, int KD, bool WWG = false, bool RELU = false, int NW = 8,
          int GH = 0, int GW = 0>
__global__ __launch_bounds__(64 * NW, WWG ? 1 : 2) void wino_bwd_fused_kernel(WinoBwdArgs a) {
  constexpr int NTH = 64 * NW;
  const TileGeo<GH, GW, RT, wino_lpad_on(1)> G(a.H, a.W, a.TY, a.TX, a.NT, a.rTX, a.rTY,
                                                a.maxrows);
  constexpr int PP = C + 4;
  constexpr int C4 = C / 4;
  constexpr int LC4 = C4 == 4 ? 2 : 3;
  constexpr int NG = RT / 16;          // dgrad tasks (16-tile groups)
  constexpr int NWG = NW - NG;         // weight-gradient waves (WWG)
  constexpr int USTR = 4 * C * 4;      // floats per xi in U_s (one ci block)
  static_assert(C == 16, "fused backward: 16 channels (LDS)");
  static_assert(WWG ? (NG == NW / 2 && (RT / 4) % NWG == 0) : (NW == 8 && NG == 4),
                "one dgrad wave per 16-tile group");
  static_assert(WWG ? (RT % 16 == 0) : (RT - 4 * KD >= 0 && (RT - 4 * KD) % 4 == 0),
                "work split");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Wl = G.WL;
  const int rowstr = Wl * PP;
  float* U_s = smem;                         // [16 xi][4 g][C][4]
  float* d_s = U_s + 16 * C * C;             // dY rows [maxrows][Wl][PP]
  float* x_s = d_s + G.maxrows * rowstr;     // x rows, same geometry
  int* tab_s = reinterpret_cast<int*>(x_s + G.maxrows * rowstr);  // [maxrows]
  int* tile_s = tab_s + G.maxrows;                                // [RT]

  // U = G g' G^T of the flipped / transposed weights (the dgrad conv)
  for (int e = threadIdx.x; e < C * C; e += NTH) {
    const int co = e % C, ci = e / C;  // ci = dY channel, co = dX channel
    float gk[3][3];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) gk[ky][kx] = a.w[(((2 - ky) * 3 + (2 - kx)) * C + co) * C + ci];
    float t[4][3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      t[0][kx] = gk[0][kx];
      t[1][kx] = 0.5f * ((gk[0][kx] + gk[1][kx]) + gk[2][kx]);
      t[2][kx] = 0.5f * ((gk[0][kx] - gk[1][kx]) + gk[2][kx]);
      t[3][kx] = gk[2][kx];
    }
    const int gq = (ci >> 2) & 3, v = ci & 3;
#pragma unroll
    for (int ra = 0; ra < 4; ++ra) {
      const float u[4] = {t[ra][0], 0.5f * ((t[ra][0] + t[ra][1]) + t[ra][2]),
                          0.5f * ((t[ra][0] - t[ra][1]) + t[ra][2]), t[ra][2]};
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) U_s[(4 * ra + rb) * USTR + (gq * C + co) * 4 + v] = u[rb];
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;

  const RangeWalk rw = range_walk(a.nranges, a.runs);
  int r = rw.r;
  if (r >= rw.end) return;
  {
    const int w0 = __builtin_amdgcn_readfirstlane(wave);
    if ((a.prio == 1 && w0 >= NW / 2) || (a.prio == 2 && w0 < NW / 2)) __builtin_amdgcn_s_setprio(1);
  }

  // staging slots: element e of both images = (row L, col, quad)
  int sl_L[MAXC], sl_o[MAXC];
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int e = threadIdx.x + k * NTH;
    const int ch = e & (C4 - 1), pix = e >> LC4;
    const int L = pix / G.WL0, col = pix - L * G.WL0;
    sl_L[k] = L < G.maxrows ? L : -1;
    sl_o[k] = (col >= 1 && col <= G.W) ? (col - 1) * C + 4 * ch : -1;
  }
  auto build_tab = [&](int rr) {
    const RangeGeom gm = G.range(rr);
    const int L = threadIdx.x;
    if (L < G.maxrows) {
      int v = -1;
      if (L < gm.rows) {
        const int p = G.part_of(gm, L);
        const int offp = G.part_off(gm, p);
        const int y = 2 * (p == 0 ? gm.tya0 : 0) - 1 + (L - offp);
        if (y >= 0 && y < G.H) v = ((gm.n0 + p) * G.H + y) * G.W * C;
      }
      tab_s[L] = v;
    }
  };
  f4 sd[MAXC], sx[MAXC];
  const int64_t nfl = static_cast<int64_t>(a.N) * G.H * G.W * C;
  const auto dyr = buf_rsrc(a.dy, nfl), xr = buf_rsrc(a.x, nfl);
  auto prefetch = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int rb = sl_L[k] >= 0 ? tab_s[sl_L[k]] : -1;
      const bool in = rb >= 0 && sl_o[k] >= 0;
      const uint32_t off = in ? static_cast<uint32_t>(rb + sl_o[k]) * 4u : kOOB;
      sd[k] = bload(dyr, off);
      sx[k] = bload(xr, off);
    }
  };
  build_tab(r);
  __syncthreads();
  prefetch();

  constexpr int NACC = WWG ? 16 : 9;  // Winograd xi (4 i + bc) or direct taps
  f4 wacc[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k) wacc[k] = f4{0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;

  for (;;) {
    __syncthreads();  // the previous range's LDS reads are done
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      if (sl_L[k] >= 0) {
        const int e = threadIdx.x + k * NTH;
        const f4 vd = sd[k], vx = sx[k];  // zero where out of the image
        const int o = ((e >> LC4) + pad_pix<decltype(G)::PADC>(sl_L[k])) * PP + 4 * (e & (C4 - 1));
        *reinterpret_cast<f4*>(d_s + o) = vd;
        *reinterpret_cast<f4*>(x_s + o) = vx;
      }
    }
    const int cur = r;
    r += rw.step;
    const RangeGeom gm = G.range(cur);
    // tile table of this range: LDS offset of each tile's patch origin
    if (threadIdx.x < RT) {
      const int t = gm.t0 + threadIdx.x;
      int v = -1;
      if (t < gm.t1) {
        const int R = G.div_tx(t), tx = t - R * G.TX;
        const int n = G.div_ty(R), ty = R - n * G.TY;
        const int p = n - gm.n0;
        const int offp = G.part_off(gm, p);
        v = ((offp + 2 * (ty - (p == 0 ? gm.tya0 : 0))) * Wl + 2 * tx) * PP;
      }
      tile_s[threadIdx.x] = v;
    }
    build_tab(r < rw.end ? r : cur);  // unconditional: see wino_conv_kernel
    __syncthreads();
    prefetch();

    // ---- data gradient: waves 0..3, one 16-tile group each
    if (wave < NG && gm.t0 + 16 * wave < gm.t1) {
      int t = gm.t0 + 16 * wave + c16;
      const bool valid = t < gm.t1;
      if (!valid) t = gm.t0;
      const int R = G.div_tx(t), tx = t - R * G.TX;
      const int n = G.div_ty(R), ty = R - n * G.TY;
      const int base = tile_s[valid ? 16 * wave + c16 : 0];
      const float* dp = d_s + base + 4 * g;
      // the skip operand of the 4 outputs: global loads issued before the
      // MFMAs so their latency hides under them
      f4 addv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int oy = 2 * ty + (q >> 1), ox = 2 * tx + (q & 1);
        const bool in = a.add != nullptr && valid && G.in_y(oy) && G.in_x(ox);
        const int64_t o = in ? ((static_cast<int64_t>(n) * G.H + oy) * G.W + ox) * C + 4 * g : 0;
        addv[q] = in ? *reinterpret_cast<const f4*>(a.add + o) : f4{0.f, 0.f, 0.f, 0.f};
      }
      f4 acc[16];
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) acc[xi] = f4{0.f, 0.f, 0.f, 0.f};
      f4 d[16];
#pragma unroll
      for (int dy = 0; dy < 4; ++dy)
#pragma unroll
        for (int dx = 0; dx < 4; ++dx)
          d[4 * dy + dx] = *reinterpret_cast<const f4*>(dp + dy * rowstr + dx * PP);
      f4 sv[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        sv[q] = tsub(d[q], d[8 + q]);
        sv[4 + q] = tadd(d[4 + q], d[8 + q]);
        sv[8 + q] = tsub(d[8 + q], d[4 + q]);
        sv[12 + q] = tsub(d[4 + q], d[12 + q]);
      }
      f4 V[16];
#pragma unroll
      for (int ra = 0; ra < 4; ++ra) {
        V[4 * ra + 0] = tsub(sv[4 * ra + 0], sv[4 * ra + 2]);
        V[4 * ra + 1] = tadd(sv[4 * ra + 1], sv[4 * ra + 2]);
        V[4 * ra + 2] = tsub(sv[4 * ra + 2], sv[4 * ra + 1]);
        V[4 * ra + 3] = tsub(sv[4 * ra + 1], sv[4 * ra + 3]);
      }
      const float* up = U_s + (g * C + c16) * 4;
#pragma unroll
      for (int xp2 = 0; xp2 < 8; ++xp2) {
        const f4 u0 = *reinterpret_cast<const f4*>(up + (2 * xp2) * USTR);
        const f4 u1 = *reinterpret_cast<const f4*>(up + (2 * xp2 + 1) * USTR);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          acc[2 * xp2] = mfma4x<1>(u0[v], V[2 * xp2][v], acc[2 * xp2], v);
          acc[2 * xp2 + 1] = mfma4x<1>(u1[v], V[2 * xp2 + 1][v], acc[2 * xp2 + 1], v);
        }
      }
      f4 tt[4][2];
#pragma unroll
      for (int ra = 0; ra < 4; ++ra) {
        tt[ra][0] = tadd(tadd(acc[4 * ra], acc[4 * ra + 1]), acc[4 * ra + 2]);
        tt[ra][1] = tsub(tsub(acc[4 * ra + 1], acc[4 * ra + 2]), acc[4 * ra + 3]);
      }
      f4 Y[4];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        Y[c] = tadd(tadd(tt[0][c], tt[1][c]), tt[2][c]);
        Y[2 + c] = tsub(tsub(tt[1][c], tt[2][c]), tt[3][c]);
      }
      const float* xm = x_s + base + 4 * g;
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          const int oy = 2 * ty + dy, ox = 2 * tx + dx;
          if (!valid || !G.in_y(oy) || !G.in_x(ox)) continue;
          const int64_t o = ((static_cast<int64_t>(n) * G.H + oy) * G.W + ox) * C + 4 * g;
          const f4 m = *reinterpret_cast<const f4*>(xm + (dy + 1) * rowstr + (dx + 1) * PP);
          f4 v = Y[2 * dy + dx];
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] = m[k] > 0.f ? v[k] : 0.f;
          v += addv[2 * dy + dx];
          *reinterpret_cast<f4*>(a.out + o) = v;
        }
    }

    if constexpr (WWG) {
      // ---- Winograd weight gradient: waves 4-7, k-step = 4 tiles (lane
      // group g = tile 4 st + g), lane c16 = input channel of V and output
      // channel of Z; acc[4 i + bc] += V[i][bc] (x) Z[i][bc]
      if (wave >= NG) {
        for (int st = wave - NG; st < RT / 4; st += NWG) {
          int base = tile_s[4 * st + kperm(g)];
          const bool valid = base >= 0;
          base = valid ? base : 0;
          const float* dp = d_s + base + rowstr + PP + c16;
          float y00 = dp[0], y01 = dp[PP], y10 = dp[rowstr], y11 = dp[rowstr + PP];
          if (!valid) y00 = y01 = y10 = y11 = 0.f;
          dbacc += (y00 + y01) + (y10 + y11);
          f4 zf[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float r0, r1;
            if (i == 0) { r0 = y00; r1 = y01; }
            else if (i == 1) { r0 = y00 + y10; r1 = y01 + y11; }
            else if (i == 2) { r0 = y00 - y10; r1 = y01 - y11; }
            else { r0 = -y10; r1 = -y11; }
            zf[i] = f4{r0, r0 + r1, r0 - r1, -r1};
          }
          const float* xp = x_s + base + c16;
          float d[4][4];
#pragma unroll
          for (int dy = 0; dy < 4; ++dy)
#pragma unroll
            for (int dx = 0; dx < 4; ++dx) {
              const float v = xp[dy * rowstr + dx * PP];
              d[dy][dx] = RELU ? relu0(v) : v;
            }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float sq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              if (i == 0) sq[q] = d[0][q] - d[2][q];
              else if (i == 1) sq[q] = d[1][q] + d[2][q];
              else if (i == 2) sq[q] = d[2][q] - d[1][q];
              else sq[q] = d[1][q] - d[3][q];
            }
            // an invalid tile's Z is zero: its products vanish without
            // zeroing V (the patch it reads is staged, finite data)
            const float V[4] = {sq[0] - sq[2], sq[1] + sq[2], sq[2] - sq[1], sq[1] - sq[3]};
#pragma unroll
            for (int bc = 0; bc < 4; ++bc)
              wacc[4 * i + bc] = mfma4x<2>(V[bc], zf[i][bc], wacc[4 * i + bc], bc);
          }
        }
      }
    } else {
      // ---- weight gradient: k-step = one tile (lane group g = its pixel g);
      // the operands of four k-steps are loaded before their MFMAs
      constexpr int REST = (RT - 4 * KD) / 4;  // k-steps per wave 4..7
      const int k0 = wave < 4 ? wave * KD : 4 * KD + (wave - 4) * REST;
      const int k1 = wave < 4 ? k0 + KD : k0 + REST;
      const int py = g >> 1, px = g & 1;
      const int poff = c16 + py * rowstr + px * PP;
      for (int kt = k0; kt < k1; kt += 4) {
        int bases[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) bases[u] = kt + u < k1 ? tile_s[kt + u] : -1;
        float bv[4], av[4][9];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int pofs = (bases[u] >= 0 ? bases[u] : 0) + poff;
          bv[u] = bases[u] >= 0 ? d_s[pofs + rowstr + PP] : 0.f;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) av[u][3 * ky + kx] = x_s[pofs + ky * rowstr + kx * PP];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          dbacc += bv[u];
#pragma unroll
          for (int tap = 0; tap < 9; ++tap) {
            const float v = RELU ? relu0(av[u][tap]) : av[u][tap];
            wacc[tap] = mfma4(v, bv[u], wacc[tap]);
          }
        }
      }
    }
    if (r >= rw.end) break;
  }

  if constexpr (WWG) {
    // ---- P = sum of waves 4-7 (fixed order), then dW = G^T P G per
    // (ci, co) into this workgroup's slot (wino_wgrad_kernel's epilogue)
    __syncthreads();
    float* P = smem;                 // [16 xi][C ci][C co]
    float* dB = smem + 16 * C * C;   // [C]
    for (int k = NG; k < NW; ++k) {
      if (wave == k) {
#pragma unroll
        for (int xi = 0; xi < 16; ++xi)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float* pp = P + (xi * C + 4 * g + q) * C + c16;
            *pp = (k == NG ? 0.f : *pp) + wacc[xi][q];
          }
        float v = dbacc;
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        if (g == 0) dB[c16] = (k == NG ? 0.f : dB[c16]) + v;
      }
      __syncthreads();
    }
    float* slot = a.part + static_cast<int64_t>(blockIdx.x) * a.rows16 * C;
    for (int e = threadIdx.x; e < C * C; e += NTH) {
      const int ci = e / C, co = e - (e / C) * C;
      float pm[4][4];
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) pm[xi >> 2][xi & 3] = P[(xi * C + ci) * C + co];
      float t[3][4];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        t[0][b] = pm[0][b] + 0.5f * (pm[1][b] + pm[2][b]);
        t[1][b] = 0.5f * (pm[1][b] - pm[2][b]);
        t[2][b] = 0.5f * (pm[1][b] + pm[2][b]) + pm[3][b];
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        slot[((3 * i + 0) * C + ci) * C + co] = t[i][0] + 0.5f * (t[i][1] + t[i][2]);
        slot[((3 * i + 1) * C + ci) * C + co] = 0.5f * (t[i][1] - t[i][2]);
        slot[((3 * i + 2) * C + ci) * C + co] = 0.5f * (t[i][1] + t[i][2]) + t[i][3];
      }
    }
    for (int co = threadIdx.x; co < C; co += NTH) slot[9 * C * C + co] = dB[co];
    return;
  }

  // ---- weight-gradient partials of the workgroup (fixed wave order)
  __syncthreads();
  float* red = smem;  // [9 * C + 1][C]
  for (int k = 0; k < NW; ++k) {
    if (wave == k) {
      // D[i = ci = 4g + q][j = co = c16]
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float* pp = red + (tap * C + 4 * g + q) * C + c16;
          *pp = (k == 0 ? 0.f : *pp) + wacc[tap][q];
        }
      float v = dbacc;
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (g == 0) {
        float* pb = red + 9 * C * C + c16;
        *pb = (k == 0 ? 0.f : *pb) + v;
      }
    }
    __syncthreads();
  }
  float* slot = a.part + static_cast<int64_t>(blockIdx.x) * a.rows16 * C;
  for (int e = threadIdx.x; e < (9 * C + 1) * C; e += NTH) slot[e] = red[e];
}

// The 32-channel convs (res32 at 18x24 and 9x12, the stage-2 head 32 -> 32)
// and the stage-1 head (16 -> 32 at 36x48): the same single pass with both
// gradients in Winograd form, for x with CX channels and dY with CY.  LDS
// holds U (16 CX CY floats) and the dY / x rows of a 32-tile range (a 64-
// tile range does not fit next to U).  Waves 0-3 run the data gradient,
// waves 4-7 the weight gradient: wave 4 + i owns B^T row i (xi = 4 i ..
// 4 i + 3) for all (ci block, co block) pairs over the range's 8 k-steps.
// Data-gradient tasks are (16-tile group, dX-channel block); with only two
// of them (CX = 16) each is split over a wave pair by dY-channel block, and
// the odd wave hands its partial output transform (A^T M A is linear in M)
// to the even one through LDS (workgroup-scope release/acquire flag).  Each
// wave role runs 64 (CX = 16) or 128 MFMAs per range.  mask_x = 0 (stage
// heads: their input is the previous stage's raw output) skips the ReLU
// mask.  Each workgroup walks a CONTIGUOUS run of ranges, so the halo rows
// a range shares with the previous one come from this CU's L2 instead of
// being refetched by another XCD.
// LDS bytes of the fused32 kernel at a staged-row pitch of Wl pixels, and
// whether a compile-time-geometry instance can afford the padded pitch
// (the 16 -> 32 head at 36x48 cannot: 166 KB)
constexpr size_t fused32_lds(int CX, int CY, int RT, int maxrows, int Wl) {
  return sizeof(float) * (16 * CX * CY + static_cast<size_t>(maxrows) * Wl * (CX + CY + 8)) +
         ((RT / 16) * (CX / 16) == 2 ? sizeof(float) * 2 * 4 * 64 * 4 : 0) +
         sizeof(int) * (2 + maxrows + RT);
}
template <int CX, int CY, int RT, int GH, int GW>
constexpr bool fused32_pad() {
  if constexpr (GH == 0 || !wino_lpad_on(2)) {
    return false;
  } else {
    constexpr int TY = (GH + 1) / 2, TX = (GW + 1) / 2;
    constexpr int maxrows = wino_maxrows(RT, TX, TY);
    return fused32_lds(CX, CY, RT, maxrows, wino_wl<GH>(TX)) <= 160 * 1024;
  }
}

template <int CX, int CY, int RT, int MAXCX, int MAXCY, bool RELU, bool MASK, int GH = 0,
          int GW = 0>
__global__ __launch_bounds__(512, 2) void wino_bwd_fused32_kernel(WinoBwdArgs a) {
  constexpr int NW = 8, NTH = 512;
  const TileGeo<GH, GW, RT, fused32_pad<CX, CY, RT, GH, GW>()> G(a.H, a.W, a.TY, a.TX, a.NT,
                                                                 a.rTX, a.rTY, a.maxrows);
  constexpr int PPX = CX + 4, PPY = CY + 4;  // odd 16-B units per pixel
  constexpr int C4X = CX / 4, C4Y = CY / 4;
  constexpr int LC4X = C4X == 4 ? 2 : 3, LC4Y = C4Y == 4 ? 2 : 3;
  constexpr int NBX = CX / 16, NBY = CY / 16;
  constexpr int NG = RT / 16;
  constexpr int NTASK = NG * NBX;            // (group, dX-channel block)
  constexpr int DSPLIT = 4 / NTASK;          // waves per task (dY blocks)
  constexpr int NBT = NBY / DSPLIT;          // dY blocks per wave
  constexpr int USTR = NBY * 4 * CX * 4;     // floats per xi in U_s
  static_assert(NTASK * DSPLIT == 4 && NBT * DSPLIT == NBY, "four data-gradient waves");
  static_assert(C4X == 4 || C4X == 8, "CX");
  static_assert(C4Y == 4 || C4Y == 8, "CY");
  static_assert(MAXCX <= 32 && MAXCY <= 32, "stager masks");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Wl = G.WL;
  const int rsx = Wl * PPX, rsy = Wl * PPY;
  float* U_s = smem;                         // [16 xi][NBY][4 g][CX][4]
  float* d_s = U_s + 16 * CX * CY;           // dY rows [maxrows][Wl][PPY]
  float* x_s = d_s + G.maxrows * rsy;        // x rows [maxrows][Wl][PPX]
  f4* ybuf = reinterpret_cast<f4*>(x_s + G.maxrows * rsx);  // [2 pairs][4][64] (DSPLIT 2)
  int* flag_s = reinterpret_cast<int*>(ybuf + (DSPLIT == 2 ? 2 * 4 * 64 : 0));  // [2]
  int* tab_s = flag_s + 2;                   // [maxrows]
  int* tile_s = tab_s + G.maxrows;           // [RT] patch-origin pixel (row * Wl + col)

  // U = G g' G^T of the flipped / transposed weights (the dgrad conv);
  // forward weights HWIO [3][3][CX][CY]
  for (int e = threadIdx.x; e < CX * CY; e += NTH) {
    const int co = e % CX, ci = e / CX;  // ci = dY channel, co = dX channel
    float gk[3][3];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) gk[ky][kx] = a.w[(((2 - ky) * 3 + (2 - kx)) * CX + co) * CY + ci];
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
        U_s[(4 * ra + rb) * USTR + ((b * 4 + gq) * CX + co) * 4 + v] = u[rb];
    }
  }
  if (threadIdx.x < 2) flag_s[threadIdx.x] = 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;

  // this workgroup's contiguous run of ranges (G <= nranges: never empty)
  const int r_end = static_cast<int>((static_cast<int64_t>(blockIdx.x) + 1) * a.nranges / gridDim.x);
  int r = static_cast<int>(static_cast<int64_t>(blockIdx.x) * a.nranges / gridDim.x);
  if (r >= r_end) return;
  {
    const int w0 = __builtin_amdgcn_readfirstlane(wave);
    if ((a.prio == 1 && w0 >= NW / 2) || (a.prio == 2 && w0 < NW / 2)) __builtin_amdgcn_s_setprio(1);
  }

  // staging slots: element e = (row L, col, quad) of the dY image and of x
  int sy_L[MAXCY], sy_o[MAXCY], sx_L[MAXCX], sx_o[MAXCX];
#pragma unroll
  for (int k = 0; k < MAXCY; ++k) {
    const int e = threadIdx.x + k * NTH;
    const int ch = e & (C4Y - 1), pix = e >> LC4Y;
    const int L = pix / G.WL0, col = pix - L * G.WL0;
    sy_L[k] = L < G.maxrows ? L : -1;
    sy_o[k] = (col >= 1 && col <= G.W) ? (col - 1) * CY + 4 * ch : -1;
  }
#pragma unroll
  for (int k = 0; k < MAXCX; ++k) {
    const int e = threadIdx.x + k * NTH;
    const int ch = e & (C4X - 1), pix = e >> LC4X;
    const int L = pix / G.WL0, col = pix - L * G.WL0;
    sx_L[k] = L < G.maxrows ? L : -1;
    sx_o[k] = (col >= 1 && col <= G.W) ? (col - 1) * CX + 4 * ch : -1;
  }
  // row table: global PIXEL index (n H + y) W of LDS row L, or -1
  auto build_tab = [&](int rr) __attribute__((always_inline)) {
    const RangeGeom gm = G.range(rr);
    const int L = threadIdx.x;
    if (L < G.maxrows) {
      int v = -1;
      if (L < gm.rows) {
        const int p = G.part_of(gm, L);
        const int offp = G.part_off(gm, p);
        const int y = 2 * (p == 0 ? gm.tya0 : 0) - 1 + (L - offp);
        if (y >= 0 && y < G.H) v = ((gm.n0 + p) * G.H + y) * G.W;
      }
      tab_s[L] = v;
    }
  };
  f4 sy[MAXCY], sx[MAXCX];
  const int64_t npx = static_cast<int64_t>(a.N) * G.H * G.W;
  const auto dyr = buf_rsrc(a.dy, npx * CY), xr = buf_rsrc(a.x, npx * CX);
  auto prefetch = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < MAXCY; ++k) {
      const int rb = sy_L[k] >= 0 ? tab_s[sy_L[k]] : -1;
      const bool in = rb >= 0 && sy_o[k] >= 0 && !knob(a.ablate, 8);
      sy[k] = bload(dyr, in ? static_cast<uint32_t>(rb * CY + sy_o[k]) * 4u : kOOB);
    }
#pragma unroll
    for (int k = 0; k < MAXCX; ++k) {
      const int rb = sx_L[k] >= 0 ? tab_s[sx_L[k]] : -1;
      const bool in = rb >= 0 && sx_o[k] >= 0;
      sx[k] = bload(xr, in ? static_cast<uint32_t>(rb * CX + sx_o[k]) * 4u : kOOB);
    }
  };
  build_tab(r);
  __syncthreads();
  prefetch();

  // Commit the prefetched range to LDS, build its tile table and the next
  // range's row table, start the next prefetch.  Both wave roles run it
  // once per range (same barrier count); the roles are separate loops so
  // the weight-gradient accumulators are not live in the data-gradient
  // code (one loop with both would need > 256 VGPRs).
  auto advance = [&]() __attribute__((always_inline)) {
    __syncthreads();  // U_s written / the previous range's LDS reads are done
#pragma unroll
    for (int k = 0; k < MAXCY; ++k) {
      if (sy_L[k] >= 0) {
        const int e = threadIdx.x + k * NTH;
        const f4 v = sy[k];  // zero where out of the image
        *reinterpret_cast<f4*>(d_s + ((e >> LC4Y) + pad_pix<decltype(G)::PADC>(sy_L[k])) * PPY + 4 * (e & (C4Y - 1))) = v;
      }
    }
#pragma unroll
    for (int k = 0; k < MAXCX; ++k) {
      if (sx_L[k] >= 0) {
        const int e = threadIdx.x + k * NTH;
        const f4 v = sx[k];  // zero where out of the image
        *reinterpret_cast<f4*>(x_s + ((e >> LC4X) + pad_pix<decltype(G)::PADC>(sx_L[k])) * PPX + 4 * (e & (C4X - 1))) = v;
      }
    }
    const int cur = r;
    ++r;
    const RangeGeom gm = G.range(cur);
    if (threadIdx.x < RT) {
      const int t = gm.t0 + threadIdx.x;
      int v = -1;
      if (t < gm.t1) {
        const int R = G.div_tx(t), tx = t - R * G.TX;
        const int n = G.div_ty(R), ty = R - n * G.TY;
        const int p = n - gm.n0;
        const int offp = G.part_off(gm, p);
        v = (offp + 2 * (ty - (p == 0 ? gm.tya0 : 0))) * Wl + 2 * tx;
      }
      tile_s[threadIdx.x] = v;
    }
    build_tab(r < r_end ? r : cur);  // unconditional: see wino_conv_kernel
    __syncthreads();
    prefetch();  // in flight under the MFMAs below
    return gm;
  };

  const int wv = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform role
  if (wv < 4) {
    // ---- data gradient: task = (16-tile group grp, dX-channel block cb),
    // this wave's dY blocks [yb0, yb0 + NBT)
    const int task = wv / DSPLIT, half = wv % DSPLIT;
    const int grp = task % NG, cb = task / NG;
    const int yb0 = half * NBT;
    int it = 0;
    for (;;) {
      const RangeGeom gm = advance();
      ++it;
      if (gm.t0 + 16 * grp < gm.t1 && !knob(a.ablate, 2)) {
        int t = gm.t0 + 16 * grp + c16;
        const bool valid = t < gm.t1;
        if (!valid) t = gm.t0;
        const int R = G.div_tx(t), tx = t - R * G.TX;
        const int n = G.div_ty(R), ty = R - n * G.TY;
        const int bpx = tile_s[valid ? 16 * grp + c16 : 0];
        const int co = 16 * cb + 4 * g;  // this lane's 4 dX channels
        f4 addv[4];
        if (half == 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int oy = 2 * ty + (q >> 1), ox = 2 * tx + (q & 1);
            const bool in = a.add != nullptr && valid && G.in_y(oy) && G.in_x(ox);
            const int64_t o = in ? ((static_cast<int64_t>(n) * G.H + oy) * G.W + ox) * CX + co : 0;
            addv[q] = in ? *reinterpret_cast<const f4*>(a.add + o) : f4{0.f, 0.f, 0.f, 0.f};
          }
        }
        f4 acc[16];
#pragma unroll
        for (int xi = 0; xi < 16; ++xi) acc[xi] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int bb = 0; bb < NBT; ++bb) {
          const int b = yb0 + bb;
          const float* dp = d_s + bpx * PPY + 16 * b + 4 * g;
          f4 d[16];
#pragma unroll
          for (int dy = 0; dy < 4; ++dy)
#pragma unroll
            for (int dx = 0; dx < 4; ++dx)
              d[4 * dy + dx] = *reinterpret_cast<const f4*>(dp + dy * rsy + dx * PPY);
          f4 sv[16];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            sv[q] = tsub(d[q], d[8 + q]);
            sv[4 + q] = tadd(d[4 + q], d[8 + q]);
            sv[8 + q] = tsub(d[8 + q], d[4 + q]);
            sv[12 + q] = tsub(d[4 + q], d[12 + q]);
          }
          f4 V[16];
#pragma unroll
          for (int ra = 0; ra < 4; ++ra) {
            V[4 * ra + 0] = tsub(sv[4 * ra + 0], sv[4 * ra + 2]);
            V[4 * ra + 1] = tadd(sv[4 * ra + 1], sv[4 * ra + 2]);
            V[4 * ra + 2] = tsub(sv[4 * ra + 2], sv[4 * ra + 1]);
            V[4 * ra + 3] = tsub(sv[4 * ra + 1], sv[4 * ra + 3]);
          }
          const float* up = U_s + ((b * 4 + g) * CX + 16 * cb + c16) * 4;
#pragma unroll
          for (int xp2 = 0; xp2 < 8; ++xp2) {
            const f4 u0 = *reinterpret_cast<const f4*>(up + (2 * xp2) * USTR);
            const f4 u1 = *reinterpret_cast<const f4*>(up + (2 * xp2 + 1) * USTR);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              acc[2 * xp2] = mfma4x<1>(u0[v], V[2 * xp2][v], acc[2 * xp2], v);
              acc[2 * xp2 + 1] = mfma4x<1>(u1[v], V[2 * xp2 + 1][v], acc[2 * xp2 + 1], v);
            }
          }
        }
        f4 tt[4][2];
#pragma unroll
        for (int ra = 0; ra < 4; ++ra) {
          tt[ra][0] = tadd(tadd(acc[4 * ra], acc[4 * ra + 1]), acc[4 * ra + 2]);
          tt[ra][1] = tsub(tsub(acc[4 * ra + 1], acc[4 * ra + 2]), acc[4 * ra + 3]);
        }
        f4 Y[4];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          Y[c] = tadd(tadd(tt[0][c], tt[1][c]), tt[2][c]);
          Y[2 + c] = tsub(tsub(tt[1][c], tt[2][c]), tt[3][c]);
        }
        if constexpr (DSPLIT == 2) {
          f4* yb = ybuf + task * 4 * 64 + lane;
          if (half == 1) {
            // hand the partial Y to the even wave of the pair
#pragma unroll
            for (int q = 0; q < 4; ++q) yb[q * 64] = Y[q];
            __hip_atomic_store(flag_s + task, it, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          } else {
            // bounded wait (~30 ms): the partner wave always publishes
            // (same task, same group condition), but a kernel must never be
            // able to spin forever.  A wait that expires fails LOUD: the
            // sticky error word makes the RMSProp guard skip this step's
            // update and count it (learner health 'conv_timeouts'), instead
            // of adding a stale partial into dX.
            bool got = false;
            if (!a.fault) {
              for (int spin = 0; spin < (1 << 20); ++spin) {
                if (__hip_atomic_load(flag_s + task, __ATOMIC_ACQUIRE,
                                      __HIP_MEMORY_SCOPE_WORKGROUP) == it) {
                  got = true;
                  break;
                }
                __builtin_amdgcn_s_sleep(1);
              }
            }
            if (got) {
#pragma unroll
              for (int q = 0; q < 4; ++q) Y[q] += yb[q * 64];
            } else {
              __hip_atomic_store((gu32*)(a.err), 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
            }
          }
        }
        if (half == 0) {
          const float* xm = x_s + bpx * PPX + co;
#pragma unroll
          for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) {
              const int oy = 2 * ty + dy, ox = 2 * tx + dx;
              if (!valid || !G.in_y(oy) || !G.in_x(ox)) continue;
              const int64_t o = ((static_cast<int64_t>(n) * G.H + oy) * G.W + ox) * CX + co;
              f4 v = Y[2 * dy + dx];
              if constexpr (MASK) {
                const f4 m = *reinterpret_cast<const f4*>(xm + (dy + 1) * rsx + (dx + 1) * PPX);
#pragma unroll
                for (int k = 0; k < 4; ++k) v[k] = m[k] > 0.f ? v[k] : 0.f;
              }
              v += addv[2 * dy + dx];
              *reinterpret_cast<f4*>(a.out + o) = v;
            }
        }
      }
      if (r >= r_end) break;
    }
    __syncthreads();  // the loop's LDS reads are done (P overwrites U)
    __syncthreads();  // P written by waves 4-7
  } else {
    // ---- Winograd weight gradient, B^T row AR of this wave: k-step = 4
    // tiles (lane group g = tile 4 st + g); lane c16 = input channel of V
    // and output channel of Z within their 16-channel blocks
    f4 wacc[4][NBX][NBY];  // [bc][x block][dY block]
#pragma unroll
    for (int bc = 0; bc < 4; ++bc)
#pragma unroll
      for (int b = 0; b < NBX; ++b)
#pragma unroll
        for (int b2 = 0; b2 < NBY; ++b2) wacc[bc][b][b2] = f4{0.f, 0.f, 0.f, 0.f};
    float dbacc[NBY];
#pragma unroll
    for (int b2 = 0; b2 < NBY; ++b2) dbacc[b2] = 0.f;
    // FULL: every tile of the range exists (all ranges but the batch's
    // last) - no per-tile validity selects in the k-step loop
    auto kloop = [&](auto ARc, auto FULLc) __attribute__((always_inline)) {
      constexpr int AR = decltype(ARc)::value;
      constexpr bool FULL = decltype(FULLc)::value;
        for (int st = 0; st < (knob(a.ablate, 4) ? 0 : RT / 4); ++st) {
          int bpx = tile_s[4 * st + kperm(g)];
          const bool valid = FULL || bpx >= 0;
          bpx = valid ? bpx : 0;
          f4 zf[NBY];
#pragma unroll
          for (int b2 = 0; b2 < NBY; ++b2) {
            const float* dp = d_s + bpx * PPY + rsy + PPY + 16 * b2 + c16;
            float y00 = dp[0], y01 = dp[PPY], y10 = dp[rsy], y11 = dp[rsy + PPY];
            if (!FULL && !valid) y00 = y01 = y10 = y11 = 0.f;
            if constexpr (AR == 0) dbacc[b2] += (y00 + y01) + (y10 + y11);
            float r0, r1;
            if constexpr (AR == 0) { r0 = y00; r1 = y01; }
            else if constexpr (AR == 1) { r0 = y00 + y10; r1 = y01 + y11; }
            else if constexpr (AR == 2) { r0 = y00 - y10; r1 = y01 - y11; }
            else { r0 = -y10; r1 = -y11; }
            zf[b2] = f4{r0, r0 + r1, r0 - r1, -r1};
          }
#pragma unroll
          for (int b = 0; b < NBX; ++b) {
            const float* xp = x_s + bpx * PPX + 16 * b + c16;
            // the two patch rows B^T row AR combines
            constexpr int RA = AR == 0 ? 0 : 1;
            constexpr int RB = AR == 3 ? 3 : 2;
            float ra[4], rb[4];
#pragma unroll
            for (int dx = 0; dx < 4; ++dx) {
              float u = xp[RA * rsx + dx * PPX], w = xp[RB * rsx + dx * PPX];
              if constexpr (RELU) {
                u = relu0(u);
                w = relu0(w);
              }
              ra[dx] = u;
              rb[dx] = w;
            }
            float sq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              if constexpr (AR == 0) sq[q] = ra[q] - rb[q];       // d0 - d2
              else if constexpr (AR == 1) sq[q] = ra[q] + rb[q];  // d1 + d2
              else if constexpr (AR == 2) sq[q] = rb[q] - ra[q];  // d2 - d1
              else sq[q] = ra[q] - rb[q];                          // d1 - d3
            }
            const float V[4] = {sq[0] - sq[2], sq[1] + sq[2], sq[2] - sq[1], sq[1] - sq[3]};
#pragma unroll
            for (int bc = 0; bc < 4; ++bc)
#pragma unroll
              for (int b2 = 0; b2 < NBY; ++b2)
                wacc[bc][b][b2] = mfma4x<2>(V[bc], zf[b2][bc], wacc[bc][b][b2], bc);
          }
        }
    };
    auto run = [&](auto ARc) __attribute__((always_inline)) {
      for (;;) {
        const RangeGeom gm = advance();
        // a FULL (selects-free) copy for whole ranges measured slower: 16->32
        // 851 -> 942 us (second loop copy; 21 spills in the 32-channel one)
        (void)gm;
        kloop(ARc, std::false_type{});
        if (r >= r_end) break;
      }
    };
    if (wv == 4) run(std::integral_constant<int, 0>{});
    else if (wv == 5) run(std::integral_constant<int, 1>{});
    else if (wv == 6) run(std::integral_constant<int, 2>{});
    else run(std::integral_constant<int, 3>{});

    // ---- P[xi][ci][co] (disjoint xi rows per wave); dW = G^T P G below
    __syncthreads();  // the loop's LDS reads are done (P overwrites U)
    float* P = smem;                   // [16 xi][CX ci][CY co]
    float* dB = smem + 16 * CX * CY;   // [CY]
    const int ar = wv - 4;
#pragma unroll
    for (int bc = 0; bc < 4; ++bc)
#pragma unroll
      for (int b = 0; b < NBX; ++b)
#pragma unroll
        for (int b2 = 0; b2 < NBY; ++b2)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            P[((4 * ar + bc) * CX + 16 * b + 4 * g + q) * CY + 16 * b2 + c16] = wacc[bc][b][b2][q];
    if (ar == 0) {
#pragma unroll
      for (int b2 = 0; b2 < NBY; ++b2) {
        float v = dbacc[b2];
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        if (g == 0) dB[16 * b2 + c16] = v;
      }
    }
    __syncthreads();
  }
  // per (ci, co) into this workgroup's slot (wino_wgrad_kernel's epilogue)
  const float* P = smem;
  const float* dB = smem + 16 * CX * CY;
  float* slot = a.part + static_cast<int64_t>(blockIdx.x) * a.rows16 * CY;
  for (int e = threadIdx.x; e < CX * CY; e += NTH) {
    const int ci = e / CY, co = e - (e / CY) * CY;
    float pm[4][4];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) pm[xi >> 2][xi & 3] = P[(xi * CX + ci) * CY + co];
    float t[3][4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      t[0][b] = pm[0][b] + 0.5f * (pm[1][b] + pm[2][b]);
      t[1][b] = 0.5f * (pm[1][b] - pm[2][b]);
      t[2][b] = 0.5f * (pm[1][b] + pm[2][b]) + pm[3][b];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      slot[((3 * i + 0) * CX + ci) * CY + co] = t[i][0] + 0.5f * (t[i][1] + t[i][2]);
      slot[((3 * i + 1) * CX + ci) * CY + co] = 0.5f * (t[i][1] - t[i][2]);
      slot[((3 * i + 2) * CX + ci) * CY + co] = 0.5f * (t[i][1] + t[i][2]) + t[i][3];
    }
  }
  for (int co = threadIdx.x; co < CY; co += NTH) slot[9 * CX * CY + co] = dB[co];
}

template <int CX, int CY, int RT, int MAXCX, int MAXCY, bool RELU, bool MASK, int GH = 0,
          int GW = 0>
bool run_wino_bwd32_g(const float* dy, const float* w, const float* x, const float* add,
                      float* out, int relu_x, int mask_x, int N, int H, int W, float* ws,
                      int64_t ws_floats, float* dw, float* db, hipStream_t s) {
  if (GH > 0 && (H != GH || W != GW)) return false;
  const int TY = (H + 1) / 2, TX = (W + 1) / 2;
  const int64_t NT = static_cast<int64_t>(N) * TY * TX;
  if (NT >= (1 << 22) || TX > 1024 || TY > 1024) return false;
  if (static_cast<int64_t>(N) * H * W * CY * 4 > kMaxBufBytes) return false;
  const int per_img = TY * TX;
  const int maxparts = (RT - 1 + per_img - 1) / per_img + 1;
  if (maxparts > kMaxParts) return false;
  const int Wl = 2 * TX + 2;
  const int WlP = wino_wl<GH, fused32_pad<CX, CY, RT, GH, GW>()>(TX);
  const int maxrows = wino_maxrows(RT, TX, TY);
  if (maxrows * Wl * (CY / 4) > MAXCY * 512 || maxrows * Wl * (CX / 4) > MAXCX * 512 ||
      maxrows > 512)
    return false;
  const size_t bytes = fused32_lds(CX, CY, RT, maxrows, WlP);
  if (bytes > 160 * 1024) return false;
  const int rows16 = ((9 * CX + 16) / 16) * 16;
  const int nranges = static_cast<int>((NT + RT - 1) / RT);
  const int64_t cap = ws_floats / (static_cast<int64_t>(rows16) * CY);
  const int G = static_cast<int>(std::min<int64_t>({nranges, conv_cus(), cap}));
  if (G < 1) return false;
  WinoBwdArgs a{};
  a.dy = dy; a.w = w; a.x = x; a.add = add; a.out = out; a.part = ws;
  a.N = N; a.H = H; a.W = W;
  a.TY = TY; a.TX = TX; a.NT = static_cast<int>(NT); a.nranges = nranges;
  a.maxrows = maxrows; a.rows16 = rows16;
  a.rTX = 1.f / static_cast<float>(TX);
  a.rTY = 1.f / static_cast<float>(TY);
  a.relu_x = relu_x;
  a.mask_x = mask_x;
  static const int ablate = measure_knob("SA_FUSED_ABLATE", 0);
  a.ablate = ablate;
  a.err = device_error_words() + 1;
  a.fault = g_wino_fault;
  static const int fprio = measure_knob("SA_FUSED_PRIO", 0);
  a.prio = fprio;
  auto kern = wino_bwd_fused32_kernel<CX, CY, RT, MAXCX, MAXCY, RELU, MASK, GH, GW>;
  allow_lds_w(kern, bytes);
  hipLaunchKernelGGL(kern, dim3(G), dim3(512), bytes, s, a);
  wgrad_reduce_slots(ws, G, rows16, CY, CX, dw, db, s);
  return true;
}

template <int CX, int CY, int RT, int MAXCX, int MAXCY, bool RELU, bool MASK>
bool run_wino_bwd32_t(const float* dy, const float* w, const float* x, const float* add,
                      float* out, int relu_x, int mask_x, int N, int H, int W, float* ws,
                      int64_t ws_floats, float* dw, float* db, hipStream_t s) {
  // the residual convs (MASK, with or without the ReLU'd operand) and the
  // stage heads (neither); the relu-without-mask form is never called
  if constexpr (MASK || !RELU) {
    const int HH = H, WW = W;
#define SA_CALL(h, w_)                                                                     \
  run_wino_bwd32_g<CX, CY, RT, MAXCX, MAXCY, RELU, MASK, h, w_>(dy, w, x, add, out, relu_x, \
                                                                mask_x, N, H, W, ws,        \
                                                                ws_floats, dw, db, s)
    if constexpr (CX == 32 || !MASK) { SA_WINO_GEO_DISPATCH(CX, CY, 4) }
#undef SA_CALL
  }
  return run_wino_bwd32_g<CX, CY, RT, MAXCX, MAXCY, RELU, MASK>(
      dy, w, x, add, out, relu_x, mask_x, N, H, W, ws, ws_floats, dw, db, s);
}

// relu_x / mask_x are compile-time in the kernel (the wgrad waves' ReLU on
// every x operand was a select per value); the residual convs use (1, 1)
// and (0, 1), the stage heads (0, 0)
template <int CX, int CY, int RT, int MAXCX, int MAXCY>
bool run_wino_bwd32(const float* dy, const float* w, const float* x, const float* add,
                    float* out, int relu_x, int mask_x, int N, int H, int W, float* ws,
                    int64_t ws_floats, float* dw, float* db, hipStream_t s) {
  if (relu_x && mask_x)
    return run_wino_bwd32_t<CX, CY, RT, MAXCX, MAXCY, true, true>(
        dy, w, x, add, out, relu_x, mask_x, N, H, W, ws, ws_floats, dw, db, s);
  if (mask_x)
    return run_wino_bwd32_t<CX, CY, RT, MAXCX, MAXCY, false, true>(
        dy, w, x, add, out, relu_x, mask_x, N, H, W, ws, ws_floats, dw, db, s);
  if (relu_x)
    return run_wino_bwd32_t<CX, CY, RT, MAXCX, MAXCY, true, false>(
        dy, w, x, add, out, relu_x, mask_x, N, H, W, ws, ws_floats, dw, db, s);
  return run_wino_bwd32_t<CX, CY, RT, MAXCX, MAXCY, false, false>(
      dy, w, x, add, out, relu_x, mask_x, N, H, W, ws, ws_floats, dw, db, s);
}

template <int C, int RT, int MAXC, int KD, bool WWG = false, int NW = 8, int GH = 0, int GW = 0>
bool run_wino_bwd_g(const float* dy, const float* w, const float* x, const float* add,
                    float* out, int relu_x, int N, int H, int W, float* ws, int64_t ws_floats,
                    float* dw, float* db, hipStream_t s) {
  if (GH > 0 && (H != GH || W != GW)) return false;
  const int TY = (H + 1) / 2, TX = (W + 1) / 2;
  const int64_t NT = static_cast<int64_t>(N) * TY * TX;
  if (NT >= (1 << 22) || TX > 1024 || TY > 1024) return false;
  if (static_cast<int64_t>(N) * H * W * C * 4 > kMaxBufBytes) return false;
  const int per_img = TY * TX;
  const int maxparts = (RT - 1 + per_img - 1) / per_img + 1;
  if (maxparts > kMaxParts) return false;
  const int Wl = 2 * TX + 2, WlP = wino_wl<GH, wino_lpad_on(1)>(TX);
  const int maxrows = wino_maxrows(RT, TX, TY);
  if (maxrows * Wl * (C / 4) > MAXC * 64 * NW || maxrows > 64 * NW) return false;
  const size_t bytes = sizeof(float) * (16 * C * C + 2 * static_cast<size_t>(maxrows) * WlP * (C + 4)) +
                       sizeof(int) * (maxrows + RT);
  if (bytes > 160 * 1024) return false;
  const int rows16 = ((9 * C + 16) / 16) * 16;
  const int nranges = static_cast<int>((NT + RT - 1) / RT);
  const int64_t cap = ws_floats / (static_cast<int64_t>(rows16) * C);
  const int G = static_cast<int>(std::min<int64_t>({nranges, conv_cus(), cap}));
  if (G < 1) return false;
  WinoBwdArgs a{};
  a.dy = dy; a.w = w; a.x = x; a.add = add; a.out = out; a.part = ws;
  a.N = N; a.H = H; a.W = W;
  a.TY = TY; a.TX = TX; a.NT = static_cast<int>(NT); a.nranges = nranges;
  a.maxrows = maxrows; a.rows16 = rows16;
  a.rTX = 1.f / static_cast<float>(TX);
  a.rTY = 1.f / static_cast<float>(TY);
  a.relu_x = relu_x;
  static const int runs = measure_knob("SA_WINO_RUNS", 1);
  a.runs = runs;
  static const int fprio = measure_knob("SA_FUSED_PRIO", 0);
  a.prio = fprio;
  auto kern = relu_x ? wino_bwd_fused_kernel<C, RT, MAXC, KD, WWG, true, NW, GH, GW>
                     : wino_bwd_fused_kernel<C, RT, MAXC, KD, WWG, false, NW, GH, GW>;
  allow_lds_w(kern, bytes);
  hipLaunchKernelGGL(kern, dim3(G), dim3(64 * NW), bytes, s, a);
  wgrad_reduce_slots(ws, G, rows16, C, C, dw, db, s);
  return true;
}

// runtime geometry (the opt-in variants) / compile-time where the map has an
// instance (the default WWG kernel)
template <int C, int RT, int MAXC, int KD, bool WWG = false, int NW = 8>
bool run_wino_bwd(const float* dy, const float* w, const float* x, const float* add,
                  float* out, int relu_x, int N, int H, int W, float* ws, int64_t ws_floats,
                  float* dw, float* db, hipStream_t s) {
  if constexpr (WWG) {
    const int HH = H, WW = W;
#define SA_CALL(h, w_)                                                                  \
  run_wino_bwd_g<C, RT, MAXC, KD, WWG, NW, h, w_>(dy, w, x, add, out, relu_x, N, H, W, ws, \
                                                  ws_floats, dw, db, s)
    SA_WINO_GEO_DISPATCH(C, C, 2)
#undef SA_CALL
  }
  return run_wino_bwd_g<C, RT, MAXC, KD, WWG, NW>(dy, w, x, add, out, relu_x, N, H, W, ws,
                                                  ws_floats, dw, db, s);
}

}  // namespace

int conv_wino_fault(int v) {
  const int old = g_wino_fault;
  if (v == 0 || v == 1) g_wino_fault = v;
  return old;
}

int conv_wino_geo(int v) {
  const int old = wino_geo_enabled() ? 1 : 0;
  if (v == 0 || v == 1) g_wino_geo = v;
  return old;
}

bool wino_enabled() {
  static const bool on = env_knob("SA_F32_WINO", 1) != 0;
  return on;
}

int64_t wino_conv_pool_side_floats(int W, int Cout) {
  return int64_t{256} * 8 * (W / 2) * (Cout / 4) * 5;  // up to 8 workgroups per CU
}

bool wino_conv_pool_launch(const float* x, const float* w, const float* b, float* pooled,
                           uint8_t* arg, float* side, int64_t side_floats, int N, int H, int W,
                           int Cin, int Cout, int stages, hipStream_t s) {
  // bit 0: stage 1, bit 1: stage 0 (stage 0: 412 vs 529 us for the direct
  // conv+pool, 10.02 -> 9.93 ms per step), bit 2: stage 2 (whole-image
  // ranges: 9.93 -> 9.90 ms), bit 3: the 42-wide stage-1 head (opt-in);
  // stages >= 0 overrides the environment (tests)
  static const int env_on = env_knob("SA_F32_WINO_POOL", 7);
  const int on = stages >= 0 ? stages : env_on;
  if (Cin == 16 && Cout == 32 && (on & 1)) {
    if (W == 48) return run_wino_pool<16, 32, 48>(x, w, b, pooled, arg, side, side_floats, N, H, W, s);
    if (W == 32) return run_wino_pool<16, 32, 32>(x, w, b, pooled, arg, side, side_floats, N, H, W, s);
    if (W == 64) return run_wino_pool<16, 32, 64>(x, w, b, pooled, arg, side, side_floats, N, H, W, s);
    // the Atari stage-1 map (42x42: 21 tile rows, a one-row last range) -
    // opt-in (bit 3): fp32 Atari step 10.04-10.07 (conv + maxpool_fwd) vs
    // 10.07-10.09 ms fused (42 tiles fill 3 groups of 16, 2 workgroups per CU)
    if (W == 42 && (on & 8))
      return run_wino_pool<16, 32, 42>(x, w, b, pooled, arg, side, side_floats, N, H, W, s);
  }
  if (Cin == 32 && Cout == 32 && (on & 4) && H == 18 && W == 24)
    return run_wino_pool_img<32, 32, 18, 24>(x, w, b, pooled, arg, N, H, W, s);
  if (Cin == 4 && Cout == 16 && (on & 2)) {
    if (W == 96) return run_wino_pool<4, 16, 96>(x, w, b, pooled, arg, side, side_floats, N, H, W, s);
    if (W == 64) return run_wino_pool<4, 16, 64>(x, w, b, pooled, arg, side, side_floats, N, H, W, s);
    // the 72x128 Doom frame (Sample Factory's doom_benchmark resolution)
    if (W == 128) return run_wino_pool<4, 16, 128>(x, w, b, pooled, arg, side, side_floats, N, H, W, s);
    // the Atari frame (BASELINE config #2): 84 tiles per range in 6 groups
    if (W == 84) return run_wino_pool<4, 16, 84>(x, w, b, pooled, arg, side, side_floats, N, H, W, s);
  }
  return false;
}

bool wino_conv_launch(const ConvArgs& c, bool flip, hipStream_t s) {
  // 3x3 / stride 1 / SAME, fp32 source, output = source dims, plain
  // placement (no phase / strided output, no pool-gradient source)
  if (c.D != 1 || c.pt != 1 || c.pl != 1 || c.Hs != c.Ho || c.Ws != c.Wo ||
      c.ostr > 0 || c.phase_c > 0 || c.pool.arg != nullptr)
    return false;
  const int cin = c.Cs, cout = c.Cout;
  // SA_WINO_CFG: alternative instances for measurement sweeps
  static const int cfg = measure_knob("SA_WINO_CFG", 0);
  if (cin == 16 && cout == 16) {
    // 3-wave workgroups over 48-tile ranges: at 36x48 every range is two
    // whole tile rows of one image (6 staged rows, 40 KB of LDS), so four
    // workgroups (three waves per SIMD) fit on a CU
    // SA_WINO_CFG=3: 8 waves over 128-tile ranges (one workgroup per CU)
    if (cfg == 3 && run_wino<16, 16, 1, 8, 128, 7, 2>(c, flip, s)) return true;
    static const int w3 = measure_knob("SA_WINO16_3W", 0);
    if (w3 && !flip) {
      const int fl = (c.relu_in ? 1 : 0) | (c.relu_out ? 2 : 0) | (c.mask ? 4 : 0) |
                     (c.add ? 8 : 0) | (c.bias ? 16 : 0);
      if (fl == 19 && run_wino<16, 16, 1, 3, 48, 7, 3, 19>(c, flip, s)) return true;
      if (fl == 24 && run_wino<16, 16, 1, 3, 48, 7, 3, 24>(c, flip, s)) return true;
    }
    return run_wino_fl<16, 16, 1, 4, 64, 10, 2>(c, flip, s);
  }
  if (cin == 16 && cout == 32) {
    if (cfg == 1) return run_wino<16, 32, 2, 4, 64, 10, 1>(c, flip, s);
    return run_wino_fl<16, 32, 1, 8, 64, 5, 2>(c, flip, s);
  }
  // 32 -> 16 (the stage-1 head's data gradient at 36x48): one workgroup of
  // four waves per CU (LDS) measured slower than the direct kernel
  // (674 vs 583 us), so it stays opt-in
  if (cin == 32 && cout == 16 && cfg == 2) return run_wino<32, 16, 1, 4, 64, 19, 1>(c, flip, s);
  if (cin == 32 && cout == 32) {
    if (cfg == 1) return run_wino<32, 32, 2, 4, 64, 15, 1>(c, flip, s);
    return run_wino_fl<32, 32, 1, 8, 64, 8, 2>(c, flip, s);
  }
  return false;
}

}  // namespace cf32
}  // namespace sa

namespace sa {
namespace cf32 {

bool wino_wgrad_enabled() {
  static const bool on = measure_knob("SA_F32_WINO_WG", 1) != 0;
  return on;
}

bool wino_wgrad_launch(const WgradArgs& c, float* ws, hipStream_t s) {
  if (c.pool.arg != nullptr || c.pt != 1 || c.pl != 1 || c.Ho != c.H || c.Wo != c.W)
    return false;
  const int cin = c.Cin, cout = c.Cout;
  // 16-channel inputs measured slower than the direct MFMA wgrad (res16
  // 449 vs 369-387 us, the stage-1 head 720 vs 623-631 us: one workgroup of
  // four waves per CU, VALU-heavy per MFMA); opt-in for sweeps
  static const int all = measure_knob("SA_WINO_WG_ALL", 0);
  if (all && cin == 16 && cout == 16) return run_wino_wgrad<16, 16, 4, 64, 10, 9>(c, ws, s);
  if (all && cin == 16 && cout == 32) return run_wino_wgrad<16, 32, 2, 64, 10, 19>(c, ws, s);
  if (cin == 32 && cout == 32) return run_wino_wgrad<32, 32, 1, 64, 15, 14>(c, ws, s);
  return false;
}

}  // namespace cf32
}  // namespace sa

namespace sa {
namespace cf32 {

bool wino_bwd_fused_enabled() {
  static const bool on = env_knob("SA_F32_FUSED_BWD", 1) != 0;
  return on;
}

bool wino_bwd_fused_launch(const float* dy, const float* w, const float* x, const float* add,
                           float* out, int relu_x, int mask_x, int N, int H, int W, int C,
                           int Cy, float* ws, int64_t ws_floats, float* dw, float* db,
                           hipStream_t s) {
  static const int kd = measure_knob("SA_FUSED_BWD_KD", 4);
  static const int wwg = measure_knob("SA_FUSED_BWD_WWG", 1);
  static const int v2 = measure_knob("SA_FUSED16_V2", 0);
  if (C == 16 && Cy == 16 && (v2 || !mask_x))
    return run_wino_bwd32<16, 16, 64, 5, 5>(dy, w, x, add, out, relu_x, mask_x, N, H, W, ws,
                                            ws_floats, dw, db, s);
  if (C == 16 && Cy == 16 && mask_x) {
    if (wwg)
      return run_wino_bwd<16, 64, 5, 0, true>(dy, w, x, add, out, relu_x, N, H, W, ws, ws_floats, dw, db, s);
    if (kd == 0) return run_wino_bwd<16, 64, 5, 0>(dy, w, x, add, out, relu_x, N, H, W, ws, ws_floats, dw, db, s);
    if (kd == 8) return run_wino_bwd<16, 64, 5, 8>(dy, w, x, add, out, relu_x, N, H, W, ws, ws_floats, dw, db, s);
    return run_wino_bwd<16, 64, 5, 4>(dy, w, x, add, out, relu_x, N, H, W, ws, ws_floats, dw, db, s);
  }
  static const int f32c = measure_knob("SA_FUSED_BWD32", 1);
  if (!f32c) return false;
  if (C == 32 && Cy == 32)
    return run_wino_bwd32<32, 32, 32, 5, 5>(dy, w, x, add, out, relu_x, mask_x, N, H, W, ws,
                                            ws_floats, dw, db, s);
  if (C == 16 && Cy == 32)
    return run_wino_bwd32<16, 32, 32, 4, 8>(dy, w, x, add, out, relu_x, mask_x, N, H, W, ws,
                                            ws_floats, dw, db, s);
  return false;
}

}  // namespace cf32
}  // namespace sa
