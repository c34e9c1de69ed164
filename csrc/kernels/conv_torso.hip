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

#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>

namespace sa {
namespace cf32 {
int conv_cus();  // conv_f32.hip: CUs left to the persistent grids
}  // namespace cf32
namespace conv {
namespace {

constexpr int kThreads = 256;
// Phase ablation for timing studies (tools/conv_bench.py, knob "ablate":
// 1 pool/gather, 2 wgrad, 4 conv, 8 LDS commit) exists only in builds with
// -DSA_CONV_ABLATE: the runtime branches around the staging commit make the
// compiler's vmcnt bookkeeping conservative (it then drains the prefetch).
#ifndef SA_LATE_PREFETCH
#define SA_LATE_PREFETCH 0
#endif
constexpr bool kLatePrefetch = SA_LATE_PREFETCH;
#ifdef SA_CONV_ABLATE
__device__ __forceinline__ bool kKeep(int xcd, int bit) { return !((xcd >> 8) & bit); }
#else
__device__ __forceinline__ constexpr bool kKeep(int, int) { return true; }
#endif
constexpr int kWaves = kThreads / 64;
constexpr int GPW = 4;  // 16-pixel groups per wave per chunk
constexpr int NREG = 4;  // staging registers (uint4) per lane per stream
// Largest tile (output pixels) of a conv whose staged input has C channels:
// the tile-height rules keep the staged halo rows within NREG*kThreads 16-B
// chunks, i.e. at most NREG*kThreads*8/C pixels.
constexpr int kMaxTilePx(int C) { return NREG * kThreads * 8 / C; }

// LDS halo images [rows][W+2][C].  32-channel images (64-B pixels) get 32 B
// of padding per row, so a row starts 2 slots (mod 4) after the previous
// one; their MFMA column groups are 2 rows x 8 pixels (GroupMap).  A
// ds_read_b128 of such a group (16 lanes x one 16-B chunk) is then
// conflict-free for any starting pixel; 16 consecutive 64-B pixels of one row
// would be 2-way conflicted.  16-channel images are unpadded, their groups
// 16 consecutive pixels (paired-tap reads of 32-B pixels are conflict-free).
__host__ __device__ constexpr int row_pitch(int C, int W) {
  return (W + 2) * C + (C == 32 ? 16 : 0);
}
__host__ __device__ constexpr int ceil_div(int a, int b) { return (a + b - 1) / b; }
// MFMA column groups of a tile of `rows` x W output pixels.
__host__ __device__ constexpr int tile_groups(int C, int rows, int W) {
  return C == 32 ? ceil_div(rows, 2) * ceil_div(W, 8) : ceil_div(rows * W, 16);
}

template <int C>
struct GroupMap {
  int Wt, rows, ncb, ngroups;
  __device__ __forceinline__ GroupMap(int Wt_, int npix) : Wt(Wt_), rows(npix / Wt_) {
    ncb = (Wt + 7) >> 3;
    ngroups = tile_groups(C, rows, Wt);
  }
  // pixel (r, c) of lane i of group g; invalid lanes get (0, 0)
  __device__ __forceinline__ bool pixel(int g, int i, int& r, int& c) const {
    bool valid;
    if constexpr (C == 32) {
      const int rp = g / ncb, cb = g - rp * ncb;
      r = 2 * rp + (i >> 3);
      c = cb * 8 + (i & 7);
      valid = r < rows && c < Wt;
    } else {
      const int q = g * 16 + i;
      valid = q < rows * Wt;
      r = q / Wt;
      c = q - r * Wt;
    }
    if (!valid) r = c = 0;
    return valid;
  }
};

// Persistent tile schedule.  xcd == 0: tile = blockIdx.x + k * gridDim.x.
// xcd == 1: XCD-aware - workgroups are dispatched round-robin over the 8 XCDs
// (b % 8), so each XCD gets one CONTIGUOUS range of tiles (proportional to
// its workgroup count) and its workgroups sweep that range together; the
// halo rows neighbouring tiles share then hit the XCD's own L2.
struct TileIter {
  int first, stride, end;
  __device__ __forceinline__ TileIter(int ntiles, int xcd) {
    if (!(xcd & 1)) {
      first = blockIdx.x;
      stride = gridDim.x;
      end = ntiles;
      return;
    }
    const int G = gridDim.x, x = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int gx = G / 8 + (x < G % 8 ? 1 : 0);
    const int before = x * (G / 8) + min(x, G % 8);
    const int lo = static_cast<int>(static_cast<int64_t>(ntiles) * before / G);
    end = static_cast<int>(static_cast<int64_t>(ntiles) * (before + gx) / G);
    first = lo + j;
    stride = gx;
  }
  __device__ __forceinline__ bool valid(int t) const { return t < end; }
  __device__ __forceinline__ int next(int t) const { return t + stride; }
};

// ----------------------------------------------------------------- forward
// Calls f(IC<n>) with n = nv in [1, N] as a compile-time constant, so chunk
// bodies are branch-free (every LDS read of a chunk can be issued ahead of
// its MFMAs) without computing padding groups.
template <int N, typename F>
__device__ __forceinline__ void for_count(int nv, F&& f) {
  if constexpr (N > 1) {
    if (nv < N) {
      for_count<N - 1>(nv, f);
      return;
    }
  }
  f(std::integral_constant<int, N>{});
}

// Chunking of a tile's 16-pixel groups over the waves: wave w computes
// groups w + kWaves * (c * gpw + gi) (chunk c, gi < gpw).  The chunk loop is
// unrolled over the kChunks a tile can need (the tile-height rules bound a
// tile to kMaxTilePx pixels): with a real loop holding global stores, the
// compiler drains vmcnt in the preheader, i.e. waits for the next tile's
// prefetch before computing this one.
template <int GP, int MAXPX, int MAPC>
struct Chunking {
  static constexpr int kGpw = GP;
  static constexpr int kMapC = MAPC;  // GroupMap of the image the MFMAs read
  static constexpr int kMaxGroups = MAXPX / 16;  // enforced by the tile rules
  static constexpr int kChunks = (kMaxGroups + kWaves * GP - 1) / (kWaves * GP);
  static constexpr int kSlots = kChunks * GP;  // groups per wave, max
};
template <int CIN, int COUT>
using FwdChunks = Chunking<GPW, kMaxTilePx(CIN), CIN>;
template <int CIN, int COUT>
using DgradChunks =
    Chunking<(CIN == 32 ? 2 : GPW), kMaxTilePx(CIN < COUT ? CIN : COUT), COUT>;

// Per-lane copy of a global [pixels][C] bf16 operand for the epilogue of
// this wave's groups (4 channels per 16-channel half), loaded BEFORE the
// next tile's prefetch is issued: vmcnt is in order, so a global load in the
// epilogue would otherwise also wait for the whole prefetch.
template <int C, typename CH>
struct EpiOperand {
  static constexpr int NH = C / 16;
  uint2 v[CH::kSlots][NH];
  __device__ __forceinline__ void load(const bf16_t* __restrict__ src,
                                       int64_t img0, int npix, int Wt) {
    const int lane = lane_id();
    const int wave = wave_id();
    const GroupMap<CH::kMapC> gm(Wt, npix);
#pragma unroll
    for (int k = 0; k < CH::kSlots; ++k) {
      // unconditional loads (invalid lanes read pixel 0): see RowStager
      int r, c;
      gm.pixel(wave + kWaves * k, lane & 15, r, c);
      const int q = r * Wt + c;
#pragma unroll
      for (int h = 0; h < NH; ++h)
        v[k][h] = *reinterpret_cast<const uint2*>(src + (img0 + q) * C + 16 * h +
                                                  4 * (lane >> 4));
    }
  }
  __device__ __forceinline__ void get(int slot, int co0, float f[4]) const {
    const uint2 o = v[slot][co0 >> 4];
    f[0] = __uint_as_float(o.x << 16);
    f[1] = __uint_as_float(o.x & 0xFFFF0000u);
    f[2] = __uint_as_float(o.y << 16);
    f[3] = __uint_as_float(o.y & 0xFFFF0000u);
  }
};

// Bias of this lane's output channels (co0 = 16 h + 4 (lane >> 4)) into
// registers, bounced through LDS `scratch` (contains a barrier; scratch is
// free again after the caller's next barrier).  Loading them with a global
// load straight into the registers used inside the tile loop makes the
// compiler re-check vmcnt there, which (in-order counter) also waits for
// the next tile's prefetch.
template <int COUT>
__device__ __forceinline__ void bias_regs(const float* __restrict__ bias,
                                          float* scratch, float breg[COUT / 16][4]) {
  for (int e = threadIdx.x; e < COUT; e += blockDim.x) scratch[e] = bias[e];
  __syncthreads();
#pragma unroll
  for (int h = 0; h < COUT / 16; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i) breg[h][i] = scratch[16 * h + 4 * (lane_id() >> 4) + i];
}

// Per-wave implicit GEMM over the tile (FwdChunks). x_s: halo tile
// [rows][Wt+2][CIN]; output pixel q=(qr,qc) reads x_s[(qr+ky)*(Wt+2)+qc+kx].
// epi(q, co0, v[4], slot) is called for every valid (pixel, 4-channel slice);
// slot = the group's index in this wave's list (compile-time after unrolling).
template <int CIN, int COUT, typename Epi>
__device__ __forceinline__ void conv_tile_fwd(const bf16_t* x_s,
                                              const bf16_t* w_s, int Wt,
                                              int npix, Epi epi) {
  static_assert(CIN == 16 || CIN == 32, "CIN");
  constexpr int NH = COUT / 16;
  // Keep the per-tap weight fragments in LDS (re-read per chunk) unless
  // they are small: hoisting 9 taps of 32-wide fragments out of the loop
  // costs 72 VGPRs and halves occupancy.
  constexpr bool kReloadW = CIN == 32 || NH == 2;
  const int lane = lane_id();
  const int wave = wave_id();
  const int RP = row_pitch(CIN, Wt);
  const GroupMap<CIN> gm(Wt, npix);
  const int ngroups = gm.ngroups;
  using CH = FwdChunks<CIN, COUT>;
#pragma unroll
  for (int c = 0; c < CH::kChunks; ++c) {
    const int g0 = wave + c * kWaves * CH::kGpw;
    if (g0 >= ngroups) break;
    if constexpr (kReloadW) asm volatile("" ::: "memory");
    const int nv = (ngroups - g0 + kWaves - 1) / kWaves;
    for_count<CH::kGpw>(nv, [&](auto NCc) {
      constexpr int NC = decltype(NCc)::value;
      f4 acc[NC][NH];
      int base[NC], qv[NC];
#pragma unroll
      for (int gi = 0; gi < NC; ++gi) {
#pragma unroll
        for (int h = 0; h < NH; ++h) acc[gi][h] = f4{0.f, 0.f, 0.f, 0.f};
        int qr, qc;
        const bool valid = gm.pixel(g0 + kWaves * gi, lane & 15, qr, qc);
        qv[gi] = valid ? qr * Wt + qc : -1;
        base[gi] = qr * RP + qc * CIN;
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap % 3;
        const int toff = ky * RP + kx * CIN;
        if constexpr (CIN == 16) {
          // paired taps: K = 32 = (kx0, kx0 + 1) x 16 ci, i.e. two
          // neighbouring pixels read as ONE conflict-free ds_read_b128 per
          // lane (6 MFMA 16x16x32 per group instead of 9 16x16x16; the
          // compiler fuses 8-byte reads into ds_read2_b64, which banks mod
          // 32 and serialises 4-way on this 32-byte pixel stride)
          if (kx == 1) continue;  // covered by the (0, 1) pair
          const int pr = kx >> 1;  // pair 0: kx 0,1; pair 1: kx 2,(3 = zero weights)
          bf8 a[NH];
#pragma unroll
          for (int h = 0; h < NH; ++h)
            a[h] = *reinterpret_cast<const bf8*>(
                w_s + (((ky * 2 + pr) * COUT + (lane & 15) + 16 * h) * 32) + 8 * (lane >> 4));
#pragma unroll
          for (int gi = 0; gi < NC; ++gi) {
            const bf8 b = *reinterpret_cast<const bf8*>(x_s + base[gi] + toff +
                                                        8 * (lane >> 4));
#pragma unroll
            for (int h = 0; h < NH; ++h) acc[gi][h] = mfma32(a[h], b, acc[gi][h]);
          }
        } else {
          bf8 a[NH];
#pragma unroll
          for (int h = 0; h < NH; ++h)
            a[h] = *reinterpret_cast<const bf8*>(
                w_s + (tap * COUT + (lane & 15) + 16 * h) * CIN + 8 * (lane >> 4));
#pragma unroll
          for (int gi = 0; gi < NC; ++gi) {
            const bf8 b = *reinterpret_cast<const bf8*>(x_s + base[gi] + toff +
                                                        8 * (lane >> 4));
#pragma unroll
            for (int h = 0; h < NH; ++h) acc[gi][h] = mfma32(a[h], b, acc[gi][h]);
          }
        }
      }
#pragma unroll
      for (int gi = 0; gi < NC; ++gi) {
        if (qv[gi] >= 0) {
#pragma unroll
          for (int h = 0; h < NH; ++h) {
            float v[4] = {acc[gi][h][0], acc[gi][h][1], acc[gi][h][2], acc[gi][h][3]};
            epi(qv[gi], 16 * h + 4 * (lane >> 4), v, c * CH::kGpw + gi);
          }
        }
      }
    });
  }
}

__device__ __forceinline__ void store4(bf16_t* dst, const float v[4]) {
  uint2 o;
  o.x = static_cast<uint32_t>(f2bf(v[0])) | (static_cast<uint32_t>(f2bf(v[1])) << 16);
  o.y = static_cast<uint32_t>(f2bf(v[2])) | (static_cast<uint32_t>(f2bf(v[3])) << 16);
  *reinterpret_cast<uint2*>(dst) = o;
}
// store4 with one v_cvt_pk_bf16_f32 per pair (same bits).  Measured per
// kernel (profiles/experiments.md): it also keeps the residual/skip operand
// arrays of the 32-channel and backward kernels out of scratch, but slows
// the 16-channel forward convs, which keep store4.
__device__ __forceinline__ void store4_pk(bf16_t* dst, const float v[4]) {
  uint2 o;
  o.x = pack_bf16x2_asm(v[0], v[1]);
  o.y = pack_bf16x2_asm(v[2], v[3]);
  *reinterpret_cast<uint2*>(dst) = o;
}
__device__ __forceinline__ void load4(const bf16_t* src, float v[4]) {
  const uint2 o = *reinterpret_cast<const uint2*>(src);
  v[0] = __uint_as_float(o.x << 16);
  v[1] = __uint_as_float(o.x & 0xFFFF0000u);
  v[2] = __uint_as_float(o.y << 16);
  v[3] = __uint_as_float(o.y & 0xFFFF0000u);
}

// Pre-pool conv outputs are stored in LDS as order-preserving 16-bit keys
// (bf16 bits with the magnitude bits of negatives flipped, so signed-int16
// order == float order).  The pooling then needs one v_and_or/v_lshl_or and
// one v_max_i32 per channel and tap: key32 = ord16 << 16 | (15 - tap code),
// so the max also yields the first maximal tap of the 3x3 window.
__device__ __forceinline__ uint32_t bf2_to_ord(uint32_t u) {
  return u ^ (((u >> 15) & 0x00010001u) * 0x7FFFu);
}

// Pre-pool LDS image y_s: order keys [Rc conv rows from cr0][W + 2][COUT],
// columns -1 and W are permanent pad columns holding kOrdMin keys (written
// once per kernel by init_pool_pads), and conv rows outside the image are
// stored as kOrdMin keys by the conv epilogue (store4_ord_in).  A pad key
// (0x8000 as int16) is below every real key (-inf is 0x807F), so the window
// max needs no bounds checks and the first maximal tap is unchanged.
constexpr uint32_t kOrdMin2 = 0x80008000u;

__device__ __forceinline__ void store4_ord_in(bf16_t* dst, const float v[4],
                                              bool in_image) {
  uint2 o;
  o.x = pack_bf16x2(v[0], v[1]);
  o.y = pack_bf16x2(v[2], v[3]);
  o.x = in_image ? bf2_to_ord(o.x) : kOrdMin2;
  o.y = in_image ? bf2_to_ord(o.y) : kOrdMin2;
  *reinterpret_cast<uint2*>(dst) = o;
}

template <int COUT>
__device__ __forceinline__ void init_pool_pads(bf16_t* y_s, int rows, int W) {
  constexpr int CH = COUT / 8;
  for (int e = threadIdx.x; e < rows * 2 * CH; e += blockDim.x) {
    const int part = e % CH, side = (e / CH) & 1, r = e / (2 * CH);
    *reinterpret_cast<uint4*>(y_s + (r * (W + 2) + (side ? W + 1 : 0)) * COUT +
                              part * 8) =
        make_uint4(kOrdMin2, kOrdMin2, kOrdMin2, kOrdMin2);
  }
}

// 3x3/2 max-pool (TF SAME padding offsets pb_h/pb_w) of the padded conv tile
// in y_s -> pooled bf16 + argmax code dy*3+dx, one 8-channel slice per
// thread.  key32 = ord16 << 16 | (15 - tap): one v_lshl_or / v_and_or and one
// v_max_i32 per channel and tap; the 9 taps are immediate-offset ds_read_b128
// from one base address.  The epilogue unpacks two channels per v_perm.
template <int COUT>
__device__ __forceinline__ void pool_tile(const bf16_t* y_s, int W, int Wo,
                                          int pb_w, int n, int Hp, int i0,
                                          int Rpv, bf16_t* __restrict__ pooled,
                                          uint8_t* __restrict__ argmax) {
  constexpr int CH = COUT / 8;
  const int Wt = W + 2;
  const int total = Rpv * Wo * CH;
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    const int part = e % CH;
    const int pj = (e / CH) % Wo;
    const int pi = e / (CH * Wo);
    // window origin: local conv row 2 pi, padded column 2 pj - pb_w + 1
    const bf16_t* base = y_s + ((2 * pi) * Wt + 2 * pj - pb_w) * COUT + COUT + part * 8;
    int best[8];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const uint4 v = *reinterpret_cast<const uint4*>(base + (dy * Wt + dx) * COUT);
        const uint32_t u[4] = {v.x, v.y, v.z, v.w};
        const uint32_t K = 15 - (dy * 3 + dx);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const int key = static_cast<int>((c & 1) ? ((u[c >> 1] & 0xFFFF0000u) | K)
                                                   : ((u[c >> 1] << 16) | K));
          best[c] = (dy | dx) ? max(best[c], key) : key;
        }
      }
    }
    const int64_t o = ((static_cast<int64_t>(n) * Hp + i0 + pi) * Wo + pj) * COUT + part * 8;
    uint32_t pv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)  // high halves of best[2k], best[2k+1]
      pv[k] = bf2_to_ord(__builtin_amdgcn_perm(static_cast<uint32_t>(best[2 * k + 1]),
                                               static_cast<uint32_t>(best[2 * k]),
                                               0x07060302u));
    *reinterpret_cast<uint4*>(pooled + o) = make_uint4(pv[0], pv[1], pv[2], pv[3]);
    uint32_t lo[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // low bytes (15 - tap) of best[4k..4k+3]
      const uint32_t a = __builtin_amdgcn_perm(static_cast<uint32_t>(best[4 * k + 1]),
                                               static_cast<uint32_t>(best[4 * k]),
                                               0x0c0c0400u);
      const uint32_t b = __builtin_amdgcn_perm(static_cast<uint32_t>(best[4 * k + 3]),
                                               static_cast<uint32_t>(best[4 * k + 2]),
                                               0x0c0c0400u);
      lo[k] = 0x0F0F0F0Fu - (a | (b << 16));
    }
    *reinterpret_cast<uint2*>(argmax + o) = make_uint2(lo[0], lo[1]);
  }
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
  using CH = DgradChunks<CIN, COUT>;  // gpw 2 for CIN 32: bound accumulators
  constexpr int GPWD = CH::kGpw;
  constexpr bool kReloadW = COUT == 32 || NH == 2;  // see conv_tile_fwd
  const int lane = lane_id();
  const int wave = wave_id();
  const int RP = row_pitch(COUT, Wt);
  const GroupMap<COUT> gm(Wt, npix);
  const int ngroups = gm.ngroups;
#pragma unroll
  for (int c = 0; c < CH::kChunks; ++c) {  // unrolled: see Chunking
    const int g0 = wave + c * kWaves * GPWD;
    if (g0 >= ngroups) break;
    if constexpr (kReloadW) asm volatile("" ::: "memory");
    const int nv = (ngroups - g0 + kWaves - 1) / kWaves;
    for_count<GPWD>(nv, [&](auto NCc) {
      constexpr int NC = decltype(NCc)::value;
      f4 acc[NC][NH];
      int base[NC], qv[NC];
#pragma unroll
      for (int gi = 0; gi < NC; ++gi) {
#pragma unroll
        for (int h = 0; h < NH; ++h) acc[gi][h] = f4{0.f, 0.f, 0.f, 0.f};
        int qr, qc;
        const bool valid = gm.pixel(g0 + kWaves * gi, lane & 15, qr, qc);
        qv[gi] = valid ? qr * Wt + qc : -1;
        base[gi] = qr * RP + qc * COUT;  // + (2-ky, 2-kx) per tap
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap % 3;
        const int toff = (2 - ky) * RP + (2 - kx) * COUT;
        if constexpr (COUT == 16) {
          // paired column offsets (see conv_tile_fwd): offsets o = 2 - kx in
          // (0, 1) and (2, 3 = zero weights), one ds_read_b128 per lane
          const int o = 2 - kx;
          if (o == 1 || o == 3) continue;
          const int pr = o >> 1, ro = 2 - ky;
          bf8 a[NH];
#pragma unroll
          for (int h = 0; h < NH; ++h)
            a[h] = *reinterpret_cast<const bf8*>(
                w_s + (((ro * 2 + pr) * CIN + (lane & 15) + 16 * h) * 32) + 8 * (lane >> 4));
#pragma unroll
          for (int gi = 0; gi < NC; ++gi) {
            const bf8 b = *reinterpret_cast<const bf8*>(d_s + base[gi] + toff +
                                                        8 * (lane >> 4));
#pragma unroll
            for (int h = 0; h < NH; ++h) acc[gi][h] = mfma32(a[h], b, acc[gi][h]);
          }
        } else {
          bf8 a[NH];
#pragma unroll
          for (int h = 0; h < NH; ++h)
            a[h] = *reinterpret_cast<const bf8*>(
                w_s + (tap * CIN + (lane & 15) + 16 * h) * COUT + 8 * (lane >> 4));
#pragma unroll
          for (int gi = 0; gi < NC; ++gi) {
            const bf8 b = *reinterpret_cast<const bf8*>(d_s + base[gi] + toff +
                                                        8 * (lane >> 4));
#pragma unroll
            for (int h = 0; h < NH; ++h) acc[gi][h] = mfma32(a[h], b, acc[gi][h]);
          }
        }
      }
#pragma unroll
      for (int gi = 0; gi < NC; ++gi) {
        if (qv[gi] >= 0) {
#pragma unroll
          for (int h = 0; h < NH; ++h) {
            float v[4] = {acc[gi][h][0], acc[gi][h][1], acc[gi][h][2], acc[gi][h][3]};
            epi(qv[gi], 16 * h + 4 * (lane >> 4), v, c * CH::kGpw + gi);
          }
        }
      }
    });
  }
}

// wgrad accumulators.  The 9 taps are split into TG tap groups (TG = 1 for
// 16x16 weights, 2 for the larger ones to bound accumulator registers); wave w
// owns tap group w % TG and visits every (4/TG)-th 16-pixel group, so the dY
// operand and the pixel addressing are read/computed 4/TG times less often
// than with one tap set per wave.  D[m=ci][n=co] per (tap, ci-half,
// co-half); the waves' partial sums are reduced through LDS once per
// workgroup (flush_wgrad).
template <int CIN, int COUT>
struct WgradAcc {
  static constexpr int HC = CIN / 16, HO = COUT / 16;
  static constexpr int TG = CIN * COUT > 512 ? 2 : 1;  // tap groups
  static constexpr int TPG = (9 + TG - 1) / TG;        // taps per group
  f4 w[TPG][HC][HO];
  f4 b[HO];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int t = 0; t < TPG; ++t)
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
  using A = WgradAcc<CIN, COUT>;
  constexpr int HC = A::HC, HO = A::HO, TG = A::TG, TPG = A::TPG;
  constexpr int GSTRIDE = kWaves / TG;
  const int lane = lane_id();
  const int wave = wave_id();
  const int tg = wave % TG;
  const int RPa = row_pitch(CIN, Wt), RPd = row_pitch(COUT, Wt);
  const int ngroups = (npix + 15) / 16;
  const int sub = lane & 15;
  const int qrow = sub >> 2;       // row of the 4x16 tr block
  const int pcol = (sub & 3) * 4;  // 4-element column chunk
  s4 ones;
  ones[0] = ones[1] = ones[2] = ones[3] = 0x3F80;  // bf16 1.0
  for (int g = wave / TG; g < ngroups; g += GSTRIDE) {
    const int q = g * 16 + 4 * (lane >> 4) + qrow;
    const bool valid = q < npix;
    const int qr = valid ? q / Wt : 0;
    const int qc = valid ? q - qr * Wt : 0;
    s4 bd[HO];
#pragma unroll
    for (int o = 0; o < HO; ++o) {
      bd[o] = lds_tr4(d_s + (valid ? (qr + 1) * RPd + (qc + 1) * COUT : zero_d) + 16 * o + pcol);
      if (tg == 0) acc.b[o] = mfma16(ones, bd[o], acc.b[o]);
    }
#pragma unroll
    for (int k = 0; k < TPG; ++k) {
      const int tap = tg * TPG + k;
      if (tap < 9) {
        const int ky = tap / 3, kx = tap % 3;
        const int aoff = (qr + ky) * RPa + (qc + kx) * CIN;
#pragma unroll
        for (int c = 0; c < HC; ++c) {
          const s4 aa = lds_tr4(a_s + (valid ? aoff : zero_a) + 16 * c + pcol);
#pragma unroll
          for (int o = 0; o < HO; ++o) acc.w[k][c][o] = mfma16(aa, bd[o], acc.w[k][c][o]);
        }
      }
    }
  }
}

// Sums the waves' accumulators through LDS (scratch: >= 4*CIN*COUT floats,
// 16-B aligned; all tile work must be finished) and adds the workgroup's
// total to dw/db with one float atomic per element.
// part != nullptr (deterministic mode): the workgroup's totals go to its own
// slot part[blockIdx.x][9*CIN*COUT + COUT] instead (every element written
// once), and slot_reduce_kernel adds the slots in a fixed order.
template <int CIN, int COUT>
__device__ __forceinline__ void flush_wgrad(const WgradAcc<CIN, COUT>& acc,
                                            float scale, float* __restrict__ dw,
                                            float* __restrict__ db,
                                            float* scratch,
                                            float* __restrict__ part) {
  float* slot = part ? part + static_cast<int64_t>(blockIdx.x) * (9 * CIN * COUT + COUT)
                     : nullptr;
  using A = WgradAcc<CIN, COUT>;
  constexpr int HC = A::HC, HO = A::HO, TG = A::TG, TPG = A::TPG;
  constexpr int PER = CIN * COUT;  // floats per wave per tap
  const int lane = lane_id();
  const int wave = wave_id();
  __syncthreads();
#pragma unroll
  for (int k = 0; k <= TPG; ++k) {  // k == TPG: bias pseudo-tap
    // [wave][c][o][i][lane]: conflict-free writes
#pragma unroll
    for (int c = 0; c < HC; ++c)
#pragma unroll
      for (int o = 0; o < HO; ++o)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = k < TPG ? acc.w[k < TPG ? k : 0][c][o][i]
                                  : (c == 0 ? acc.b[o][i] : 0.f);
          scratch[wave * PER + ((c * HO + o) * 4 + i) * 64 + lane] = v;
        }
    __syncthreads();
    for (int e = threadIdx.x; e < TG * PER; e += kThreads) {
      const int tg = e / PER;
      const int r = e - tg * PER;
      float v = 0.f;
#pragma unroll
      for (int w = tg; w < kWaves; w += TG) v += scratch[w * PER + r];
      const int l = r & 63;
      const int i = (r >> 6) & 3;
      const int co_h = (r >> 8) % HO;
      const int ci_h = (r >> 8) / HO;
      const int ci = 16 * ci_h + 4 * (l >> 4) + i;
      const int co = 16 * co_h + (l & 15);
      const int tap = tg * TPG + k;
      if (k < TPG) {
        if (tap < 9) {
          const int o = (tap * CIN + ci) * COUT + co;
          if (slot) slot[o] = v * scale;
          else atomicAdd(dw + o, v * scale);
        }
      } else if (tg == 0 && ci_h == 0 && (l >> 4) == 0 && i == 0) {
        // bias: every D row holds the column sum
        if (slot) slot[9 * CIN * COUT + co] = v;
        else atomicAdd(db + co, v);
      }
    }
    __syncthreads();
  }
}

// ----------------------------------------------------------------- staging
// Register-staged loads: issue() puts a tile's global loads in flight (16-B
// per lane), commit() writes them into LDS after the previous tile's compute
// finished.  A persistent workgroup thus overlaps the HBM reads of tile k+1
// with the MFMA work and stores of tile k (cdna_hip_programming.md T14).

// Full-width NHWC rows [r_begin, r_begin+rows) of image n (rows outside
// [0,H) read as zero) -> LDS [rows][W(+2)][C]; HALO adds zeroed halo columns.
template <int C, int NREG>
struct RowStager {
  uint4 v[NREG];
  int total, r_begin, H;
  // Every lane issues all NREG loads (addresses clamped into the image) and
  // commit() zeroes what lies outside: the staging registers are then always
  // written by a load and always read after the wait, so the compiler's
  // vmcnt bookkeeping stays exact (a zero-init of a register that may still
  // have a load in flight costs a full vmcnt(0) drain).
  __device__ __forceinline__ void issue(const bf16_t* __restrict__ src, int n,
                                        int H_, int W, int r_begin_, int rows) {
    constexpr int CH = C / 8;
    const int rc = W * CH;
    total = rows * rc;
    r_begin = r_begin_;
    H = H_;
#pragma unroll
    for (int k = 0; k < NREG; ++k) {
      const int e = min(static_cast<int>(threadIdx.x) + k * kThreads, total - 1);
      const int rr = e / rc;
      const int r = min(max(r_begin + rr, 0), H - 1);
      v[k] = *reinterpret_cast<const uint4*>(
          src + (static_cast<int64_t>(n) * H + r) * W * C + (e - rr * rc) * 8);
    }
  }
  template <bool RELU, bool HALO>
  __device__ __forceinline__ void commit(bf16_t* lds, int W) const {
    constexpr int CH = C / 8;
    const int rc = W * CH;
    const int RP = HALO ? row_pitch(C, W) : W * C;
#pragma unroll
    for (int k = 0; k < NREG; ++k) {
      const int e = threadIdx.x + k * kThreads;
      if (e < total) {
        const int rr = e / rc;
        const int rem = e - rr * rc;
        const int px = rem / CH;
        const int part = rem - px * CH;
        const int r = r_begin + rr;
        uint4 x = (r >= 0 && r < H) ? v[k] : make_uint4(0, 0, 0, 0);
        if (RELU) x = relu8(x);
        *reinterpret_cast<uint4*>(lds + rr * RP + (px + (HALO ? 1 : 0)) * C +
                                  part * 8) = x;
      }
    }
    if (HALO) {
      // halo columns of every row, plus the first pixel after the last row
      // (read, with zero weights, by the paired-tap MFMAs of the last row)
      const int rows = total / rc;
      for (int e = threadIdx.x; e < (rows * 2 + 1) * CH; e += kThreads) {
        const int rr = e / (2 * CH);
        const int side = (e / CH) & 1;
        const int part = e % CH;
        *reinterpret_cast<uint4*>(lds + rr * RP + (side ? W + 1 : 0) * C +
                                  part * 8) = make_uint4(0, 0, 0, 0);
      }
    }
  }
};

// Contiguous byte span [off, off+bytes) of `src` (16-B aligned) -> LDS.
template <int NREG>
struct SpanStager {
  uint4 v[NREG];
  int total;
  __device__ __forceinline__ void issue(const uint8_t* __restrict__ src,
                                        int64_t off, int bytes) {
    total = bytes / 16;
#pragma unroll
    for (int k = 0; k < NREG; ++k) {
      const int e = threadIdx.x + k * kThreads;
      v[k] = make_uint4(0, 0, 0, 0);
      if (e < total) v[k] = *reinterpret_cast<const uint4*>(src + off + e * 16);
    }
  }
  __device__ __forceinline__ void commit(uint8_t* lds) const {
#pragma unroll
    for (int k = 0; k < NREG; ++k) {
      const int e = threadIdx.x + k * kThreads;
      if (e < total) *reinterpret_cast<uint4*>(lds + e * 16) = v[k];
    }
  }
};

// uint8 frame rows (CPX = 3 RGB channels or 4 stacked Atari frames per
// pixel), staged as groups of 4 pixels (4 CPX bytes = CPX dwords) per lane:
// when the rows are dword aligned (W % 4 == 0, or CPX == 4) a group is CPX
// dword loads; otherwise it falls back to bytes.
constexpr int kU8Groups = 2;  // 4-pixel groups per lane per tile

template <int NG, int CPX>
struct U8Stager {
  static_assert(CPX == 3 || CPX == 4, "frame channels");
  uint32_t v[CPX * NG];
  int npix;   // pixels in the (clipped) row span
  int row0;   // first staged row (tile coordinates)
  int nrows;  // staged image rows
  __device__ __forceinline__ void issue(const uint8_t* __restrict__ src, int n,
                                        int H, int W, int r_begin, int rows) {
    const int rlo = max(r_begin, 0), rhi = min(r_begin + rows, H);
    row0 = rlo - r_begin;
    nrows = rhi > rlo ? rhi - rlo : 0;
    npix = nrows * W;
    const uint8_t* base = src + (static_cast<int64_t>(n) * H + rlo) * W * CPX;
    const bool aligned =
        (((CPX == 4 ? 0 : W) & 3) | (reinterpret_cast<uintptr_t>(src) & 3)) == 0;
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int g = threadIdx.x + k * kThreads;
#pragma unroll
      for (int j = 0; j < CPX; ++j) v[CPX * k + j] = 0;
      if (4 * g < npix) {
        if (aligned && 4 * g + 4 <= npix) {
          const uint32_t* b32 = reinterpret_cast<const uint32_t*>(base) + CPX * g;
#pragma unroll
          for (int j = 0; j < CPX; ++j) v[CPX * k + j] = b32[j];
        } else {
#pragma unroll
          for (int b = 0; b < 4 * CPX; ++b)
            if (4 * CPX * g + b < CPX * npix)
              v[CPX * k + b / 4] |= static_cast<uint32_t>(base[4 * CPX * g + b]) << (8 * (b % 4));
        }
      }
    }
  }
};

// Staged uint8 rows -> bf16x4 halo tile [rows][W+2][4] (channel 3 zero for
// RGB frames; halo zero); `pad` extra zero pixels follow the tile (MFMA reads
// may run 3 pixels past the last row into weights-zero columns).  Every LDS
// pixel is written exactly once (data, halo or zero row), so no barrier is
// needed inside.
template <int NG, int CPX>
__device__ __forceinline__ void commit_x4(const U8Stager<NG, CPX>& st, bf16_t* x4,
                                          int W, int rows, int pad) {
  const int Wp = W + 2;
  uint2* px4 = reinterpret_cast<uint2*>(x4);
  const uint2 z = make_uint2(0, 0);
  // halo columns of every row, then the trailing pad pixels
  for (int e = threadIdx.x; e < 2 * rows + pad; e += kThreads)
    px4[e < 2 * rows ? (e >> 1) * Wp + (e & 1) * (W + 1) : rows * Wp + e - 2 * rows] = z;
  // rows outside the image
  const int top = st.row0 * W, bot = (rows - st.row0 - st.nrows) * W;
  for (int e = threadIdx.x; e < top + bot; e += kThreads) {
    const int r = e < top ? e / W : st.row0 + st.nrows + (e - top) / W;
    const int c = e < top ? e - (e / W) * W : (e - top) - ((e - top) / W) * W;
    px4[r * Wp + c + 1] = z;
  }
#pragma unroll
  for (int k = 0; k < NG; ++k) {
    const int g = threadIdx.x + k * kThreads;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = 4 * g + j;
      if (p < st.npix) {
        const int rr = p / W, c = p - rr * W;
        uint32_t ch[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int ci = 0; ci < CPX; ++ci) {
          const int b = CPX * j + ci;  // byte within the 4 CPX-byte group
          // byte values are exact in bf16: take the top half of the fp32
          ch[ci] = __float_as_uint(static_cast<float>(
                       (st.v[CPX * k + b / 4] >> (8 * (b % 4))) & 0xFF)) >> 16;
        }
        px4[(st.row0 + rr) * Wp + c + 1] =
            make_uint2(ch[0] | (ch[1] << 16), ch[2] | (ch[3] << 16));
      }
    }
  }
}

// LDS elements of a weight image (paired-tap layouts are 6 x 32 x M).
__host__ __device__ constexpr int w_lds_elems(int CIN, int COUT, bool FWD) {
  return (FWD && CIN == 16) ? 192 * COUT : (!FWD && COUT == 16) ? 192 * CIN : 9 * CIN * COUT;
}

// Fast fp32 [3][3][CIN][COUT] -> LDS bf16 weight load (float4 over co).
template <int CIN, int COUT, bool FWD>
__device__ __forceinline__ void load_weights4(const float* __restrict__ w,
                                              bf16_t* lds) {
  if constexpr ((FWD && CIN == 16) || (!FWD && COUT == 16)) {
    // paired-tap layouts (conv_tile_fwd / conv_tile_dgrad, 16-wide K):
    //  FWD : [ky][pair][co][32], k < 16: kx = 2 pair, ci = k; else kx + 1
    //  !FWD: [2-ky][pair][ci][32] over column offsets o = 2 - kx (o = 2 pair
    //        + (k >= 16)), co = k & 15; kx outside 0..2 -> zero
    constexpr int M = FWD ? COUT : CIN;
    for (int e = threadIdx.x; e < 6 * M * 32; e += blockDim.x) {
      const int kk = e & 31, m = (e >> 5) % M, pair = e / (32 * M);
      const int r = pair >> 1, pr = pair & 1;
      float v = 0.f;
      if (FWD) {
        const int kx = 2 * pr + (kk >> 4), ci = kk & 15;
        if (kx < 3) v = w[((r * 3 + kx) * CIN + ci) * COUT + m];
      } else {
        const int kx = 2 - (2 * pr + (kk >> 4)), co = kk & 15, ky = 2 - r;
        if (kx >= 0) v = w[((ky * 3 + kx) * CIN + m) * COUT + co];
      }
      lds[e] = f2bf(v);
    }
    return;
  }
  const int total = 9 * CIN * COUT / 4;
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(w)[e];
    const int co = (e * 4) % COUT;
    const int ci = ((e * 4) / COUT) % CIN;
    const int tap = (e * 4) / (COUT * CIN);
    const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (FWD)
        lds[(tap * COUT + co + i) * CIN + ci] = f2bf(f[i]);
      else
        lds[(tap * CIN + ci) * COUT + co + i] = f2bf(f[i]);
    }
  }
}

// ----------------------------------------------------------------- kernels

template <int C, bool RESID, bool POST_RELU, bool RELU_IN, int HC, int WC, int RC>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2))) void res_conv_fwd_kernel(
    const bf16_t* __restrict__ x, const float* __restrict__ w,
    const float* __restrict__ bias, const bf16_t* __restrict__ resid,
    bf16_t* __restrict__ y, int N, int H_, int W_, int R_, int xcd) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = HC ? HC : H_, W = WC ? WC : W_, R = RC ? RC : R_;
  bf16_t* w_s = reinterpret_cast<bf16_t*>(smem);
  bf16_t* x_s = w_s + w_lds_elems(C, C, true);  // + one pad pixel (paired taps)
  load_weights4<C, C, true>(w, w_s);
  float breg[C / 16][4];
  bias_regs<C>(bias, reinterpret_cast<float*>(x_s), breg);
  const int tpi = (H + R - 1) / R;
  const int ntiles = N * tpi;
  RowStager<C, NREG> sx;
  const TileIter it(ntiles, xcd);
  int tile = it.first;
  if (it.valid(tile)) {
    const int n = tile / tpi, r0 = (tile - n * tpi) * R, Rv = min(R, H - r0);
    sx.issue(x, n, H, W, r0 - 1, Rv + 2);
  }
  for (; it.valid(tile); tile = it.next(tile)) {
    const int n = tile / tpi, r0 = (tile - n * tpi) * R, Rv = min(R, H - r0);
    __syncthreads();
    if (kKeep(xcd, 8))
    sx.template commit<RELU_IN, true>(x_s, W);
    __syncthreads();
    const int64_t img0 = (static_cast<int64_t>(n) * H + r0) * W;
    // residual straight from HBM into registers (no staging LDS), issued
    // before the prefetch so the epilogue does not wait for the prefetch
    EpiOperand<C, FwdChunks<C, C>> rop;
    if (RESID) rop.load(resid, img0, Rv * W, W);
    const int nt = it.next(tile);
    auto prefetch = [&]() {
      {  // unconditional: see issue() in the backward kernels
        const int t2 = it.valid(nt) ? nt : tile;
        const int n2 = t2 / tpi, r2 = (t2 - n2 * tpi) * R, Rv2 = min(R, H - r2);
        sx.issue(x, n2, H, W, r2 - 1, Rv2 + 2);
      }
    };
    if (!kLatePrefetch) prefetch();
    if (kKeep(xcd, 4))
    conv_tile_fwd<C, C>(x_s, w_s, W, Rv * W, [&](int q, int co0, float v[4], int slot) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] += breg[co0 >> 4][i];
      if (RESID) {
        float r[4];
        rop.get(slot, co0, r);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] += r[i];
      }
      if (POST_RELU) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], 0.f);
      }
      if constexpr (C == 16)
        store4(y + (img0 + q) * C + co0, v);
      else
        store4_pk(y + (img0 + q) * C + co0, v);
    });
    if (kLatePrefetch) prefetch();
  }
}

// Whole residual block forward in one pass (reference experiment.py:170-175):
//   t = relu(conv1(relu(x)) + b1)          (stored ReLU'd, for the backward)
//   y = conv2(t) + b2 + x  [+ final relu]
// A tile of R output rows stages x rows [r0-2, r0+R+2) once, computes t for
// rows [r0-1, r0+R+1) into an LDS halo image (the two halo rows are
// recomputed by the neighbouring tiles too; rows outside the image are the
// zero padding of conv2), writes t rows [r0, r0+R) to HBM and y straight
// from conv2's epilogue.  Against two res_conv_fwd launches this removes the
// HBM write+read of t by conv2 and one launch per block.
template <int C, bool POST_RELU, int HC, int WC, int RC>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2))) void res_block_fwd_kernel(
    const bf16_t* __restrict__ x, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ w2,
    const float* __restrict__ b2, bf16_t* __restrict__ t_out,
    bf16_t* __restrict__ y, int N, int H_, int W_, int R_, int xcd) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = HC ? HC : H_, W = WC ? WC : W_, R = RC ? RC : R_;
  const int RP = row_pitch(C, W);
  bf16_t* w1_s = reinterpret_cast<bf16_t*>(smem);
  bf16_t* w2_s = w1_s + w_lds_elems(C, C, true);
  bf16_t* x_s = w2_s + w_lds_elems(C, C, true);   // (R+4) rows + pad pixel
  bf16_t* t_s = x_s + (R + 4) * RP + C;           // (R+2) rows + pad pixel
  load_weights4<C, C, true>(w1, w1_s);
  load_weights4<C, C, true>(w2, w2_s);
  float bq1[C / 16][4], bq2[C / 16][4];
  bias_regs<C>(b1, reinterpret_cast<float*>(x_s), bq1);
  __syncthreads();
  bias_regs<C>(b2, reinterpret_cast<float*>(x_s) + C, bq2);
  // t_s halo columns stay zero for the whole kernel (epilogues write only
  // interior pixels)
  for (int e = threadIdx.x; e < (R + 2) * 2 * (C / 8); e += kThreads) {
    const int rr = e / (2 * (C / 8)), side = (e / (C / 8)) & 1, part = e % (C / 8);
    *reinterpret_cast<uint4*>(t_s + rr * RP + (side ? W + 1 : 0) * C + part * 8) =
        make_uint4(0, 0, 0, 0);
  }
  const int tpi = (H + R - 1) / R;
  const int ntiles = N * tpi;
  RowStager<C, NREG> sx;
  const TileIter it(ntiles, xcd);
  int tile = it.first;
  if (it.valid(tile)) {
    const int n = tile / tpi, r0 = (tile - n * tpi) * R, Rv = min(R, H - r0);
    sx.issue(x, n, H, W, r0 - 2, Rv + 4);
  }
  for (; it.valid(tile); tile = it.next(tile)) {
    const int n = tile / tpi, r0 = (tile - n * tpi) * R, Rv = min(R, H - r0);
    __syncthreads();
    if (kKeep(xcd, 8))
    sx.template commit<true, true>(x_s, W);
    // zero pixel after t's last row (read with zero weights by paired taps)
    for (int e = threadIdx.x; e < C / 8; e += kThreads)
      *reinterpret_cast<uint4*>(t_s + (Rv + 2) * RP + e * 8) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const int64_t img0 = (static_cast<int64_t>(n) * H + r0) * W;
    EpiOperand<C, FwdChunks<C, C>> rop;  // skip = raw x rows [r0, r0+Rv)
    rop.load(x, img0, Rv * W, W);
    const int nt = it.next(tile);
    {  // unconditional: see issue() in the backward kernels
      const int t2 = it.valid(nt) ? nt : tile;
      const int n2 = t2 / tpi, r2 = (t2 - n2 * tpi) * R, Rv2 = min(R, H - r2);
      sx.issue(x, n2, H, W, r2 - 2, Rv2 + 4);
    }
    if (kKeep(xcd, 4))
    conv_tile_fwd<C, C>(x_s, w1_s, W, (Rv + 2) * W, [&](int q, int co0, float v[4], int) {
      const int qr = q / W, qc = q - qr * W;
      const int r = r0 - 1 + qr;  // image row of this t pixel
      const bool in = r >= 0 && r < H;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = in ? fmaxf(v[i] + bq1[co0 >> 4][i], 0.f) : 0.f;
      store4_pk(t_s + qr * RP + (qc + 1) * C + co0, v);
      if (qr >= 1 && qr <= Rv) store4_pk(t_out + (img0 + q - W) * C + co0, v);
    });
    __syncthreads();
    if (kKeep(xcd, 4))
    conv_tile_fwd<C, C>(t_s, w2_s, W, Rv * W, [&](int q, int co0, float v[4], int slot) {
      float r[4];
      rop.get(slot, co0, r);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] += bq2[co0 >> 4][i];  // same rounding order as res_conv_fwd
        v[i] += r[i];
        if (POST_RELU) v[i] = fmaxf(v[i], 0.f);
      }
      store4_pk(y + (img0 + q) * C + co0, v);
    });
  }
}

template <int CIN, int COUT, int HC, int WC, int RC>
__global__ __launch_bounds__(kThreads) void conv_pool_fwd_kernel(
    const bf16_t* __restrict__ x, const float* __restrict__ w,
    const float* __restrict__ bias, bf16_t* __restrict__ pooled,
    uint8_t* __restrict__ argmax, int N, int H_, int W_, int Rp_, int pb_h,
    int pb_w, int xcd) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = HC ? HC : H_, W = WC ? WC : W_, Rp = RC ? RC : Rp_;
  const int Hp = (H + 1) / 2, Wo = (W + 1) / 2;
  bf16_t* w_s = reinterpret_cast<bf16_t*>(smem);
  bf16_t* x_s = w_s + w_lds_elems(CIN, COUT, true);
  bf16_t* y_s = x_s + (2 * Rp + 3) * row_pitch(CIN, W) + CIN;  // + pad pixel
  load_weights4<CIN, COUT, true>(w, w_s);
  float breg[COUT / 16][4];
  bias_regs<COUT>(bias, reinterpret_cast<float*>(x_s), breg);
  init_pool_pads<COUT>(y_s, 2 * Rp + 1, W);
  const int tpi = (Hp + Rp - 1) / Rp;
  const int ntiles = N * tpi;
  RowStager<CIN, NREG> sx;
  auto issue = [&](int t) {
    const int n = t / tpi, i0 = (t - n * tpi) * Rp, Rpv = min(Rp, Hp - i0);
    sx.issue(x, n, H, W, 2 * i0 - pb_h - 1, 2 * Rpv + 3);
  };
  const TileIter it(ntiles, xcd);
  int tile = it.first;
  if (it.valid(tile)) issue(tile);
  for (; it.valid(tile); tile = it.next(tile)) {
    const int n = tile / tpi, i0 = (tile - n * tpi) * Rp, Rpv = min(Rp, Hp - i0);
    const int cr0 = 2 * i0 - pb_h;
    const int Rc = 2 * Rpv + 1;
    __syncthreads();
    if (kKeep(xcd, 8))
    sx.template commit<false, true>(x_s, W);
    __syncthreads();
    // unconditional (no next tile: re-issue this one, unused) - a conditional
    // issue leaves a join at the loop back-edge
    issue(it.valid(it.next(tile)) ? it.next(tile) : tile);
    if (kKeep(xcd, 4))
    conv_tile_fwd<CIN, COUT>(x_s, w_s, W, Rc * W, [&](int q, int co0, float v[4], int) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] += breg[co0 >> 4][i];
      const int qr = q / W;
      store4_ord_in(y_s + (q + 2 * qr + 1) * COUT + co0, v,
                    static_cast<unsigned>(cr0 + qr) < static_cast<unsigned>(H));
    });
    __syncthreads();
    if (kKeep(xcd, 1))
    pool_tile<COUT>(y_s, W, Wo, pb_w, n, Hp, i0, Rpv, pooled, argmax);
  }
}

// First layer: the uint8 frame tile is staged as bf16x4 pixels (raw byte
// values are exact in bf16; 1/255 is folded into the weights).  With 4 values
// per pixel, one 16x16x16 MFMA covers a whole kernel row (kx = 0..2 plus a
// zero-weight kx = 3, ci = 0..3): 3 MFMAs and 3 ds_read_b64 per 16 pixels,
// for RGB (CPX = 3, ci = 3 zero-weight) and 4-frame stacks (CPX = 4) alike.
template <int CPX, int HC, int WC, int RC>
__global__ __launch_bounds__(kThreads) void conv1_pool_fwd_kernel(
    const uint8_t* __restrict__ x, const float* __restrict__ w,
    const float* __restrict__ bias, bf16_t* __restrict__ pooled,
    uint8_t* __restrict__ argmax, int N, int H_, int W_, int Rp_, int pb_h,
    int pb_w, int xcd) {
  constexpr int COUT = 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = HC ? HC : H_, W = WC ? WC : W_, Rp = RC ? RC : Rp_;
  const int Hp = (H + 1) / 2, Wo = (W + 1) / 2;
  const int Wp = W + 2;
  bf16_t* w_s = reinterpret_cast<bf16_t*>(smem);        // [3 ky][16 co][16 k]
  bf16_t* y_s = w_s + 3 * 16 * 16;                        // [2Rp+1][W+2][16]
  bf16_t* x4 = y_s + (2 * Rp + 1) * (W + 2) * COUT;       // [(2Rp+3)][W+2][4] + pad
  for (int e = threadIdx.x; e < 3 * 16 * 16; e += blockDim.x) {
    const int ky = e / 256, co = (e / 16) % 16, k = e % 16;
    const int kx = k / 4, ci = k % 4;
    w_s[e] = (kx < 3 && ci < CPX)
                 ? f2bf(w[((ky * 3 + kx) * CPX + ci) * COUT + co] * (1.0f / 255.0f))
                 : 0;
  }
  const int lane = lane_id();
  const int wave = wave_id();
  const int tpi = (Hp + Rp - 1) / Rp;
  const int ntiles = N * tpi;
  U8Stager<kU8Groups, CPX> sx;
  auto issue = [&](int t) {
    const int n = t / tpi, i0 = (t - n * tpi) * Rp, Rpv = min(Rp, Hp - i0);
    sx.issue(x, n, H, W, 2 * i0 - pb_h - 1, 2 * Rpv + 3);
  };
  float breg[1][4];
  bias_regs<COUT>(bias, reinterpret_cast<float*>(y_s), breg);
  const float b0 = breg[0][0], b1 = breg[0][1], b2 = breg[0][2], b3 = breg[0][3];
  __syncthreads();  // bias scratch (in y_s) read before the pads overwrite it
  init_pool_pads<COUT>(y_s, 2 * Rp + 1, W);
  const TileIter it(ntiles, xcd);
  int tile = it.first;
  if (it.valid(tile)) issue(tile);
  for (; it.valid(tile); tile = it.next(tile)) {
    const int n = tile / tpi, i0 = (tile - n * tpi) * Rp, Rpv = min(Rp, Hp - i0);
    const int cr0 = 2 * i0 - pb_h;
    const int Rc = 2 * Rpv + 1;
    const int npix = Rc * W;
    __syncthreads();
    if (kKeep(xcd, 8))
    commit_x4(sx, x4, W, Rc + 2, 4);
    __syncthreads();
    // unconditional (no next tile: re-issue this one, unused) - a conditional
    // issue leaves a join at the loop back-edge
    issue(it.valid(it.next(tile)) ? it.next(tile) : tile);
    s4 a[3];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
      a[ky] = *reinterpret_cast<const s4*>(w_s + (ky * 16 + (lane & 15)) * 16 +
                                           4 * (lane >> 4));
    const int ngroups = (npix + 15) / 16;
    for (int g = wave; g < (kKeep(xcd, 4) ? ngroups : 0); g += kWaves) {
      int q = g * 16 + (lane & 15);
      const bool valid = q < npix;
      if (!valid) q = 0;
      const int qr = q / W, qc = q - (q / W) * W;
      f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const s4 bv = *reinterpret_cast<const s4*>(
            x4 + ((qr + ky) * Wp + qc + (lane >> 4)) * 4);
        acc = mfma16(a[ky], bv, acc);
      }
      if (valid) {
        const float v[4] = {acc[0] + b0, acc[1] + b1, acc[2] + b2, acc[3] + b3};
        store4_ord_in(y_s + (q + 2 * qr + 1) * COUT + 4 * (lane >> 4), v,
                      static_cast<unsigned>(cr0 + qr) < static_cast<unsigned>(H));
      }
    }
    __syncthreads();
    if (kKeep(xcd, 1))
    pool_tile<COUT>(y_s, W, Wo, pb_w, n, Hp, i0, Rpv, pooled, argmax);
  }
}

template <int C, bool ADD_SKIP, bool RELU_ACT, int HC, int WC, int RC>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2))) void res_conv_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ act,
    const bf16_t* __restrict__ skip, const float* __restrict__ w,
    bf16_t* __restrict__ dx, float* __restrict__ dw, float* __restrict__ db,
    int N, int H_, int W_, int R_, int xcd, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = HC ? HC : H_, W = WC ? WC : W_, R = RC ? RC : R_;
  const int RP = row_pitch(C, W);
  const int tile_elems = (R + 2) * RP;
  bf16_t* w_s = reinterpret_cast<bf16_t*>(smem);
  bf16_t* d_s = w_s + w_lds_elems(C, C, false);
  bf16_t* a_s = d_s + tile_elems + C;  // + one zero pixel each
  load_weights4<C, C, false>(w, w_s);
  for (int e = threadIdx.x; e < C; e += blockDim.x) {
    d_s[tile_elems + e] = 0;
    a_s[tile_elems + e] = 0;
  }
  WgradAcc<C, C> acc;
  acc.zero();
  const int tpi = (H + R - 1) / R;
  const int ntiles = N * tpi;
  RowStager<C, NREG> sd, sa;
  auto issue = [&](int t) {
    const int n = t / tpi, r0 = (t - n * tpi) * R, Rv = min(R, H - r0);
    sd.issue(dy, n, H, W, r0 - 1, Rv + 2);
    sa.issue(act, n, H, W, r0 - 1, Rv + 2);
  };
  const TileIter it(ntiles, xcd);
  int tile = it.first;
  if (it.valid(tile)) issue(tile);
  for (; it.valid(tile); tile = it.next(tile)) {
    const int n = tile / tpi, r0 = (tile - n * tpi) * R, Rv = min(R, H - r0);
    __syncthreads();  // previous tile's LDS reads done
    if (kKeep(xcd, 8))
    sd.template commit<false, true>(d_s, W);
    if (kKeep(xcd, 8))
    sa.template commit<RELU_ACT, true>(a_s, W);
    __syncthreads();
    const int npix = Rv * W;
    const int64_t img0 = (static_cast<int64_t>(n) * H + r0) * W;
    EpiOperand<C, DgradChunks<C, C>> sop;  // skip grad, before the prefetch
    if (ADD_SKIP) sop.load(skip, img0, npix, W);
    if (!kLatePrefetch && it.valid(it.next(tile))) issue(it.next(tile));
    if (kKeep(xcd, 4))
    conv_tile_dgrad<C, C>(d_s, w_s, W, npix, [&](int q, int ci0, float v[4], int slot) {
      const int qr = q / W, qc = q - (q / W) * W;
      float m[4];
      load4(a_s + (qr + 1) * RP + (qc + 1) * C + ci0, m);
      float s[4] = {0.f, 0.f, 0.f, 0.f};
      if (ADD_SKIP) sop.get(slot, ci0, s);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = s[i] + (m[i] > 0.f ? v[i] : 0.f);
      store4_pk(dx + (img0 + q) * C + ci0, v);
    });
    if (kKeep(xcd, 2))
    conv_tile_wgrad<C, C>(a_s, d_s, W, npix, tile_elems, tile_elems, acc);
    if (kLatePrefetch && it.valid(it.next(tile))) issue(it.next(tile));
  }
  flush_wgrad<C, C>(acc, 1.f, dw, db, reinterpret_cast<float*>(smem), part);
}

// dY of the conv feeding a max-pool as an LDS halo tile (rows [r_begin,
// r_begin+rows) x cols [-1, W], pitch row_pitch(COUT, W)), built per 2x2
// block of conv positions.  Block (i, j)
// holds conv rows 2i-pb_h+{0,1} x cols 2j-pb_w+{0,1}; its cells can only be
// the argmax of pooled windows (i,j), (i-1,j), (i,j-1), (i-1,j-1) (a window's
// dy/dx = 2 cells are the next block's offset-0 cells).  Each thread loads
// those 4 windows once and writes 4 cells:
//   (1,1) <- (i,j):4       (0,1) <- (i,j):1 + (i-1,j):7
//   (1,0) <- (i,j):3 + (i,j-1):5
//   (0,0) <- (i,j):0 + (i-1,j):6 + (i,j-1):2 + (i-1,j-1):8
// (window:code).  ~2x fewer VALU ops and 4x fewer LDS reads than checking
// every window of every cell.  Halo columns are zeroed separately.
template <int COUT>
__device__ __forceinline__ void gather_pool_grad_blocks(
    const bf16_t* p_s, const uint8_t* g_s, int i_lo, int i_hi, int W, int Wo,
    int pb_h, int pb_w, int r_begin, int rows, bf16_t* d_s) {
  constexpr int CH = COUT / 8;
  const int RPd = row_pitch(COUT, W);
  // halo columns -1 and W
  for (int e = threadIdx.x; e < rows * 2 * CH; e += blockDim.x) {
    const int part = e % CH;
    const int side = (e / CH) & 1;
    const int rr = e / (2 * CH);
    *reinterpret_cast<uint4*>(d_s + rr * RPd + (side ? W + 1 : 0) * COUT +
                              part * 8) = make_uint4(0, 0, 0, 0);
  }
  // blocks whose rows intersect [r_begin, r_begin + rows)
  const int t0 = r_begin + pb_h;
  const int ib0 = t0 >= 0 ? t0 / 2 : -((1 - t0) / 2);  // floor(t0 / 2)
  const int ib1 = (r_begin + rows - 1 + pb_h) / 2;
  const int nbr = ib1 - ib0 + 1;
  const int total = nbr * Wo * CH;
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    const int part = e % CH;
    const int jb = (e / CH) % Wo;
    const int ib = ib0 + e / (CH * Wo);
    uint32_t cw[4][2];  // codes of windows (i,j), (i-1,j), (i,j-1), (i-1,j-1)
    uint32_t vw[4][4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int i = ib - (w & 1), j = jb - (w >> 1);
      if (i >= i_lo && i <= i_hi && j >= 0) {
        const int o = ((i - i_lo) * Wo + j) * COUT + part * 8;
        const uint2 c = *reinterpret_cast<const uint2*>(g_s + o);
        const uint4 v = *reinterpret_cast<const uint4*>(p_s + o);
        cw[w][0] = c.x; cw[w][1] = c.y;
        vw[w][0] = v.x; vw[w][1] = v.y; vw[w][2] = v.z; vw[w][3] = v.w;
      } else {
        cw[w][0] = cw[w][1] = 0xFFFFFFFFu;  // matches no code
        vw[w][0] = vw[w][1] = vw[w][2] = vw[w][3] = 0;
      }
    }
    float cell[4][8];  // (a,b) = (0,0), (0,1), (1,0), (1,1)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v[4];
      int code[4];
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const uint32_t u = vw[w][k >> 1];
        v[w] = __uint_as_float((k & 1) ? (u & 0xFFFF0000u) : (u << 16));
        code[w] = (cw[w][k >> 2] >> (8 * (k & 3))) & 0xFF;
      }
      cell[3][k] = code[0] == 4 ? v[0] : 0.f;
      cell[1][k] = (code[0] == 1 ? v[0] : 0.f) + (code[1] == 7 ? v[1] : 0.f);
      cell[2][k] = (code[0] == 3 ? v[0] : 0.f) + (code[2] == 5 ? v[2] : 0.f);
      cell[0][k] = (code[0] == 0 ? v[0] : 0.f) + (code[1] == 6 ? v[1] : 0.f) +
                   (code[2] == 2 ? v[2] : 0.f) + (code[3] == 8 ? v[3] : 0.f);
    }
#pragma unroll
    for (int cidx = 0; cidx < 4; ++cidx) {
      const int rr = 2 * ib - pb_h + (cidx >> 1) - r_begin;
      const int cc = 2 * jb - pb_w + (cidx & 1);
      if (rr >= 0 && rr < rows && cc >= 0 && cc < W) {
        uint4 o;
        o.x = pack_bf16x2(cell[cidx][0], cell[cidx][1]);
        o.y = pack_bf16x2(cell[cidx][2], cell[cidx][3]);
        o.z = pack_bf16x2(cell[cidx][4], cell[cidx][5]);
        o.w = pack_bf16x2(cell[cidx][6], cell[cidx][7]);
        *reinterpret_cast<uint4*>(d_s + rr * RPd + (cc + 1) * COUT + part * 8) = o;
      }
    }
  }
}

__host__ __device__ __forceinline__ void pooled_rows(int r_begin, int rows,
                                                     int pb_h, int Hp, int* lo,
                                                     int* hi) {
  const int a = r_begin + pb_h - 1;
  *lo = a < 0 ? 0 : a / 2;
  int h = (r_begin + rows - 1 + pb_h) / 2;
  *hi = h > Hp - 1 ? Hp - 1 : h;
}

template <int CIN, int COUT, bool NEED_DX, int HC, int WC, int RC>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2))) void pool_conv_bwd_kernel(
    const bf16_t* __restrict__ dP, const uint8_t* __restrict__ argmax,
    const bf16_t* __restrict__ x, const float* __restrict__ w,
    bf16_t* __restrict__ dx, float* __restrict__ dw, float* __restrict__ db,
    int N, int H_, int W_, int R_, int pb_h, int pb_w, int xcd,
    float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = HC ? HC : H_, W = WC ? WC : W_, R = RC ? RC : R_;
  const int Hp = (H + 1) / 2, Wo = (W + 1) / 2;
  const int d_elems = (R + 2) * row_pitch(COUT, W);
  const int x_elems = (R + 2) * row_pitch(CIN, W);
  const int prow_max = (R + 2) / 2 + 2;
  bf16_t* w_s = reinterpret_cast<bf16_t*>(smem);
  bf16_t* d_s = w_s + w_lds_elems(CIN, COUT, false);
  bf16_t* x_s = d_s + d_elems + COUT;
  bf16_t* p_s = x_s + x_elems + CIN;
  uint8_t* g_s = reinterpret_cast<uint8_t*>(p_s + prow_max * Wo * COUT);
  load_weights4<CIN, COUT, false>(w, w_s);
  for (int e = threadIdx.x; e < COUT; e += blockDim.x) d_s[d_elems + e] = 0;
  for (int e = threadIdx.x; e < CIN; e += blockDim.x) x_s[x_elems + e] = 0;
  WgradAcc<CIN, COUT> acc;
  acc.zero();
  const int tpi = (H + R - 1) / R;
  const int ntiles = N * tpi;
  RowStager<CIN, NREG> sx;
  SpanStager<NREG> sp, sg;
  const int prow_bytes = Wo * COUT;
  auto issue = [&](int t) {
    const int n = t / tpi, r0 = (t - n * tpi) * R, Rv = min(R, H - r0);
    sx.issue(x, n, H, W, r0 - 1, Rv + 2);
    int lo, hi;
    pooled_rows(r0 - 1, Rv + 2, pb_h, Hp, &lo, &hi);
    const int64_t prow0 = static_cast<int64_t>(n) * Hp + lo;
    sp.issue(reinterpret_cast<const uint8_t*>(dP), prow0 * prow_bytes * 2,
             (hi - lo + 1) * prow_bytes * 2);
    sg.issue(argmax, prow0 * prow_bytes, (hi - lo + 1) * prow_bytes);
  };
  const TileIter it(ntiles, xcd);
  int tile = it.first;
  if (it.valid(tile)) issue(tile);
  for (; it.valid(tile); tile = it.next(tile)) {
    const int n = tile / tpi, r0 = (tile - n * tpi) * R, Rv = min(R, H - r0);
    int lo, hi;
    pooled_rows(r0 - 1, Rv + 2, pb_h, Hp, &lo, &hi);
    __syncthreads();
    if (kKeep(xcd, 8))
    sx.template commit<false, true>(x_s, W);
    if (kKeep(xcd, 8))
    sp.commit(reinterpret_cast<uint8_t*>(p_s));
    if (kKeep(xcd, 8))
    sg.commit(g_s);
    __syncthreads();
    // unconditional (no next tile: re-issue this one, unused) - a conditional
    // issue leaves a join at the loop back-edge
    issue(it.valid(it.next(tile)) ? it.next(tile) : tile);
    if (kKeep(xcd, 1))
    gather_pool_grad_blocks<COUT>(p_s, g_s, lo, hi, W, Wo, pb_h, pb_w, r0 - 1,
                                  Rv + 2, d_s);
    __syncthreads();
    const int npix = Rv * W;
    if (NEED_DX) {
      const int64_t img0 = (static_cast<int64_t>(n) * H + r0) * W;
    if (kKeep(xcd, 4))
      conv_tile_dgrad<CIN, COUT>(d_s, w_s, W, npix, [&](int q, int ci0, float v[4], int) {
        store4_pk(dx + (img0 + q) * CIN + ci0, v);
      });
    }
    if (kKeep(xcd, 2))
    conv_tile_wgrad<CIN, COUT>(x_s, d_s, W, npix, x_elems, d_elems, acc);
  }
  flush_wgrad<CIN, COUT>(acc, 1.f, dw, db, reinterpret_cast<float*>(smem), part);
}

// First-layer weight gradient on the bf16x4 frame tile: for each kernel row
// ky, D[m = 4 kx + ci][co] += X4[p + (ky-1, kx-1)][ci] dY[p][co]; the A tile
// (4 pixels x 16 contiguous values = kx 0..3 x ci 0..3) and dY both come from
// transposed LDS reads.  Scaled by 1/255 at the flush.  CPX input channels
// (3 RGB, 4 stacked frames).
template <int CPX, int HC, int WC, int RC>
__global__ __launch_bounds__(kThreads) void conv1_pool_bwd_kernel(
    const bf16_t* __restrict__ dP, const uint8_t* __restrict__ argmax,
    const uint8_t* __restrict__ x, float* __restrict__ dw,
    float* __restrict__ db, int N, int H_, int W_, int R_, int pb_h, int pb_w,
    int xcd, float* __restrict__ part) {
  constexpr int COUT = 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = HC ? HC : H_, W = WC ? WC : W_, R = RC ? RC : R_;
  const int Wp = W + 2;
  const int Hp = (H + 1) / 2, Wo = (W + 1) / 2;
  const int d_elems = (R + 2) * Wp * COUT;
  const int prow_max = (R + 2) / 2 + 2;
  bf16_t* d_s = reinterpret_cast<bf16_t*>(smem);
  bf16_t* x4 = d_s + d_elems + COUT;                     // [(R+2)][W+2][4] + pad
  bf16_t* p_s = x4 + (((R + 2) * Wp + 4 + 1) & ~1) * 4;  // keep 16-B alignment
  uint8_t* g_s = reinterpret_cast<uint8_t*>(p_s + prow_max * Wo * COUT);
  for (int e = threadIdx.x; e < COUT; e += blockDim.x) d_s[d_elems + e] = 0;
  const int lane = lane_id();
  const int wave = wave_id();
  const int sub = lane & 15;
  f4 accw[3] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f},
                f4{0.f, 0.f, 0.f, 0.f}};
  f4 accb = f4{0.f, 0.f, 0.f, 0.f};
  s4 ones;
  ones[0] = ones[1] = ones[2] = ones[3] = 0x3F80;
  const int tpi = (H + R - 1) / R;
  const int ntiles = N * tpi;
  U8Stager<kU8Groups, CPX> sx;
  SpanStager<NREG> sp, sg;
  const int prow_bytes = Wo * COUT;
  auto issue = [&](int t) {
    const int n = t / tpi, r0 = (t - n * tpi) * R, Rv = min(R, H - r0);
    sx.issue(x, n, H, W, r0 - 1, Rv + 2);
    int lo, hi;
    pooled_rows(r0 - 1, Rv + 2, pb_h, Hp, &lo, &hi);
    const int64_t prow0 = static_cast<int64_t>(n) * Hp + lo;
    sp.issue(reinterpret_cast<const uint8_t*>(dP), prow0 * prow_bytes * 2,
             (hi - lo + 1) * prow_bytes * 2);
    sg.issue(argmax, prow0 * prow_bytes, (hi - lo + 1) * prow_bytes);
  };
  const TileIter it(ntiles, xcd);
  int tile = it.first;
  if (it.valid(tile)) issue(tile);
  for (; it.valid(tile); tile = it.next(tile)) {
    const int n = tile / tpi, r0 = (tile - n * tpi) * R, Rv = min(R, H - r0);
    int lo, hi;
    pooled_rows(r0 - 1, Rv + 2, pb_h, Hp, &lo, &hi);
    __syncthreads();
    if (kKeep(xcd, 8))
    commit_x4(sx, x4, W, Rv + 2, 4);
    if (kKeep(xcd, 8))
    sp.commit(reinterpret_cast<uint8_t*>(p_s));
    if (kKeep(xcd, 8))
    sg.commit(g_s);
    __syncthreads();
    // unconditional (no next tile: re-issue this one, unused) - a conditional
    // issue leaves a join at the loop back-edge
    issue(it.valid(it.next(tile)) ? it.next(tile) : tile);
    const int npix = Rv * W;
    if (kKeep(xcd, 1))
    gather_pool_grad_blocks<COUT>(p_s, g_s, lo, hi, W, Wo, pb_h, pb_w, r0 - 1,
                                  Rv + 2, d_s);
    __syncthreads();
    const int ngroups = (npix + 15) / 16;
    for (int g = wave; g < (kKeep(xcd, 2) ? ngroups : 0); g += kWaves) {
      const int qb = g * 16 + 4 * (lane >> 4) + (sub >> 2);
      const bool vb = qb < npix;
      const int qbr = vb ? qb / W : 0, qbc = vb ? qb - qbr * W : 0;
      const s4 bd = lds_tr4(d_s + (vb ? ((qbr + 1) * Wp + qbc + 1) * COUT : d_elems) +
                            (sub & 3) * 4);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        // row = pixel qb (invalid pixels read halo zeros of row 0), columns =
        // 16 contiguous values starting at x4 pixel (qbr+ky, qbc) -> (kx, ci)
        const int prow = vb ? (qbr + ky) * Wp + qbc : 0;
        const s4 aa = lds_tr4(x4 + (prow + (sub & 3)) * 4);
        accw[ky] = mfma16(aa, bd, accw[ky]);
      }
      accb = mfma16(ones, bd, accb);
    }
  }
  // deterministic mode: one slot per WAVE (27*16 + 16 floats), reduced in a
  // fixed order by slot_reduce_kernel; otherwise float atomics
  float* slot = part ? part + (static_cast<int64_t>(blockIdx.x) * kWaves + wave) *
                                  (9 * CPX * COUT + COUT)
                     : nullptr;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kx = lane >> 4, ci = i;
      if (kx < 3 && ci < CPX) {
        const int o = ((ky * 3 + kx) * CPX + ci) * COUT + sub;
        const float v = accw[ky][i] * (1.0f / 255.0f);
        if (slot) slot[o] = v;
        else atomicAdd(dw + o, v);
      }
    }
  if ((lane >> 4) == 0) {
    if (slot) slot[9 * CPX * COUT + sub] = accb[0];
    else atomicAdd(db + sub, accb[0]);
  }
}

// dw[e] (e < ndw) / db[e - ndw] += sum over S slots of part[s][e], in a fixed
// order (deterministic mode of the wgrad flushes): thread = element x one of
// 4 slot groups, 8 independent accumulators, the groups combined in LDS.
__global__ __launch_bounds__(256) void slot_reduce_kernel(
    const float* __restrict__ part, int S, int nel, int ndw, float* __restrict__ dw,
    float* __restrict__ db) {
  __shared__ float red[4][64];
  const int e = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sg = threadIdx.x >> 6;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (e < nel) {
    for (int k = sg; k < S; k += 32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int kk = k + 4 * u;
        if (kk < S) acc[u] += part[static_cast<int64_t>(kk) * nel + e];
      }
    }
  }
  red[sg][threadIdx.x & 63] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) +
                              ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (sg != 0 || e >= nel) return;
  const int l = threadIdx.x;
  const float v = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
  if (e < ndw) dw[e] += v;
  else db[e - ndw] += v;
}

int num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 0;
    if (cus <= 0) cus = 256;  // MI355X
  }
  return cus;
}

// Persistent grid: enough workgroups for `per_cu` resident per CU, on the
// CUs the fp32 torso's grids use too (conv_f32.hip conv_cus: all but the
// CUs per XCD reserved for a concurrent stream, cf32_cu_reserve).
int grid_for(int ntiles, size_t smem, int per_cu_cap) {
  int per_cu = static_cast<int>((160 * 1024) / (smem + 1024));
  if (per_cu > per_cu_cap) per_cu = per_cu_cap;
  if (per_cu < 1) per_cu = 1;
  const int reserved = num_cus() - sa::cf32::conv_cus();  // 8 R on MI355X
  const int g = (num_cus() - reserved) * per_cu;
  return ntiles < g ? ntiles : g;
}

template <typename K>
void set_smem(K kernel, size_t bytes) {
  if (bytes > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          static_cast<int>(bytes)) != hipSuccess)
    (void)hipGetLastError();  // the launch itself reports an LDS request it cannot meet
}

// ----- tile-height rules (constexpr: the same rule picks the compiled
// geometry at build time and the runtime tile height at launch) -----------

// SA_ROWS_BALANCE=1: when a rule's tallest fitting tile R leaves a last tile
// of under R / 4 rows, the image's ceil(H / R) tiles are made equally tall
// (ceil(H / n) rows): the same number of tiles and staged halo rows without
// the sliver (Atari 21 rows: 7+7+7 instead of 10+10+1; 42 rows of the
// 16->32 head backward: 9+9+9+9+6 instead of 10+10+10+10+2).  Measured
// (bf16 learner, one box, 3 runs per arm): Atari 84x84x4 4.767-4.779 ->
// 4.714-4.731 ms with every tile balanced; balancing the IMPALA 18x24 maps
// too (8+8+2 -> 6+6+6) cost the 72x96 learner 0.02-0.04 ms, hence the R / 4
// threshold, which leaves every 72x96 tile unchanged.
#ifndef SA_ROWS_BALANCE
#define SA_ROWS_BALANCE 1
#endif
constexpr int balance_rows(int H, int R) {
  if (!SA_ROWS_BALANCE || R >= H || R < 1) return R;
  const int n = (H + R - 1) / R;
  const int last = H - (n - 1) * R;
  return 4 * last < R ? (H + n - 1) / n : R;
}

// rows per tile such that the staged halo fits NREG*256 16-B chunks per
// stream and the tile holds ~target pixels
constexpr int rows_for(int H, int W, int C, int target) {
  int R = target / W;
  if (R < 1) R = 1;
  while (R > 1 && ((R + 2) * W * C / 8 > NREG * kThreads ||
                   tile_groups(C, R, W) > kMaxTilePx(C) / 16))
    --R;
  return balance_rows(H, R < H ? R : H);
}
// fused residual block: x staged with 2 halo rows each side, t computed
// for R + 2 rows
constexpr int rows_block(int H, int W, int C, int target) {
  int R = target / W;
  if (R < 1) R = 1;
  while (R > 1 && ((R + 4) * W * C / 8 > NREG * kThreads ||
                   tile_groups(C, R + 2, W) > kMaxTilePx(C) / 16))
    --R;
  return R < H ? R : H;
}
constexpr int rows_pool_fwd(int H, int W, int CIN, int px) {
  const int Hp = (H + 1) / 2;
  int Rp = (px / W - 1) / 2;
  if (Rp < 1) Rp = 1;
  while (Rp > 1 && ((2 * Rp + 3) * W * CIN / 8 > NREG * kThreads ||
                    tile_groups(CIN, 2 * Rp + 1, W) > kMaxTilePx(CIN) / 16))
    --Rp;
  return balance_rows(Hp, Rp > Hp ? Hp : Rp);
}
// LDS bytes of conv1_pool_fwd_kernel at Rp pooled rows (its launcher's smem)
constexpr int conv1_fwd_lds(int Rp, int W) {
  return (3 * 16 * 16 + (2 * Rp + 1) * (W + 2) * 16 + ((2 * Rp + 3) * (W + 2) + 4) * 4) * 2;
}
constexpr int rows_conv1_fwd(int H, int W, int px) {
  const int Hp = (H + 1) / 2;
  int Rp = (px / W - 1) / 2;
  if (Rp < 1) Rp = 1;
  while (Rp > 1 && ((2 * Rp + 3) * W + 3) / 4 > kU8Groups * kThreads) --Rp;
  // four forward workgroups per CU (ConvTune::cap_fwd) must fit in its LDS
  while (Rp > 1 && conv1_fwd_lds(Rp, W) * 4 > 160 * 1024) --Rp;
  return balance_rows(Hp, Rp > Hp ? Hp : Rp);
}
constexpr int rows_pool_bwd(int H, int W, int CIN, int COUT, int px) {
  const int Wo = (W + 1) / 2;
  int R = rows_for(H, W, CIN, px);
  while (R > 1 && (((R + 2) / 2 + 2) * Wo * COUT * 2 > NREG * kThreads * 16 ||
                   tile_groups(COUT, R, W) > kMaxTilePx(CIN < COUT ? CIN : COUT) / 16))
    --R;
  return balance_rows(H, R);
}
constexpr int rows_conv1_bwd(int H, int W, int px) {
  const int Wo = (W + 1) / 2;
  int R = px / W;
  if (R < 1) R = 1;
  while (R > 1 && (((R + 2) / 2 + 2) * Wo * 16 * 2 > NREG * kThreads * 16 ||
                   ((R + 2) * W + 3) / 4 > kU8Groups * kThreads))
    --R;
  return balance_rows(H, R > H ? H : R);
}

// Host-side guard: the tile-height rules stop at one row, so a frame too wide
// for even a one-row tile must be rejected (the kernels assume the staged
// halo fits their staging registers and kMaxTilePx).
void require_fit(bool ok, const char* what) {
  if (!ok)
    throw std::invalid_argument(std::string(what) +
                                ": frame too wide for the conv tile staging");
}

}  // namespace

// ----------------------------------------------------------------- launchers
// Launch-shape knobs (defaults = the tuned configuration); exposed for
// measurement through conv_tune_set (tools/conv_bench.py).  Changing a tile
// knob away from its default makes the launchers fall back to the
// runtime-geometry kernels.
struct ConvTune {
  int xcd = 1;            // XCD-aware contiguous tile ranges
  int cap_fwd = 4;        // max resident workgroups per CU, forward kernels
  int cap_bwd = 2;        // ... backward kernels
  int px_res_fwd = 384;   // target pixels per tile
  int px_res_bwd = 384;
  int px_pool_fwd = 400;  // conv pixels per tile (pre-pool)
  // stage 0: 4 pooled rows at W = 96 and 84 (84x84: 5 rows measured 4 %
  // slower), 12 conv rows at 96 and 14 (6 equal tiles) at 84 (13 rows: 7 %
  // slower, tools/micro/conv1_probe.py SWEEP=1)
  int px_conv1_fwd = 900;
  int px_pool_bwd = 512;
  int px_conv1_bwd = 1176;
  int specialize = 1;     // use compile-time-geometry kernels when they match
  int ablate = 0;         // timing-only, -DSA_CONV_ABLATE builds: skip phases
  int deterministic = 0;  // wgrad: per-workgroup slots + fixed-order reduce
};
constexpr ConvTune kDef{};
static ConvTune g_tune;

int conv_tune_set(const char* key, int value) {
  struct { const char* k; int* v; } table[] = {
      {"xcd", &g_tune.xcd}, {"cap_fwd", &g_tune.cap_fwd},
      {"cap_bwd", &g_tune.cap_bwd}, {"px_res_fwd", &g_tune.px_res_fwd},
      {"px_res_bwd", &g_tune.px_res_bwd}, {"px_pool_fwd", &g_tune.px_pool_fwd},
      {"px_conv1_fwd", &g_tune.px_conv1_fwd},
      {"px_pool_bwd", &g_tune.px_pool_bwd},
      {"px_conv1_bwd", &g_tune.px_conv1_bwd},
      {"specialize", &g_tune.specialize}, {"ablate", &g_tune.ablate},
      {"deterministic", &g_tune.deterministic}};
  for (auto& e : table) {
    if (std::strcmp(e.k, key) == 0) {
      const int old = *e.v;
      if (value >= 0) *e.v = value;
      return old;
    }
  }
  return -1;
}

namespace {

template <int V>
using IC = std::integral_constant<int, V>;

// Compiled geometries: the IMPALA frame (72x96), the Doom frame (72x128) and
// the Atari frame (84x84: BASELINE config #2) at every torso stage.  f(IC<H>, IC<W>, IC<R>) is called with the matching
// compile-time geometry, or with zeros (runtime shapes).
template <int HH, int WW, int RR, typename F>
bool geo_try(int H, int W, int R, F& f) {
  if (H == HH && W == WW && R == RR) {
    f(IC<HH>{}, IC<WW>{}, IC<RR>{});
    return true;
  }
  return false;
}

enum Stage { kConv1, kStage1, kStage2, kStage3 };

// R(H, W) for a kernel family, as a constexpr functor.
template <int STAGE, typename RF, typename F>
void with_geo(int H, int W, int R, F&& f) {
  if (g_tune.specialize) {
    if constexpr (STAGE == kConv1) {
      if (geo_try<72, 96, RF::rows(72, 96)>(H, W, R, f)) return;
      if (geo_try<72, 128, RF::rows(72, 128)>(H, W, R, f)) return;
      if (geo_try<84, 84, RF::rows(84, 84)>(H, W, R, f)) return;
    } else if constexpr (STAGE == kStage1) {
      if (geo_try<36, 48, RF::rows(36, 48)>(H, W, R, f)) return;
      if (geo_try<36, 64, RF::rows(36, 64)>(H, W, R, f)) return;
      if (geo_try<42, 42, RF::rows(42, 42)>(H, W, R, f)) return;
    } else if constexpr (STAGE == kStage2) {
      if (geo_try<18, 24, RF::rows(18, 24)>(H, W, R, f)) return;
      if (geo_try<18, 32, RF::rows(18, 32)>(H, W, R, f)) return;
      if (geo_try<21, 21, RF::rows(21, 21)>(H, W, R, f)) return;
    } else {
      if (geo_try<9, 12, RF::rows(9, 12)>(H, W, R, f)) return;
      if (geo_try<9, 16, RF::rows(9, 16)>(H, W, R, f)) return;
      if (geo_try<11, 11, RF::rows(11, 11)>(H, W, R, f)) return;
    }
  }
  f(IC<0>{}, IC<0>{}, IC<0>{});
}

template <int C>
struct RowsResFwd {
  static constexpr int rows(int H, int W) { return rows_for(H, W, C, kDef.px_res_fwd); }
};
template <int C>
struct RowsBlockFwd {
  static constexpr int rows(int H, int W) { return rows_block(H, W, C, kDef.px_res_fwd); }
};
template <int C>
struct RowsResBwd {
  static constexpr int rows(int H, int W) { return rows_for(H, W, C, kDef.px_res_bwd); }
};
template <int CIN>
struct RowsPoolFwd {
  static constexpr int rows(int H, int W) { return rows_pool_fwd(H, W, CIN, kDef.px_pool_fwd); }
};
struct RowsConv1Fwd {
  static constexpr int rows(int H, int W) { return rows_conv1_fwd(H, W, kDef.px_conv1_fwd); }
};
template <int CIN, int COUT>
struct RowsPoolBwd {
  static constexpr int rows(int H, int W) {
    return rows_pool_bwd(H, W, CIN, COUT, kDef.px_pool_bwd);
  }
};
struct RowsConv1Bwd {
  static constexpr int rows(int H, int W) { return rows_conv1_bwd(H, W, kDef.px_conv1_bwd); }
};

}  // namespace

int res_conv_rows(int H, int W) { return rows_for(H, W, 32, g_tune.px_res_fwd); }

void res_block_fwd_launch(const void* x, const float* w1, const float* b1,
                          const float* w2, const float* b2, void* t, void* y,
                          int N, int H, int W, int C, bool post_relu,
                          hipStream_t s) {
  const int R = rows_block(H, W, C, g_tune.px_res_fwd);
  require_fit((R + 4) * W * C / 8 <= NREG * kThreads &&
                  tile_groups(C, R + 2, W) <= kMaxTilePx(C) / 16,
              "res_block_fwd");
  const int ntiles = N * ((H + R - 1) / R);
  const size_t smem = (2 * w_lds_elems(C, C, true) + (R + 4) * row_pitch(C, W) + C +
                       (R + 2) * row_pitch(C, W) + C) * sizeof(bf16_t);
  const int grid = grid_for(ntiles, smem, g_tune.cap_fwd);
  auto X = static_cast<const bf16_t*>(x);
  auto Tt = static_cast<bf16_t*>(t);
  auto Y = static_cast<bf16_t*>(y);
  const int xcd = g_tune.xcd | (g_tune.ablate << 8);
  auto go = [&](auto kernel) {
    set_smem(kernel, smem);
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kThreads), smem, s, X, w1, b1,
                       w2, b2, Tt, Y, N, H, W, R, xcd);
  };
#define SA_RB(CC, PR, STG)                                                     \
  with_geo<STG, RowsBlockFwd<CC>>(H, W, R, [&](auto h, auto ww, auto r) {      \
    go(res_block_fwd_kernel<CC, PR, decltype(h)::value, decltype(ww)::value,   \
                            decltype(r)::value>);                              \
  })
  if (C == 16) {
    if (post_relu) SA_RB(16, true, kStage1); else SA_RB(16, false, kStage1);
  } else if (H * 2 > 18 + 9) {
    if (post_relu) SA_RB(32, true, kStage2); else SA_RB(32, false, kStage2);
  } else {
    if (post_relu) SA_RB(32, true, kStage3); else SA_RB(32, false, kStage3);
  }
#undef SA_RB
}

void res_conv_fwd_launch(const void* x, const float* w, const float* b,
                         const void* resid, void* y, int N, int H, int W,
                         int C, bool post_relu, bool relu_in, hipStream_t s) {
  const int R = rows_for(H, W, C, g_tune.px_res_fwd);
  require_fit((R + 2) * W * C / 8 <= NREG * kThreads &&
                  tile_groups(C, R, W) <= kMaxTilePx(C) / 16,
              "res_conv_fwd");
  const int ntiles = N * ((H + R - 1) / R);
  const size_t smem = (w_lds_elems(C, C, true) + (R + 2) * row_pitch(C, W) + C) * sizeof(bf16_t);
  const int grid = grid_for(ntiles, smem, g_tune.cap_fwd);
  auto X = static_cast<const bf16_t*>(x);
  auto RS = static_cast<const bf16_t*>(resid);
  auto Y = static_cast<bf16_t*>(y);
  const int xcd = g_tune.xcd | (g_tune.ablate << 8);
  auto go = [&](auto kernel) {
    set_smem(kernel, smem);
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kThreads), smem, s, X, w, b,
                       RS, Y, N, H, W, R, xcd);
  };
#define SA_RF(CC, RE, PR, RI, STG)                                             \
  with_geo<STG, RowsResFwd<CC>>(H, W, R, [&](auto h, auto ww, auto r) {        \
    go(res_conv_fwd_kernel<CC, RE, PR, RI, decltype(h)::value,                 \
                           decltype(ww)::value, decltype(r)::value>);          \
  })
  // Instantiated combinations: (relu_in, resid, post_relu) in
  //   {(1,0,*): block conv 1, (0,1,*): block conv 2, (1,1,*): reference form}
  const bool re = resid != nullptr;
#define SA_RF_C(CC, STG)                                                       \
  if (relu_in && !re && !post_relu) SA_RF(CC, false, false, true, STG);        \
  else if (relu_in && !re) SA_RF(CC, false, true, true, STG);                  \
  else if (relu_in && !post_relu) SA_RF(CC, true, false, true, STG);           \
  else if (relu_in) SA_RF(CC, true, true, true, STG);                          \
  else if (re && !post_relu) SA_RF(CC, true, false, false, STG);               \
  else if (re) SA_RF(CC, true, true, false, STG);                              \
  else if (!post_relu) SA_RF(CC, false, false, false, STG);                   \
  else SA_RF(CC, false, true, false, STG)
  if (C == 16) {
    SA_RF_C(16, kStage1);
  } else if (H * 2 > 18 + 9) {
    SA_RF_C(32, kStage2);
  } else {
    SA_RF_C(32, kStage3);
  }
#undef SA_RF_C
#undef SA_RF
}

void conv_pool_fwd_launch(const void* x, const float* w, const float* b,
                          void* pooled, uint8_t* argmax, int N, int H, int W,
                          int CIN, int COUT, int pb_h, int pb_w, hipStream_t s) {
  const int Hp = (H + 1) / 2;
  const int Rp = rows_pool_fwd(H, W, CIN, g_tune.px_pool_fwd);
  require_fit((2 * Rp + 3) * W * CIN / 8 <= NREG * kThreads &&
                  tile_groups(CIN, 2 * Rp + 1, W) <= kMaxTilePx(CIN) / 16,
              "conv_pool_fwd");
  const int ntiles = N * ((Hp + Rp - 1) / Rp);
  const size_t smem = (w_lds_elems(CIN, COUT, true) + (2 * Rp + 3) * row_pitch(CIN, W) + CIN +
                       (2 * Rp + 1) * (W + 2) * COUT) * sizeof(bf16_t);
  const int grid = grid_for(ntiles, smem, g_tune.cap_fwd);
  auto X = static_cast<const bf16_t*>(x);
  auto P = static_cast<bf16_t*>(pooled);
  const int xcd = g_tune.xcd | (g_tune.ablate << 8);
  auto go = [&](auto kernel) {
    set_smem(kernel, smem);
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kThreads), smem, s, X, w, b,
                       P, argmax, N, H, W, Rp, pb_h, pb_w, xcd);
  };
#define SA_CP(CI, CO, STG)                                                     \
  with_geo<STG, RowsPoolFwd<CI>>(H, W, Rp, [&](auto h, auto ww, auto r) {      \
    go(conv_pool_fwd_kernel<CI, CO, decltype(h)::value, decltype(ww)::value,   \
                            decltype(r)::value>);                              \
  })
  if (CIN == 16 && COUT == 32) SA_CP(16, 32, kStage1);
  else if (CIN == 32 && COUT == 32) SA_CP(32, 32, kStage2);
  else if (CIN == 16 && COUT == 16) SA_CP(16, 16, kStage1);
#undef SA_CP
}

void conv1_pool_fwd_launch(const uint8_t* x, const float* w, const float* b,
                           void* pooled, uint8_t* argmax, int N, int H, int W,
                           int C, int pb_h, int pb_w, hipStream_t s) {
  const int Hp = (H + 1) / 2;
  const int Rp = rows_conv1_fwd(H, W, g_tune.px_conv1_fwd);
  require_fit(((2 * Rp + 3) * W + 3) / 4 <= kU8Groups * kThreads, "conv1_pool_fwd");
  const int ntiles = N * ((Hp + Rp - 1) / Rp);
  const size_t smem = (3 * 16 * 16 + (2 * Rp + 1) * (W + 2) * 16 +
                       ((2 * Rp + 3) * (W + 2) + 4) * 4) * sizeof(bf16_t);
  const int grid = grid_for(ntiles, smem, g_tune.cap_fwd);
  auto P = static_cast<bf16_t*>(pooled);
  const int xcd = g_tune.xcd | (g_tune.ablate << 8);
  require_fit(C == 3 || C == 4, "conv1_pool_fwd: 3 or 4 frame channels");
  with_geo<kConv1, RowsConv1Fwd>(H, W, Rp, [&](auto h, auto ww, auto r) {
    auto k3 = conv1_pool_fwd_kernel<3, decltype(h)::value, decltype(ww)::value,
                                    decltype(r)::value>;
    auto k4 = conv1_pool_fwd_kernel<4, decltype(h)::value, decltype(ww)::value,
                                    decltype(r)::value>;
    auto k = C == 4 ? k4 : k3;
    set_smem(k, smem);
    hipLaunchKernelGGL(k, dim3(grid), dim3(kThreads), smem, s, x, w, b, P,
                       argmax, N, H, W, Rp, pb_h, pb_w, xcd);
  });
}

// Deterministic mode: floats of the slot workspace a wgrad launch needs (0
// when off); the slots are summed by slot_reduce_kernel after the launch.
int64_t wgrad_part_floats(int cin, int cout, bool conv1) {
  if (!g_tune.deterministic) return 0;
  const int64_t nel = conv1 ? 9 * cin * 16 + 16 : 9 * cin * cout + cout;
  const int64_t slots = static_cast<int64_t>(num_cus()) *
                        std::max(1, std::max(g_tune.cap_bwd, 1)) * (conv1 ? kWaves : 1);
  return slots * nel;
}

static void reduce_slots(const float* part, int slots, int nel, int ndw, float* dw,
                         float* db, hipStream_t s) {
  hipLaunchKernelGGL(slot_reduce_kernel, dim3((nel + 63) / 64), dim3(256), 0, s, part,
                     slots, nel, ndw, dw, db);
}

void res_conv_bwd_launch(const void* dy, const void* act, const void* skip,
                         const float* w, void* dx, float* dw, float* db, int N,
                         int H, int W, int C, bool relu_act, hipStream_t s,
                         float* part) {
  const int R = rows_for(H, W, C, g_tune.px_res_bwd);
  require_fit((R + 2) * W * C / 8 <= NREG * kThreads &&
                  tile_groups(C, R, W) <= kMaxTilePx(C) / 16,
              "res_conv_bwd");
  const int ntiles = N * ((H + R - 1) / R);
  const size_t smem = (w_lds_elems(C, C, false) + 2 * ((R + 2) * row_pitch(C, W) + C)) * sizeof(bf16_t);
  const int grid = grid_for(ntiles, smem, g_tune.cap_bwd);
  auto DY = static_cast<const bf16_t*>(dy);
  auto A = static_cast<const bf16_t*>(act);
  auto SK = static_cast<const bf16_t*>(skip);
  auto DX = static_cast<bf16_t*>(dx);
  const int xcd = g_tune.xcd | (g_tune.ablate << 8);
  auto go = [&](auto kernel) {
    set_smem(kernel, smem);
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kThreads), smem, s, DY, A, SK,
                       w, DX, dw, db, N, H, W, R, xcd, part);
  };
#define SA_RB(CC, SKP, RA, STG)                                                \
  with_geo<STG, RowsResBwd<CC>>(H, W, R, [&](auto h, auto ww, auto r) {        \
    go(res_conv_bwd_kernel<CC, SKP, RA, decltype(h)::value,                    \
                           decltype(ww)::value, decltype(r)::value>);          \
  })
#define SA_RB_C(CC, STG)                                                       \
  if (skip && relu_act) SA_RB(CC, true, true, STG);                            \
  else if (skip) SA_RB(CC, true, false, STG);                                  \
  else if (relu_act) SA_RB(CC, false, true, STG);                              \
  else SA_RB(CC, false, false, STG)
  if (C == 16) {
    SA_RB_C(16, kStage1);
  } else if (H * 2 > 18 + 9) {
    SA_RB_C(32, kStage2);
  } else {
    SA_RB_C(32, kStage3);
  }
#undef SA_RB_C
#undef SA_RB
  if (part) reduce_slots(part, grid, 9 * C * C + C, 9 * C * C, dw, db, s);
}

void pool_conv_bwd_launch(const void* dP, const uint8_t* argmax, const void* x,
                          const float* w, void* dx, float* dw, float* db, int N,
                          int H, int W, int CIN, int COUT, int pb_h, int pb_w,
                          hipStream_t s, float* part) {
  const int Wo = (W + 1) / 2;
  const int R = rows_pool_bwd(H, W, CIN, COUT, g_tune.px_pool_bwd);
  require_fit((R + 2) * W * CIN / 8 <= NREG * kThreads &&
                  tile_groups(COUT, R, W) <= kMaxTilePx(CIN < COUT ? CIN : COUT) / 16 &&
                  ((R + 2) / 2 + 2) * Wo * COUT * 2 <= NREG * kThreads * 16,
              "pool_conv_bwd");
  const int prow_max = (R + 2) / 2 + 2;
  const int ntiles = N * ((H + R - 1) / R);
  const size_t smem = (w_lds_elems(CIN, COUT, false) +
                       (R + 2) * (row_pitch(CIN, W) + row_pitch(COUT, W)) +
                       CIN + COUT + prow_max * Wo * COUT) * sizeof(bf16_t) +
                      prow_max * Wo * COUT;
  const int grid = grid_for(ntiles, smem, g_tune.cap_bwd);
  auto DP = static_cast<const bf16_t*>(dP);
  auto X = static_cast<const bf16_t*>(x);
  auto DX = static_cast<bf16_t*>(dx);
  const int xcd = g_tune.xcd | (g_tune.ablate << 8);
  auto go = [&](auto kernel) {
    set_smem(kernel, smem);
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kThreads), smem, s, DP, argmax,
                       X, w, DX, dw, db, N, H, W, R, pb_h, pb_w, xcd, part);
  };
#define SA_PB(CI, CO, NDX, STG)                                                \
  with_geo<STG, RowsPoolBwd<CI, CO>>(H, W, R, [&](auto h, auto ww, auto r) {   \
    go(pool_conv_bwd_kernel<CI, CO, NDX, decltype(h)::value,                   \
                            decltype(ww)::value, decltype(r)::value>);         \
  })
  const bool ndx = dx != nullptr;
  if (CIN == 16 && COUT == 32) {
    if (ndx) SA_PB(16, 32, true, kStage1);
    else SA_PB(16, 32, false, kStage1);
  } else if (CIN == 32 && COUT == 32) {
    if (ndx) SA_PB(32, 32, true, kStage2);
    else SA_PB(32, 32, false, kStage2);
  } else if (CIN == 16 && COUT == 16) {
    if (ndx) SA_PB(16, 16, true, kStage1);
    else SA_PB(16, 16, false, kStage1);
  }
#undef SA_PB
  if (part)
    reduce_slots(part, grid, 9 * CIN * COUT + COUT, 9 * CIN * COUT, dw, db, s);
}

void conv1_pool_bwd_launch(const void* dP, const uint8_t* argmax,
                           const uint8_t* x, float* dw, float* db, int N,
                           int H, int W, int C, int pb_h, int pb_w, hipStream_t s,
                           float* part) {
  const int Wo = (W + 1) / 2;
  const int R = rows_conv1_bwd(H, W, g_tune.px_conv1_bwd);
  require_fit(((R + 2) * W + 3) / 4 <= kU8Groups * kThreads &&
                  ((R + 2) / 2 + 2) * ((W + 1) / 2) * 16 * 2 <= NREG * kThreads * 16,
              "conv1_pool_bwd");
  const int prow_max = (R + 2) / 2 + 2;
  const int ntiles = N * ((H + R - 1) / R);
  const size_t smem = ((R + 2) * (W + 2) * 16 + 16 + (((R + 2) * (W + 2) + 5) & ~1) * 4 +
                       prow_max * Wo * 16) * sizeof(bf16_t) +
                      prow_max * Wo * 16;
  const int grid = grid_for(ntiles, smem, g_tune.cap_bwd);
  auto DP = static_cast<const bf16_t*>(dP);
  const int xcd = g_tune.xcd | (g_tune.ablate << 8);
  require_fit(C == 3 || C == 4, "conv1_pool_bwd: 3 or 4 frame channels");
  with_geo<kConv1, RowsConv1Bwd>(H, W, R, [&](auto h, auto ww, auto r) {
    auto k3 = conv1_pool_bwd_kernel<3, decltype(h)::value, decltype(ww)::value,
                                    decltype(r)::value>;
    auto k4 = conv1_pool_bwd_kernel<4, decltype(h)::value, decltype(ww)::value,
                                    decltype(r)::value>;
    auto k = C == 4 ? k4 : k3;
    set_smem(k, smem);
    hipLaunchKernelGGL(k, dim3(grid), dim3(kThreads), smem, s, DP, argmax, x,
                       dw, db, N, H, W, R, pb_h, pb_w, xcd, part);
  });
  if (part)
    reduce_slots(part, grid * kWaves, 9 * C * 16 + 16, 9 * C * 16, dw, db, s);
}

}  // namespace conv
}  // namespace sa
