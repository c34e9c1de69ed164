// LSTMBlockCell(256) recurrence with done-reset, fp32.
//
// Reference: experiment.py:228-235 (tf.where(done, zero_state, state) before
// every LSTMBlockCell step) with TF gate order i, c~, f, o and forget bias +1.
// The input projection x_t W_x + b for ALL steps is one hipBLASLt GEMM done by
// the caller; these kernels carry only the serial part:
//
//   fwd step t : gates = xw_t + (keep_t h_{t-1}) W_h ; c_t = f (keep_t c_{t-1})
//                + i g ; h_t = o tanh(c_t)      (saves i, g, f, o and c_t)
//   bwd step t : dh_t = dH_t + keep_{t+1} (dG_{t+1} W_h^T) ; dc_t = dcarry +
//                dh_t o (1 - tanh^2 c_t) ; dG_t = [di, dg, df, do] * act'
//                dcarry' = dc_t f_t keep_t
// dW_h = sum_t (keep_t h_{t-1})^T dG_t and dX are plain GEMMs on the caller.
//
// Latency design: the 101 dependent steps per direction are replayed from a
// hipGraph (~1.6 us per dependent launch on MI355X, measured by
// tools/launch_bench.py), so each step kernel must finish in ~1-2 us.  The
// recurrent product runs on the exact-fp32 MFMA (v_mfma_f32_16x16x4_f32, a
// k-ordered fmaf chain) with BOTH operands loaded straight from global into
// registers (no LDS staging, no bank conflicts); the K dimension is split
// across the waves of the workgroup and reduced once through LDS.
#include "launchers.h"
#include "knobs.h"

#include <hip/hip_bf16.h>

#include <cstdlib>

namespace sa {
namespace {

typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ f4v mfma_f32(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- forward
// Workgroup = 16 gate columns (4 units x 4 gates, packed n = 4u + g) x 32 rows.
// 8 waves; wave w owns k in [H/8 w, H/8 (w+1)).  w4: [H/4][H][16].
// h_pk_in / h_pk_out: h in MFMA-operand order, [row tile][wave][mt][s][lane]
// with lane l <-> (row 16 mt + (l&15), k = KW w + 4 s + (l>>4)): every operand
// load is one contiguous 256-B wave access.
// h_pk_in == nullptr (the first step) reads the A operand straight from the
// unpacked h_prev [B,H] (no host-side packing pass).  hpm_t (optional) gets
// keep_t * h_prev, the A operand of the dW_h = sum_t hpm_t^T dG_t GEMM.
// RW: batch rows per workgroup (32, or 16 = half a packed row tile: twice
// the workgroups, each streaming half of h)
template <int H, int RW = 32, int NW = 8>
__global__ __launch_bounds__(64 * NW) void lstm_fwd_step_kernel(
    const float* __restrict__ xw_t, const float* __restrict__ h_pk_in,
    const float* __restrict__ h_prev, const float* __restrict__ c_prev,
    const uint8_t* __restrict__ done_t, const float* __restrict__ w4,
    float* __restrict__ h_t, float* __restrict__ h_pk_out,
    float* __restrict__ c_t, float* __restrict__ acts_t,
    float* __restrict__ hpm_t, int B, int xpack) {
  static_assert(NW == 8 || NW == 4, "waves per workgroup");
  static_assert(16 * RW <= 64 * NW, "one reduce thread per output");
  constexpr int KW = H / NW;     // k per wave
  constexpr int NS = KW / 4;     // mfma k-steps per wave
  __shared__ f4v red[NW][2][64];  // per wave, per row tile, per lane
  __shared__ float g_s[32][17];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  // xpack > 1: only every xpack-th block works, so with round-robin XCD
  // dispatch all working blocks share one XCD (and its L2)
  if (blockIdx.x % xpack) return;
  const int blk = blockIdx.x / xpack;
  static_assert(RW == 32 || RW == 16, "rows per workgroup");
  constexpr int NMT = RW / 16;  // MFMA row tiles
  const int r0 = blockIdx.y * RW;
  const int t32 = r0 >> 5, mt0 = (r0 >> 4) & 1;  // packed 32-row tile, half
  // epilogue operands (thread = (row r, unit u) for tid < 4 RW)
  const int er = tid >> 2, eu = tid & 3;
  const int egr = r0 + er;
  const int ej = blk * 4 + eu;
  // Every operand load below is issued up front with a clamped (always valid)
  // address and consumed only where it is needed: converting a done byte
  // next to its load (or loading under a per-row branch) made each group of
  // loads wait for all earlier ones, three serialized memory round trips per
  // step instead of one.  The done-reset of the A operand is applied to the
  // reduced product rows instead of to h ((keep h) W == keep (h W) row by
  // row, keep in {0, 1}, selected rather than multiplied: bitwise the same).
  // The done defaults are the (non-constant, nonzero) B: with a constant
  // default the compiler folds the done test into the loading branch, which
  // then waits for the byte right there.
  float xi = 0.f, xc = 0.f, xf = 0.f, xo = 0.f, cp = 0.f, hp = 0.f;
  uint32_t edone = static_cast<uint32_t>(B);
  if (tid < 4 * RW) {
    const int egc = egr < B ? egr : B - 1;
    const int64_t g0 = static_cast<int64_t>(egc) * 4 * H + ej;
    xi = xw_t[g0];
    xc = xw_t[g0 + H];
    xf = xw_t[g0 + 2 * H];
    xo = xw_t[g0 + 3 * H];
    cp = c_prev[static_cast<int64_t>(egc) * H + ej];
    if (hpm_t) hp = h_prev[static_cast<int64_t>(egc) * H + ej];
    edone = done_t[egc];
  }
  // reduce-thread row (tid < 16 RW): its done byte masks the product row
  uint32_t rdone = static_cast<uint32_t>(B);
  if (tid < 16 * RW) {
    const int rg = r0 + (tid >> 4);
    rdone = done_t[rg < B ? rg : B - 1];
  }
  // B operand: W[k = kw0 + 4s + (l>>4)][n = l&15]
  const int kw0 = wave * KW;
  float wb[NS];
  const float* wsrc = w4 + (static_cast<int64_t>(blk) * H + kw0 + (lane >> 4)) * 16 + (lane & 15);
#pragma unroll
  for (int s = 0; s < NS; ++s) wb[s] = wsrc[s * 4 * 16];
  // A operand: h[row = r0 + 16 mt + (l&15)][k = kw0 + 4s + (l>>4)]
  float ha[NMT][NS];
  if (h_pk_in != nullptr) {
    const float* pk = h_pk_in + static_cast<int64_t>(t32) * 32 * H +
                      wave * 2 * NS * 64 + lane;
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
      for (int s = 0; s < NS; ++s) ha[mt][s] = pk[((mt0 + mt) * NS + s) * 64];
  } else {
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) {
      const int row = r0 + 16 * mt + (lane & 15);
      const float* hr = h_prev + static_cast<int64_t>(row < B ? row : B - 1) * H + kw0 + (lane >> 4);
#pragma unroll
      for (int s = 0; s < NS; ++s) ha[mt][s] = hr[4 * s];
    }
  }
  f4v acc[2] = {f4v{0.f, 0.f, 0.f, 0.f}, f4v{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) acc[mt] = mfma_f32(ha[mt][s], wb[s], acc[mt]);
  red[wave][0][lane] = acc[0];
  if (NMT == 2) red[wave][1][lane] = acc[1];
  __syncthreads();
  // reduce: output (row m in 0..RW-1, col n in 0..15); D[m=4(l>>4)+i][n=l&15]
  if (tid < 16 * RW) {
    const int m = tid >> 4, n = tid & 15;  // 512 threads == 32 x 16 outputs
    const int mt = m >> 4, mm = m & 15;
    const int src_lane = ((mm >> 2) << 4) | n;
    const int i = mm & 3;
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) sum += red[w][mt][src_lane][i];
    g_s[m][n] = rdone ? 0.f : sum;
  }
  __syncthreads();
  if (tid < 4 * RW && egr < B) {
    const float ekeep = edone ? 0.f : 1.f;
    const float i = sigm(g_s[er][eu * 4 + 0] + xi);
    const float g = tanhf(g_s[er][eu * 4 + 1] + xc);
    const float f = sigm(g_s[er][eu * 4 + 2] + xf + 1.0f);
    const float o = sigm(g_s[er][eu * 4 + 3] + xo);
    const float c = f * ekeep * cp + i * g;
    const float h = o * tanhf(c);
    const int64_t hj = static_cast<int64_t>(egr) * H + ej;
    const int64_t g0 = static_cast<int64_t>(egr) * 4 * H + ej;
    c_t[hj] = c;
    h_t[hj] = h;
    {  // packed copy for the next step's A operand
      const int k = ej, rr = egr - 32 * t32;
      const int w = k / KW, s2 = (k % KW) >> 2, q = k & 3;
      h_pk_out[static_cast<int64_t>(t32) * 32 * H +
               ((w * 2 + (rr >> 4)) * NS + s2) * 64 + (q << 4) + (rr & 15)] = h;
    }
    acts_t[g0] = i;
    acts_t[g0 + H] = g;
    acts_t[g0 + 2 * H] = f;
    acts_t[g0 + 3 * H] = o;
    if (hpm_t) hpm_t[hj] = ekeep * hp;
  }
}

// ---------------------------------------------------------------- backward
// Workgroup = 16 hidden units x 32 rows; 16 waves, wave w owns n (gate
// columns of dG) in [4H/16 w, 4H/16 (w+1)).  dh_rec = dG_{t+1} W_h^T.
// dg_pk_in/out: dG in MFMA-operand order [row tile][wave][mt][s][lane];
// wt: W_h^T packed [H/16][wave][s][lane] (lane <-> unit l&15, n = 4s+(l>>4)).
template <int H, int RW = 32, int NW = 16>
__global__ __launch_bounds__(64 * NW) void lstm_bwd_step_kernel(
    const float* __restrict__ dh_out_t, const float* __restrict__ dg_pk_in,
    const uint8_t* __restrict__ done_next, const uint8_t* __restrict__ done_t,
    const float* __restrict__ wt, const float* __restrict__ acts_t,
    const float* __restrict__ c_t, const float* __restrict__ c_prev,
    const float* __restrict__ dcarry_in, float* __restrict__ dcarry_out,
    float* __restrict__ dg_t, float* __restrict__ dg_pk_out,
    __hip_bfloat16* __restrict__ dg16_t, int B, int xpack) {
  const float* dg_next = dg_pk_in;
  constexpr int NWID = 4 * H / NW;  // n per wave
  constexpr int NS = NWID / 4;
  __shared__ f4v red[NW][2][64];
  __shared__ float r_s[32][17];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  if (blockIdx.x % xpack) return;
  const int bx = blockIdx.x / xpack;
  const int u0 = bx * 16;
  static_assert(RW == 32 || RW == 16, "rows per workgroup");
  constexpr int NMT = RW / 16;
  const int r0 = blockIdx.y * RW;
  const int t32 = r0 >> 5, mt0 = (r0 >> 4) & 1;
  // epilogue operands: thread = (row er, unit eu) for tid < 16 RW
  const int er = tid >> 4, eu = tid & 15;
  const int egr = r0 + er;
  const int ej = u0 + eu;
  const bool eok = tid < 16 * RW && egr < B;
  // operands issued up front from clamped addresses, done bytes converted
  // only in the epilogue (see the forward kernel: one memory round trip)
  float dho = 0.f, ai = 0.f, ag = 0.f, af = 0.f, ao = 0.f, cc = 0.f, cpv = 0.f,
        dci = 0.f;
  uint32_t kdone = static_cast<uint32_t>(B), ndone = static_cast<uint32_t>(B);
  if (tid < 16 * RW) {
    const int egc = egr < B ? egr : B - 1;
    const int64_t hj = static_cast<int64_t>(egc) * H + ej;
    const int64_t g0 = static_cast<int64_t>(egc) * 4 * H + ej;
    dho = dh_out_t[hj];
    ai = acts_t[g0];
    ag = acts_t[g0 + H];
    af = acts_t[g0 + 2 * H];
    ao = acts_t[g0 + 3 * H];
    cc = c_t[hj];
    cpv = c_prev[hj];
    if (dcarry_in) dci = dcarry_in[hj];
    kdone = done_t[egc];
    ndone = done_next ? done_next[egc] : 0u;
  }
  if (dg_next != nullptr) {
    // B[k = n][col = unit]: W_h[u0 + (l&15)][n0 + 4s + (l>>4)] (packed)
    float wb[NS];
    const float* wsrc = wt + (static_cast<int64_t>(bx) * NW + wave) * NS * 64 + lane;
#pragma unroll
    for (int s = 0; s < NS; ++s) wb[s] = wsrc[s * 64];
    float da[NMT][NS];
    const float* pk = dg_pk_in + static_cast<int64_t>(t32) * 32 * 4 * H +
                      wave * 2 * NS * 64 + lane;
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
      for (int s = 0; s < NS; ++s) da[mt][s] = pk[((mt0 + mt) * NS + s) * 64];
    f4v acc[2] = {f4v{0.f, 0.f, 0.f, 0.f}, f4v{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt) acc[mt] = mfma_f32(da[mt][s], wb[s], acc[mt]);
    red[wave][0][lane] = acc[0];
    if (NMT == 2) red[wave][1][lane] = acc[1];
    __syncthreads();
    if (tid < 16 * RW) {
      const int m = tid >> 4, n = tid & 15;
      const int mt = m >> 4, mm = m & 15;
      const int src_lane = ((mm >> 2) << 4) | n;
      const int i = mm & 3;
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) sum += red[w][mt][src_lane][i];
      r_s[m][n] = sum;
    }
    __syncthreads();
  }
  if (eok) {
    const float kf = kdone ? 0.f : 1.f;
    const float knext = ndone ? 0.f : 1.f;
    const float rec = dg_next != nullptr ? r_s[er][eu] : 0.f;
    const int64_t hj = static_cast<int64_t>(egr) * H + ej;
    const int64_t g0 = static_cast<int64_t>(egr) * 4 * H + ej;
    const float dh = dho + knext * rec;
    const float tc = tanhf(cc);
    const float dc = dci + dh * ao * (1.f - tc * tc);
    const float dgv[4] = {dc * ag * ai * (1.f - ai), dc * ai * (1.f - ag * ag),
                          dc * kf * cpv * af * (1.f - af),
                          dh * tc * ao * (1.f - ao)};
    const int rr = egr - 32 * t32;
    float* pko = dg_pk_out + static_cast<int64_t>(t32) * 32 * 4 * H;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      dg_t[g0 + g * H] = dgv[g];
      if (dg16_t) dg16_t[g0 + g * H] = __float2bfloat16(dgv[g]);
      const int n = g * H + ej;
      const int w = n / NWID, s2 = (n % NWID) >> 2, q = n & 3;
      pko[((w * 2 + (rr >> 4)) * NS + s2) * 64 + (q << 4) + (rr & 15)] = dgv[g];
    }
    dcarry_out[hj] = dc * af * kf;
  }
}

// W_h [H,4H] -> w4 (fwd B operand, [H/4][H][4 units][4 gates]) and wt (bwd
// B operand, W_h^T [H/16][16 waves][4H/64][4][16]) in one pass.
template <int H>
__global__ __launch_bounds__(256) void lstm_pack_weights_kernel(
    const float* __restrict__ w, float* __restrict__ w4, float* __restrict__ wt) {
  constexpr int H4 = 4 * H;
  constexpr int NWID = H4 / 16;  // bwd n per wave
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= H * H4) return;
  const int k = idx / H4, n = idx - k * H4;
  const float v = w[idx];
  const int g = n / H, u = n - g * H;
  w4[((static_cast<int64_t>(u >> 2) * H + k) * 4 + (u & 3)) * 4 + g] = v;
  const int wv = n / NWID, r = n - wv * NWID, s2 = r >> 2, q = r & 3;
  wt[(((static_cast<int64_t>(k >> 4) * 16 + wv) * (NWID / 4) + s2) * 4 + q) * 16 + (k & 15)] = v;
}

}  // namespace

void lstm_pack_weights_launch(const float* w, float* w4, float* wt, int H,
                              hipStream_t stream) {
  const int n = H * 4 * H;
  if (H == 256)
    hipLaunchKernelGGL(lstm_pack_weights_kernel<256>, dim3((n + 255) / 256), dim3(256), 0,
                       stream, w, w4, wt);
  else if (H == 64)
    hipLaunchKernelGGL(lstm_pack_weights_kernel<64>, dim3((n + 255) / 256), dim3(256), 0,
                       stream, w, w4, wt);
}

// Default 2 (working blocks on 4 of the 8 XCDs).  Round 1 measured 4 best
// (469 -> 448 us fwd, 739 -> 724 us bwd per T=101 unroll vs 1; 8 = one XCD
// oversubscribes its 32 CUs); with every operand load issued up front
// (round 4) the full fp32 step is 9.650 / 9.654 ms at 2 vs 9.782 at 4, 9.664
// at 1 and 9.650-9.685 at 3 (SA_LSTM_XPACK sweep on one box).
static int g_xpack = [] {
  const int v = sa::measure_knob("SA_LSTM_XPACK", 2);
  return v >= 1 && v <= 8 ? v : 2;
}();
// 16 batch rows per step workgroup (twice the workgroups, each streaming
// half the packed h / dG): fp32 learner 13.01/13.05 -> 12.75/12.81 ms per
// step at B = 32 (A/B/A/B on one box); SA_LSTM_ROWS=32 restores 32 rows
static bool g_rows16 = sa::measure_knob("SA_LSTM_ROWS", 16) != 32;
// backward packing (SA_LSTM_XPACK_BWD; 0 = the forward's)
static int g_xpack_bwd = [] {
  const int v = sa::measure_knob("SA_LSTM_XPACK_BWD", 0);
  return v >= 1 && v <= 8 ? v : 0;
}();
int lstm_xpack(int v) {
  const int old = g_xpack;
  if (v >= 1 && v <= 8) g_xpack = v;
  return old;
}

void lstm_fwd_step_launch(const float* xw_t, const float* h_pk_in,
                          const float* h_prev, const float* c_prev,
                          const uint8_t* done_t, const float* w4, float* h_t,
                          float* h_pk_out, float* c_t, float* acts_t,
                          float* hpm_t, int B, int H, hipStream_t stream) {
  const int xp = g_xpack;
  // SA_LSTM_FWD_NW=4: four waves per workgroup (K split four ways)
  static const bool w4w = sa::measure_knob("SA_LSTM_FWD_NW", 8) == 4;
  if (H == 256 && g_rows16 && w4w) {
    dim3 grid16(H / 4 * xp, (B + 15) / 16);
    hipLaunchKernelGGL((lstm_fwd_step_kernel<256, 16, 4>), grid16, dim3(256), 0, stream,
                       xw_t, h_pk_in, h_prev, c_prev, done_t, w4, h_t, h_pk_out,
                       c_t, acts_t, hpm_t, B, xp);
    return;
  }
  if (H == 256 && g_rows16) {
    dim3 grid16(H / 4 * xp, (B + 15) / 16);
    hipLaunchKernelGGL((lstm_fwd_step_kernel<256, 16>), grid16, dim3(512), 0, stream,
                       xw_t, h_pk_in, h_prev, c_prev, done_t, w4, h_t, h_pk_out,
                       c_t, acts_t, hpm_t, B, xp);
    return;
  }
  dim3 grid(H / 4 * xp, (B + 31) / 32);
  if (H == 256) {
    hipLaunchKernelGGL(lstm_fwd_step_kernel<256>, grid, dim3(512), 0, stream,
                       xw_t, h_pk_in, h_prev, c_prev, done_t, w4, h_t, h_pk_out,
                       c_t, acts_t, hpm_t, B, xp);
  } else if (H == 64) {
    hipLaunchKernelGGL(lstm_fwd_step_kernel<64>, grid, dim3(512), 0, stream,
                       xw_t, h_pk_in, h_prev, c_prev, done_t, w4, h_t, h_pk_out,
                       c_t, acts_t, hpm_t, B, xp);
  }
}

void lstm_bwd_step_launch(const float* dh_out_t, const float* dg_pk_in,
                          const uint8_t* done_next, const uint8_t* done_t,
                          const float* wt, const float* acts_t,
                          const float* c_t, const float* c_prev,
                          const float* dcarry_in, float* dcarry_out,
                          float* dg_t, float* dg_pk_out, void* dg16_t, int B,
                          int H, hipStream_t stream) {
  const int xp = g_xpack_bwd ? g_xpack_bwd : g_xpack;
  dim3 grid(H / 16 * xp, (B + 31) / 32);
  __hip_bfloat16* d16 = static_cast<__hip_bfloat16*>(dg16_t);
  static const bool w8 = sa::measure_knob("SA_LSTM_BWD_W8", 0) == 1;
  if (H == 256 && g_rows16 && w8) {
    // 8 waves of 128 gate columns each (the packed W_h^T layout is the same:
    // each wave's slice is contiguous); the packed dG layout is private to
    // this kernel's own step-to-step hand-off
    dim3 grid16(H / 16 * xp, (B + 15) / 16);
    hipLaunchKernelGGL((lstm_bwd_step_kernel<256, 16, 8>), grid16, dim3(512), 0, stream,
                       dh_out_t, dg_pk_in, done_next, done_t, wt, acts_t, c_t,
                       c_prev, dcarry_in, dcarry_out, dg_t, dg_pk_out, d16, B, xp);
    return;
  }
  if (H == 256 && g_rows16) {
    dim3 grid16(H / 16 * xp, (B + 15) / 16);
    hipLaunchKernelGGL((lstm_bwd_step_kernel<256, 16>), grid16, dim3(1024), 0, stream,
                       dh_out_t, dg_pk_in, done_next, done_t, wt, acts_t, c_t,
                       c_prev, dcarry_in, dcarry_out, dg_t, dg_pk_out, d16, B, xp);
    return;
  }
  if (H == 256) {
    hipLaunchKernelGGL(lstm_bwd_step_kernel<256>, grid, dim3(1024), 0, stream,
                       dh_out_t, dg_pk_in, done_next, done_t, wt, acts_t, c_t,
                       c_prev, dcarry_in, dcarry_out, dg_t, dg_pk_out, d16, B, xp);
  } else if (H == 64) {
    hipLaunchKernelGGL(lstm_bwd_step_kernel<64>, grid, dim3(1024), 0, stream,
                       dh_out_t, dg_pk_in, done_next, done_t, wt, acts_t, c_t,
                       c_prev, dcarry_in, dcarry_out, dg_t, dg_pk_out, d16, B, xp);
  }
}

}  // namespace sa
