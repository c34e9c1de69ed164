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
// Mapping (gfx950, wave64): a workgroup owns UB=4 hidden units (16 gate
// columns) for up to 32 batch rows; thread = (row, unit, k-split) with the
// 8-way k-split on the lowest lane bits so the partial dot products reduce
// with three __shfl_xor.  The W_h slice and the (masked) h_{t-1} tile are
// staged through LDS once per step and reused by all rows / all units.
#include "launchers.h"

namespace sa {
namespace {

constexpr int UB = 4;      // hidden units per workgroup
constexpr int KS = 8;      // k-split lanes
constexpr int RB = 32;     // batch rows per workgroup
constexpr int kThreads = RB * UB * KS;  // 1024

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

template <int H>
__global__ __launch_bounds__(kThreads) void lstm_fwd_step_kernel(
    const float* __restrict__ xw_t, const float* __restrict__ h_prev,
    const float* __restrict__ c_prev, const uint8_t* __restrict__ done_t,
    const float* __restrict__ w_h, float* __restrict__ h_t,
    float* __restrict__ c_t, float* __restrict__ acts_t, int B) {
  __shared__ float4 w_s[H * UB];     // [k][unit] -> (i, c, f, o)
  __shared__ float h_s[RB * H];      // [row][k], masked by keep
  const int tid = threadIdx.x;
  const int u0 = blockIdx.x * UB;
  const int r0 = blockIdx.y * RB;
  for (int e = tid; e < H * UB; e += kThreads) {
    const int k = e / UB, u = e - k * UB;
    const float* row = w_h + static_cast<int64_t>(k) * 4 * H + u0 + u;
    w_s[e] = make_float4(row[0], row[H], row[2 * H], row[3 * H]);
  }
  for (int e = tid; e < RB * H; e += kThreads) {
    const int r = e / H;
    const int gr = r0 + r;
    float v = 0.f;
    if (gr < B && !done_t[gr]) v = h_prev[static_cast<int64_t>(gr) * H + (e - r * H)];
    h_s[e] = v;
  }
  __syncthreads();
  const int ks = tid & (KS - 1);
  const int u = (tid / KS) & (UB - 1);
  const int r = tid / (KS * UB);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
  for (int kk = 0; kk < H / KS; ++kk) {
    const int k = kk * KS + ks;
    const float hv = h_s[r * H + k];
    const float4 w = w_s[k * UB + u];
    acc.x += hv * w.x;
    acc.y += hv * w.y;
    acc.z += hv * w.z;
    acc.w += hv * w.w;
  }
#pragma unroll
  for (int off = 1; off < KS; off <<= 1) {
    acc.x += __shfl_xor(acc.x, off, 64);
    acc.y += __shfl_xor(acc.y, off, 64);
    acc.z += __shfl_xor(acc.z, off, 64);
    acc.w += __shfl_xor(acc.w, off, 64);
  }
  const int gr = r0 + r;
  if (ks == 0 && gr < B) {
    const int j = u0 + u;
    const int64_t g0 = static_cast<int64_t>(gr) * 4 * H + j;
    const float ai = acc.x + xw_t[g0];
    const float ac = acc.y + xw_t[g0 + H];
    const float af = acc.z + xw_t[g0 + 2 * H];
    const float ao = acc.w + xw_t[g0 + 3 * H];
    const float i = sigm(ai), g = tanhf(ac), f = sigm(af + 1.0f), o = sigm(ao);
    const float keep = done_t[gr] ? 0.f : 1.f;
    const float c = f * keep * c_prev[static_cast<int64_t>(gr) * H + j] + i * g;
    const float h = o * tanhf(c);
    c_t[static_cast<int64_t>(gr) * H + j] = c;
    h_t[static_cast<int64_t>(gr) * H + j] = h;
    acts_t[g0] = i;
    acts_t[g0 + H] = g;
    acts_t[g0 + 2 * H] = f;
    acts_t[g0 + 3 * H] = o;
  }
}

template <int H>
__global__ __launch_bounds__(kThreads) void lstm_bwd_step_kernel(
    const float* __restrict__ dh_out_t, const float* __restrict__ dg_next,
    const uint8_t* __restrict__ done_next, const uint8_t* __restrict__ done_t,
    const float* __restrict__ w_h, const float* __restrict__ acts_t,
    const float* __restrict__ c_t, const float* __restrict__ c_prev,
    const float* __restrict__ dcarry_in, float* __restrict__ dcarry_out,
    float* __restrict__ dg_t, int B) {
  __shared__ float w_s[UB * 4 * H];  // W_h rows u0..u0+3, all 4H columns
  const int tid = threadIdx.x;
  const int u0 = blockIdx.x * UB;
  const int r0 = blockIdx.y * RB;
  const int ks = tid & (KS - 1);
  const int u = (tid / KS) & (UB - 1);
  const int r = tid / (KS * UB);
  const int gr = r0 + r;
  float acc = 0.f;
  if (dg_next != nullptr) {
    for (int e = tid; e < UB * 4 * H; e += kThreads) {
      const int uu = e / (4 * H);
      w_s[e] = w_h[static_cast<int64_t>(u0 + uu) * 4 * H + (e - uu * 4 * H)];
    }
    __syncthreads();
    if (gr < B) {
      const float* dg = dg_next + static_cast<int64_t>(gr) * 4 * H;
      const float* w = w_s + u * 4 * H;
#pragma unroll 8
      for (int kk = 0; kk < 4 * H / KS; ++kk) {
        const int n = kk * KS + ks;
        acc += dg[n] * w[n];
      }
    }
  }
#pragma unroll
  for (int off = 1; off < KS; off <<= 1) acc += __shfl_xor(acc, off, 64);
  if (ks == 0 && gr < B) {
    const int j = u0 + u;
    const int64_t hj = static_cast<int64_t>(gr) * H + j;
    const int64_t g0 = static_cast<int64_t>(gr) * 4 * H + j;
    const float keep_next = (done_next != nullptr && done_next[gr]) ? 0.f : 1.f;
    const float keep = done_t[gr] ? 0.f : 1.f;
    const float dh = dh_out_t[hj] + keep_next * acc;
    const float i = acts_t[g0], g = acts_t[g0 + H], f = acts_t[g0 + 2 * H],
                o = acts_t[g0 + 3 * H];
    const float c = c_t[hj];
    const float tc = tanhf(c);
    const float dc = (dcarry_in ? dcarry_in[hj] : 0.f) + dh * o * (1.f - tc * tc);
    const float cp = keep * c_prev[hj];
    dg_t[g0] = dc * g * i * (1.f - i);
    dg_t[g0 + H] = dc * i * (1.f - g * g);
    dg_t[g0 + 2 * H] = dc * cp * f * (1.f - f);
    dg_t[g0 + 3 * H] = dh * tc * o * (1.f - o);
    dcarry_out[hj] = dc * f * keep;
  }
}

}  // namespace

void lstm_fwd_step_launch(const float* xw_t, const float* h_prev,
                          const float* c_prev, const uint8_t* done_t,
                          const float* w_h, float* h_t, float* c_t,
                          float* acts_t, int B, int H, hipStream_t stream) {
  dim3 grid(H / UB, (B + RB - 1) / RB);
  if (H == 256) {
    hipLaunchKernelGGL(lstm_fwd_step_kernel<256>, grid, dim3(kThreads), 0,
                       stream, xw_t, h_prev, c_prev, done_t, w_h, h_t, c_t,
                       acts_t, B);
  } else if (H == 64) {
    hipLaunchKernelGGL(lstm_fwd_step_kernel<64>, grid, dim3(kThreads), 0,
                       stream, xw_t, h_prev, c_prev, done_t, w_h, h_t, c_t,
                       acts_t, B);
  }
}

void lstm_bwd_step_launch(const float* dh_out_t, const float* dg_next,
                          const uint8_t* done_next, const uint8_t* done_t,
                          const float* w_h, const float* acts_t,
                          const float* c_t, const float* c_prev,
                          const float* dcarry_in, float* dcarry_out,
                          float* dg_t, int B, int H, hipStream_t stream) {
  dim3 grid(H / UB, (B + RB - 1) / RB);
  if (H == 256) {
    hipLaunchKernelGGL(lstm_bwd_step_kernel<256>, grid, dim3(kThreads), 0,
                       stream, dh_out_t, dg_next, done_next, done_t, w_h,
                       acts_t, c_t, c_prev, dcarry_in, dcarry_out, dg_t, B);
  } else if (H == 64) {
    hipLaunchKernelGGL(lstm_bwd_step_kernel<64>, grid, dim3(kThreads), 0,
                       stream, dh_out_t, dg_next, done_next, done_t, w_h,
                       acts_t, c_t, c_prev, dcarry_in, dcarry_out, dg_t, B);
  }
}

}  // namespace sa
