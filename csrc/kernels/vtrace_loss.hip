// Fused V-trace + IMPALA loss + analytic gradients.
//
// Reference semantics: vtrace.py:71-280 (from_logits / from_importance_
// weights) and experiment.py:324-343, 377-407 (losses, reward clipping,
// discounts).  The reference runs V-trace on the CPU with a serial tf.scan;
// here the whole thing is ONE single-workgroup launch:
//
//   phase 1 (all T*B elements in parallel): log-softmax gathers of target and
//            behaviour logits, rho / clipped rho / c, clipped reward, discount,
//            delta_t = rho_bar_t (r_t + gamma_t V_{t+1} - V_t);
//   phase 2 (per batch column, one wave): the reverse recursion
//            acc_t = delta_t + gamma_t c_t acc_{t+1} as a wave-level parallel
//            affine scan ((a,b) o (a',b') = (a a', b + a b')) over 64 lanes;
//   phase 3 (parallel): pg advantages, the three loss sums and their
//            gradients:  dL/dz = (softmax - onehot) * pg_adv
//                              + entropy_cost * p (log p + H),
//                        dL/dV = -baseline_cost (vs - V).
// V-trace targets are stop-gradient, so the bootstrap value gets no gradient.
#include "launchers.h"

namespace sa {
namespace {

constexpr int kThreads = 1024;

__device__ __forceinline__ float clip_reward(float r, int mode) {
  if (mode == 0) return fminf(fmaxf(r, -1.f), 1.f);       // abs_one
  const float sq = tanhf(r / 5.0f);                         // soft_asymmetric
  return (r < 0.f ? 0.3f * sq : sq) * 5.0f;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__global__ __launch_bounds__(kThreads) void vtrace_loss_kernel(
    const float* __restrict__ behaviour, const float* __restrict__ target,
    const int64_t* __restrict__ actions, const float* __restrict__ rewards,
    const uint8_t* __restrict__ done, const float* __restrict__ values,
    const float* __restrict__ bootstrap, int T, int B, int A,
    float discounting, int clip_mode, float clip_rho, float clip_pg_rho,
    float baseline_cost, float entropy_cost, float* __restrict__ loss,
    float* __restrict__ dlogits, float* __restrict__ dvalues,
    float* __restrict__ vs_out, float* __restrict__ pg_adv_out,
    float* __restrict__ work) {
  const int N = T * B;
  float* w_a = work;            // gamma_t * c_t
  float* w_delta = work + N;    // delta_t
  float* w_pg = work + 2 * N;   // clipped pg rho
  float* w_vs = work + 3 * N;   // vs_t
  const int tid = threadIdx.x;

  // ---------------- phase 1
  for (int idx = tid; idx < N; idx += kThreads) {
    const int t = idx / B;
    const int b = idx - t * B;
    const float* zt = target + static_cast<int64_t>(idx) * A;
    const float* zb = behaviour + static_cast<int64_t>(idx) * A;
    const int a = static_cast<int>(actions[idx]);
    float mt = -INFINITY, mb = -INFINITY;
    for (int j = 0; j < A; ++j) {
      mt = fmaxf(mt, zt[j]);
      mb = fmaxf(mb, zb[j]);
    }
    float st = 0.f, sb = 0.f;
    for (int j = 0; j < A; ++j) {
      st += __expf(zt[j] - mt);
      sb += __expf(zb[j] - mb);
    }
    const float log_pi = zt[a] - mt - __logf(st);
    const float log_mu = zb[a] - mb - __logf(sb);
    const float rho = __expf(log_pi - log_mu);
    const float crho = fminf(clip_rho, rho);
    const float cs = fminf(1.0f, rho);
    const float r = clip_reward(rewards[idx], clip_mode);
    const float disc = done[idx] ? 0.f : discounting;
    const float v = values[idx];
    const float v1 = (t + 1 < T) ? values[idx + B] : bootstrap[b];
    w_a[idx] = disc * cs;
    w_delta[idx] = crho * (r + disc * v1 - v);
    w_pg[idx] = fminf(clip_pg_rho, rho);
  }
  __syncthreads();

  // ---------------- phase 2: per-column reverse affine scan, one wave each
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int nwaves = kThreads / 64;
  const int C = (T + 63) / 64;  // time steps per lane
  for (int b = wave; b < B; b += nwaves) {
    const int t0 = lane * C;
    const int t1 = min(t0 + C, T);
    float ca = 1.f, cb = 0.f;  // acc_{t0} = cb + ca * acc_{t1}
    for (int t = t1 - 1; t >= t0; --t) {
      const float at = w_a[t * B + b];
      cb = w_delta[t * B + b] + at * cb;
      ca = at * ca;
    }
    // inclusive suffix composition S_l = f_l o f_{l+1} o ... o f_63
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const float na = __shfl_down(ca, d, 64);
      const float nb = __shfl_down(cb, d, 64);
      if (lane + d < 64) {
        cb = cb + ca * nb;
        ca = ca * na;
      }
    }
    float acc = __shfl_down(cb, 1, 64);  // acc at this chunk's end
    if (lane == 63) acc = 0.f;
    for (int t = t1 - 1; t >= t0; --t) {
      acc = w_delta[t * B + b] + w_a[t * B + b] * acc;
      w_vs[t * B + b] = acc + values[t * B + b];
    }
  }
  __syncthreads();

  // ---------------- phase 3
  float l_pg = 0.f, l_bl = 0.f, l_ent = 0.f;
  for (int idx = tid; idx < N; idx += kThreads) {
    const int t = idx / B;
    const int b = idx - t * B;
    const float* zt = target + static_cast<int64_t>(idx) * A;
    float* dz = dlogits + static_cast<int64_t>(idx) * A;
    const int a = static_cast<int>(actions[idx]);
    const float r = clip_reward(rewards[idx], clip_mode);
    const float disc = done[idx] ? 0.f : discounting;
    const float v = values[idx];
    const float vs = w_vs[idx];
    const float vs1 = (t + 1 < T) ? w_vs[idx + B] : bootstrap[b];
    const float pg_adv = w_pg[idx] * (r + disc * vs1 - v);
    float m = -INFINITY;
    for (int j = 0; j < A; ++j) m = fmaxf(m, zt[j]);
    float s = 0.f;
    for (int j = 0; j < A; ++j) s += __expf(zt[j] - m);
    const float lse = m + __logf(s);
    float H = 0.f;
    for (int j = 0; j < A; ++j) {
      const float lp = zt[j] - lse;
      H -= __expf(lp) * lp;
    }
    for (int j = 0; j < A; ++j) {
      const float lp = zt[j] - lse;
      const float p = __expf(lp);
      dz[j] = (p - (j == a ? 1.f : 0.f)) * pg_adv +
              entropy_cost * p * (lp + H);
    }
    dvalues[idx] = -baseline_cost * (vs - v);
    if (vs_out) vs_out[idx] = vs;
    if (pg_adv_out) pg_adv_out[idx] = pg_adv;
    l_pg += (lse - zt[a]) * pg_adv;
    l_bl += 0.5f * (vs - v) * (vs - v);
    l_ent -= H;
  }
  __shared__ float red[3][kThreads / 64];
  l_pg = wave_sum(l_pg);
  l_bl = wave_sum(l_bl);
  l_ent = wave_sum(l_ent);
  if (lane == 0) {
    red[0][wave] = l_pg;
    red[1][wave] = l_bl;
    red[2][wave] = l_ent;
  }
  __syncthreads();
  if (tid == 0) {
    float pg = 0.f, bl = 0.f, en = 0.f;
    for (int w = 0; w < nwaves; ++w) {
      pg += red[0][w];
      bl += red[1][w];
      en += red[2][w];
    }
    loss[1] = pg;
    loss[2] = bl;
    loss[3] = en;
    loss[0] = pg + baseline_cost * bl + entropy_cost * en;
  }
}

}  // namespace

void vtrace_loss_launch(const float* behaviour, const float* target,
                        const int64_t* actions, const float* rewards,
                        const uint8_t* done, const float* values,
                        const float* bootstrap, int T, int B, int A,
                        float discounting, int clip_mode, float clip_rho,
                        float clip_pg_rho, float baseline_cost,
                        float entropy_cost, float* loss, float* dlogits,
                        float* dvalues, float* vs_out, float* pg_adv_out,
                        float* work, hipStream_t stream) {
  hipLaunchKernelGGL(vtrace_loss_kernel, dim3(1), dim3(kThreads), 0, stream,
                     behaviour, target, actions, rewards, done, values,
                     bootstrap, T, B, A, discounting, clip_mode, clip_rho,
                     clip_pg_rho, baseline_cost, entropy_cost, loss, dlogits,
                     dvalues, vs_out, pg_adv_out, work);
}

}  // namespace sa
