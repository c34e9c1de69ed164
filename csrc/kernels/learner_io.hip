// Learner glue kernels around the LSTM core: they replace ~40 small PyTorch
// launches per learner step (slices, concats, one-hots, bias adds, column
// sums, ReLU masks, the policy/baseline heads and their gradients) with a
// handful of fused launches.
//
//  * learner_head_fwd  policy + baseline heads (experiment.py:200-210) for all
//                      T+1 steps, then V-trace + IMPALA loss + their analytic
//                      gradients (vtrace.py:71-280, experiment.py:324-407):
//                      ONE workgroup per batch column b (the V-trace scan runs
//                      along time inside the workgroup), the four loss sums
//                      finished by the last workgroup to arrive (ticket) in a
//                      fixed order, so the loss is deterministic.
//                      Multi-task PopArt (Hessel et al. 2019; the learner's
//                      popart.py): K value heads, batch column b reads head
//                      task[b]; V-trace runs on the de-normalised values
//                      sigma n + mu, the baseline error is (vs - mu) / sigma - n
//                      and the policy-gradient advantage is divided by sigma;
//                      the targets vs go out for the statistics update.
//  * learner_head_bwd  dcore = g (dlogits W_p^T + dv W_b[:, task]^T) and the
//                      heads' weight/bias gradients (per-row-chunk slots
//                      summed in a fixed order), g = the incoming loss
//                      gradient.
//  * core_aug_fwd      [clip(r), one_hot(a), 0...] columns next to the torso
//                      output, so the core-input concat (experiment.py:185-198)
//                      and the x W_x projection are ONE GEMM.
//  * colsum_f32        column sums of an fp32 matrix accumulated into a vector
//                      (LSTM bias gradient).
//  * relu_bwd_colsum   dY *= (Y > 0) in place on bf16 + column sums (torso FC
//                      ReLU + bias gradient).
//  * relu_mask_bf16    dX *= (X > 0) in place (the torso's final ReLU).
#include "launchers.h"

#include <hip/hip_bf16.h>

namespace sa {
namespace {

typedef unsigned short bf16_t;  // raw bf16 bits
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(static_cast<unsigned>(v) << 16);
}
__device__ __forceinline__ bf16_t f2bf(float f) {  // round to nearest even
  unsigned u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<bf16_t>(u >> 16);
}

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

// Phase timestamps of block 0 for tools/micro/head_trace.hip (compiled out).
#ifdef SA_HEAD_TRACE
}  // namespace
__device__ unsigned long long sa_head_trace[16];
namespace {
#define HEAD_TRACE(i) \
  if (threadIdx.x == 0 && blockIdx.x == 0) sa_head_trace[i] = __builtin_amdgcn_s_memtime()
#else
#define HEAD_TRACE(i)
#endif

constexpr int kHeadThreads = 1024;
// PopArt sigma bounds (popart.py SIGMA_MIN / SIGMA_MAX)
constexpr float kPopArtSigmaMin = 1e-4f;
constexpr float kPopArtSigmaMax = 1e6f;
constexpr int kHeadWaves = kHeadThreads / 64;
constexpr int kMaxA = 31;      // A + 1 head outputs <= 32

// ------------------------------------------------------------ heads + V-trace
// core [T1,B,H] (H == 256), Wp [H,A], Wb [H] (one value head).  The V-trace
// inputs are the learner's time-shifted views (compute_loss): target logits
// / values = heads at t < T, bootstrap = value at T, behaviour logits,
// actions, rewards, done = rows 1..T of the batch (the caller passes
// pointers to row 1).  Every global operand of the column is fetched in the
// prologue with all loads in flight (one memory round trip), then the
// phases run out of LDS.  The heads are fp32 MFMA (16x16x4): wave w owns
// rows [16w, 16w+16) of the column, lane l sums k in [64(l>>4), +64), so its
// A operand is 64 contiguous floats of one core row.  LDS (dynamic, 4-byte
// words): W [H][MAXC] (zero-padded) | logits/values [T1][A+1] | behaviour
// [T][A] | a_t, delta_t, pgrho_t [T] | vs_t [T+1] | reward [T] | action [T]
// | done [T].
template <int MAXC>
__global__ __launch_bounds__(kHeadThreads) void learner_head_fwd_kernel(
    const float* __restrict__ core, const float* __restrict__ wp,
    const float* __restrict__ bp, const float* __restrict__ wb,
    const float* __restrict__ bb, const float* __restrict__ behaviour,
    const int64_t* __restrict__ actions, const float* __restrict__ rewards,
    const uint8_t* __restrict__ done, int T, int B, int A, float discounting,
    int clip_mode, float clip_rho, float clip_pg_rho, float baseline_cost,
    float entropy_cost, float* __restrict__ dlogits, float* __restrict__ dvalues,
    float* __restrict__ partial, unsigned* __restrict__ ticket,
    float* __restrict__ loss, HeadTasks tk) {
  constexpr int H = 256;
  extern __shared__ float smem[];
  const int A1 = A + 1;
  const int T1 = T + 1;
  float* w_s = smem;                 // [H][MAXC] + 4 x 16 pad
  float* lv_s = w_s + H * MAXC + 64; // [T1][A1]: logits then value
  float* beh_s = lv_s + T1 * A1;     // [T][A]
  float* a_s = beh_s + T * A;        // gamma_t c_t
  float* d_s = a_s + T;              // delta_t
  float* p_s = d_s + T;              // clipped pg rho
  float* vs_s = p_s + T;             // vs_t, vs_s[T] = bootstrap
  float* r_s = vs_s + T + 1;         // clipped reward
  int* act_s = reinterpret_cast<int*>(r_s + T);
  float* disc_s = reinterpret_cast<float*>(act_s + T);
  __shared__ float scan_a[kHeadThreads], scan_b[kHeadThreads];
  __shared__ float red[3][kHeadWaves];
  __shared__ bool last_s;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  // this column's value head and its PopArt statistics (identity without)
  // a task id outside [0, K) reads head 0 (no out-of-bounds access) with a
  // NaN sigma: the column's gradients turn NaN and the RMSProp step guard
  // drops the update (counted in skipped_updates) instead of training on it
  const int64_t kt_raw = tk.task != nullptr ? tk.task[b] : 0;
  const bool kt_bad = kt_raw < 0 || kt_raw >= tk.K;
  const int kt = kt_bad ? 0 : static_cast<int>(kt_raw);
  float sig = 1.f, mu = 0.f;
  if (tk.mu != nullptr) {
    mu = tk.mu[kt];
    const float var = fmaxf(tk.nu[kt] - mu * mu, kPopArtSigmaMin * kPopArtSigmaMin);
    sig = fminf(fmaxf(sqrtf(var), kPopArtSigmaMin), kPopArtSigmaMax);
  }
  if (kt_bad) sig = __builtin_nanf("");
  const float rsig = 1.f / sig;

  HEAD_TRACE(0);
  // ---- prologue: every load of the column issued before any is consumed
  constexpr int NCT = MAXC / 16;  // 16-wide output column tiles
  const int ntiles = (T1 + 15) / 16;
  const int arow = lane & 15, kq = lane >> 4;
  float4 xa[16];  // A operand: core[16 tile + arow][64 kq + 4j .. +3]
  auto load_a = [&](int tile) {
    const int t = 16 * tile + arow;
    const float4* src = reinterpret_cast<const float4*>(
        core + (static_cast<int64_t>(t < T1 ? t : 0) * B + b) * H + 64 * kq);
#pragma unroll
    for (int j = 0; j < 16; ++j) xa[j] = t < T1 ? src[j] : float4{0.f, 0.f, 0.f, 0.f};
  };
  if (wave < ntiles) load_a(wave);
  float bias[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    const int c = 16 * ct + arow;
    bias[ct] = c < A ? bp[c] : (c == A ? bb[kt] : 0.f);
  }
  // (register-staged: every load below is issued before the first LDS store)
  constexpr int WPT = H * MAXC / kHeadThreads;
  float wv[WPT];
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const int i = tid + j * kHeadThreads;
    const int k = i / MAXC, c = i - k * MAXC;
    wv[j] = c < A ? wp[k * A + c] : (c == A ? wb[k * tk.K + kt] : 0.f);
  }
  constexpr int BPT = 2;  // behaviour logits per thread staged in registers
  float bv[BPT];
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int i = tid + j * kHeadThreads;
    const int t = i / A, jj = i - t * A;
    bv[j] = i < T * A ? behaviour[(static_cast<int64_t>(t) * B + b) * A + jj] : 0.f;
  }
  float rv = 0.f, dn = 0.f;
  int av = 0;
  if (tid < T) {
    const int64_t idx = static_cast<int64_t>(tid) * B + b;  // row t+1 of batch
    rv = rewards[idx];
    av = static_cast<int>(actions[idx]);
    dn = done[idx] ? 0.f : discounting;
  }
  // W (k, c) at k MAXC + 16 (k / 64) + c: the 4 k-quarters of a wave's B
  // operand reads land 16 banks apart
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const int i = tid + j * kHeadThreads;
    w_s[i + 16 * ((i / MAXC) >> 6)] = wv[j];
  }
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int i = tid + j * kHeadThreads;
    if (i < T * A) beh_s[i] = bv[j];
  }
  for (int i = tid + BPT * kHeadThreads; i < T * A; i += kHeadThreads) {
    const int t = i / A, jj = i - t * A;  // long unrolls only
    beh_s[i] = behaviour[(static_cast<int64_t>(t) * B + b) * A + jj];
  }
  if (tid < T) {
    r_s[tid] = clip_reward(rv, clip_mode);
    act_s[tid] = av;
    disc_s[tid] = dn;
  }
  for (int t = tid + kHeadThreads; t < T; t += kHeadThreads) {
    const int64_t idx = static_cast<int64_t>(t) * B + b;
    r_s[t] = clip_reward(rewards[idx], clip_mode);
    act_s[t] = static_cast<int>(actions[idx]);
    disc_s[t] = done[idx] ? 0.f : discounting;
  }
  __syncthreads();
  HEAD_TRACE(1);

  // ---- heads: [16 rows x 256] x [256 x 16 cols] per wave on fp32 MFMA
  for (int tile = wave; tile < ntiles; tile += kHeadWaves) {
    if (tile != wave) load_a(tile);
    f4v acc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[ct] = f4v{0.f, 0.f, 0.f, 0.f};
    const float* wk = w_s + (64 * kq) * MAXC + 16 * kq + arow;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float av[4] = {xa[j].x, xa[j].y, xa[j].z, xa[j].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
          acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(
              av[q], wk[(4 * j + q) * MAXC + 16 * ct], acc[ct], 0, 0, 0);
      }
    }
    // D[row 4 kq + i][col arow]
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const int c = 16 * ct + arow;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = 16 * tile + 4 * kq + i;
        if (t < T1 && c < A1) lv_s[t * A1 + c] = acc[ct][i] + bias[ct];
      }
    }
  }
  __syncthreads();
  HEAD_TRACE(2);

  // ---- V-trace elementwise (vtrace.py:143-147, 235-262)
  for (int t = tid; t < T; t += kHeadThreads) {
    const float* zt = lv_s + t * A1;
    const float* zb = beh_s + t * A;
    const int a = act_s[t];
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
    const float disc = disc_s[t];
    const float v = sig * zt[A] + mu;  // de-normalised (PopArt) values
    const float v1 = sig * lv_s[(t + 1) * A1 + A] + mu;
    a_s[t] = disc * fminf(1.0f, rho);
    d_s[t] = fminf(clip_rho, rho) * (r_s[t] + disc * v1 - v);
    p_s[t] = fminf(clip_pg_rho, rho);
  }
  __syncthreads();
  HEAD_TRACE(3);

  // ---- reverse recursion acc_t = delta_t + a_t acc_{t+1}: each thread
  // composes a chunk of C steps, then a workgroup suffix scan of the maps
  const int C = (T + kHeadThreads - 1) / kHeadThreads;
  const int t0 = tid * C;
  const int t1 = min(t0 + C, T);
  float ca = 1.f, cb = 0.f;  // acc_{t0} = cb + ca * acc_{t1}
  for (int t = t1 - 1; t >= t0; --t) {
    cb = d_s[t] + a_s[t] * cb;
    ca = a_s[t] * ca;
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {  // wave-level inclusive suffix
    const float na = __shfl_down(ca, d, 64);
    const float nb = __shfl_down(cb, d, 64);
    if (lane + d < 64) {
      cb = cb + ca * nb;
      ca = ca * na;
    }
  }
  scan_a[tid] = ca;
  scan_b[tid] = cb;
  __syncthreads();
  HEAD_TRACE(4);
  // acc entering this thread's chunk from the right: the later waves'
  // totals, then the next lane's inclusive suffix in this wave
  float acc = 0.f;
  for (int w = kHeadWaves - 1; w > wave; --w) acc = scan_b[w * 64] + scan_a[w * 64] * acc;
  if (lane < 63) acc = scan_b[tid + 1] + scan_a[tid + 1] * acc;
  for (int t = t1 - 1; t >= t0; --t) {
    acc = d_s[t] + a_s[t] * acc;
    vs_s[t] = acc + (sig * lv_s[t * A1 + A] + mu);
  }
  if (tid == 0) vs_s[T] = sig * lv_s[T * A1 + A] + mu;  // bootstrap
  __syncthreads();
  HEAD_TRACE(5);

  // ---- advantages, loss terms and their gradients
  float l_pg = 0.f, l_bl = 0.f, l_ent = 0.f;
  for (int t = tid; t < T; t += kHeadThreads) {
    const int64_t idx = static_cast<int64_t>(t) * B + b;
    const float* zt = lv_s + t * A1;
    float* dz = dlogits + idx * A;
    const int a = act_s[t];
    const float n = zt[A];
    const float v = sig * n + mu;
    const float vs = vs_s[t];
    // PopArt: advantages in normalised units, baseline error against the
    // normalised target (sig = 1, mu = 0: the plain IMPALA loss, bitwise)
    const float pg_adv = p_s[t] * (r_s[t] + disc_s[t] * vs_s[t + 1] - v) * rsig;
    const float err = (vs - mu) * rsig - n;
    if (tk.vs_out != nullptr) tk.vs_out[idx] = vs;
    float m = -INFINITY;
    for (int j = 0; j < A; ++j) m = fmaxf(m, zt[j]);
    float s = 0.f;
    for (int j = 0; j < A; ++j) s += __expf(zt[j] - m);
    const float lse = m + __logf(s);
    float Hn = 0.f;
    for (int j = 0; j < A; ++j) {
      const float lp = zt[j] - lse;
      Hn -= __expf(lp) * lp;
    }
    for (int j = 0; j < A; ++j) {
      const float lp = zt[j] - lse;
      const float p = __expf(lp);
      dz[j] = (p - (j == a ? 1.f : 0.f)) * pg_adv + entropy_cost * p * (lp + Hn);
    }
    dvalues[idx] = -baseline_cost * err;
    l_pg += (lse - zt[a]) * pg_adv;
    l_bl += 0.5f * err * err;
    l_ent -= Hn;
  }
  l_pg = wave_sum(l_pg);
  l_bl = wave_sum(l_bl);
  l_ent = wave_sum(l_ent);
  if (lane == 0) {
    red[0][wave] = l_pg;
    red[1][wave] = l_bl;
    red[2][wave] = l_ent;
  }
  __syncthreads();
  HEAD_TRACE(6);
  if (tid == 0) {
    float pg = 0.f, bl = 0.f, en = 0.f;
    for (int w = 0; w < kHeadWaves; ++w) {
      pg += red[0][w];
      bl += red[1][w];
      en += red[2][w];
    }
    // publish the partials write-through (sc1), wait for them, then take a
    // ticket; the last block reads them with sc1 loads after its add
    // returned - no L2 write-back / invalidate fences (MI355X_MICROARCH.md,
    // inter-workgroup visibility, the one-lane sc1 hand-off)
    __hip_atomic_store(partial + b * 3 + 0, pg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(partial + b * 3 + 1, bl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(partial + b * 3 + 2, en, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    last_s = (prev == static_cast<unsigned>(gridDim.x) - 1);
  }
  __syncthreads();
  HEAD_TRACE(7);
  if (last_s && tid == 0) {
    float pg = 0.f, bl = 0.f, en = 0.f;
    for (int j = 0; j < B; ++j) {  // fixed order: deterministic
      pg += __hip_atomic_load(partial + j * 3 + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bl += __hip_atomic_load(partial + j * 3 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      en += __hip_atomic_load(partial + j * 3 + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    loss[1] = pg;
    loss[2] = bl;
    loss[3] = en;
    loss[0] = pg + baseline_cost * bl + entropy_cost * en;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
  }
  HEAD_TRACE(8);
}

// dcore [N1, H] = g (dlogits W_p^T + dv W_b[:, task]^T) (rows >= Ng get
// zero), and g core^T [dlogits | dv routed to the row's value head] and its
// column sums into per-row-chunk slots.  Columns: c < A policy, A + k value
// head k (K heads; row r = t B + b reads head task[b]).  Block = 16 hidden
// units x a chunk of ROWS rows (thread = (unit kk, row lane rl), ROWS / 16
// rows per thread, all core and dlogits loads of the chunk in flight at
// once); the 16 row lanes are reduced in registers/LDS, then one slot value
// per (unit, output) per block.
template <int MAXC>
constexpr int head_bwd_rows() { return MAXC <= 32 ? 256 : 128; }

template <int MAXC>
__global__ __launch_bounds__(256) void learner_head_bwd_kernel(
    const float* __restrict__ gscale, const float* __restrict__ core,
    const float* __restrict__ dlogits, const float* __restrict__ dvalues,
    const float* __restrict__ wp, const float* __restrict__ wb, int N1, int Ng,
    int A, int B, const int64_t* __restrict__ task, int K,
    float* __restrict__ dcore, float* __restrict__ part) {
  constexpr int H = 256;
  constexpr int ROWS = head_bwd_rows<MAXC>();
  constexpr int RPT = ROWS / 16;
  __shared__ float dl_s[ROWS][MAXC];
  __shared__ float red_s[4][16][MAXC];
  const int tid = threadIdx.x;
  const int kk = tid & 15, rl = tid >> 4;
  const int k = blockIdx.x * 16 + kk;
  const int r0 = blockIdx.y * ROWS;
  const int rows = min(ROWS, N1 - r0);
  const int A1 = A + K;
  // prologue: this thread's core values, the chunk's dlogits, the weights
  float x[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int rr = rl + 16 * i;
    x[i] = rr < rows ? core[static_cast<int64_t>(r0 + rr) * H + k] : 0.f;
  }
  const float g = gscale ? *gscale : 1.f;
  // dlogits / dv of the chunk: MAXC values per thread, all loads in flight;
  // a row's dv sits in its value head's column, the other heads get 0
  float dv_r[ROWS * MAXC / 256];
#pragma unroll
  for (int j = 0; j < ROWS * MAXC / 256; ++j) {
    const int i = tid + 256 * j;
    const int rr = i / MAXC, c = i - rr * MAXC;
    const int r = r0 + rr;
    float v = 0.f;
    if (rr < rows && r < Ng && c < A1) {
      if (c < A) {
        v = dlogits[static_cast<int64_t>(r) * A + c];
      } else {
        const int64_t kt = task != nullptr ? task[r % B] : 0;  // out of
        // range: no column matches (the forward made this row NaN already)
        v = (c - A == kt) ? dvalues[r] : 0.f;
      }
    }
    dv_r[j] = v;
  }
#pragma unroll
  for (int j = 0; j < ROWS * MAXC / 256; ++j) {
    const int i = tid + 256 * j;
    dl_s[i / MAXC][i % MAXC] = dv_r[j];
  }
  float w[MAXC], acc[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    w[c] = c < A ? wp[k * A + c] : (c < A1 ? wb[k * K + (c - A)] : 0.f);
    acc[c] = 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int rr = rl + 16 * i;
    if (rr < rows) {
      float d = 0.f;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        if (c < A1) {
          const float dc = dl_s[rr][c];
          d += dc * w[c];
          acc[c] += x[i] * dc;
        }
      }
      dcore[static_cast<int64_t>(r0 + rr) * H + k] = g * d;
    }
  }
  // reduce the 16 row lanes: lanes kk, kk+16, kk+32, kk+48 of a wave share
  // a unit; then the 4 waves through LDS
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    if (c < A1) {
      float v = acc[c];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) red_s[wave][lane][c] = v;
    }
  }
  __syncthreads();
  // this row chunk's totals go to its slot part[blockIdx.y][257 * A1]
  // ([unit k][A1] weight rows, then the A1 bias sums); head_grad_reduce
  // adds the slots in a fixed order (bitwise reproducible, no atomics)
  float* slot = part + static_cast<int64_t>(blockIdx.y) * 257 * A1;
  for (int i = tid; i < 16 * A1; i += 256) {
    const int u = i / A1, c = i - u * A1;
    const float v = g * (red_s[0][u][c] + red_s[1][u][c] + red_s[2][u][c] +
                         red_s[3][u][c]);
    slot[(blockIdx.x * 16 + u) * A1 + c] = v;
  }
  if (blockIdx.x == 0 && tid >= 256 - A1) {  // bias grads: column sums
    const int c = tid - (256 - A1);
    float s = 0.f;
    for (int rr = 0; rr < rows; ++rr) s += dl_s[rr][c];
    slot[256 * A1 + c] = g * s;
  }
}

// Fixed-order sum of the head-gradient slots into gwp [256, A], gwb [256, K],
// gbp [A], gbb [K].
__global__ __launch_bounds__(256) void head_grad_reduce_kernel(
    const float* __restrict__ part, int S, int A, int K, float* __restrict__ gwp,
    float* __restrict__ gbp, float* __restrict__ gwb, float* __restrict__ gbb) {
  const int A1 = A + K;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= 257 * A1) return;
  float v = 0.f;
  for (int s = 0; s < S; ++s) v += part[static_cast<int64_t>(s) * 257 * A1 + e];
  if (e < 256 * A1) {
    const int ku = e / A1, c = e - ku * A1;
    if (c < A) gwp[ku * A + c] += v;
    else gwb[ku * K + (c - A)] += v;
  } else {
    const int c = e - 256 * A1;
    if (c < A) gbp[c] += v;
    else gbb[c - A] += v;
  }
}

// out[c] += sum_s part[s][c] in slot order (the colsum kernels' partials).
__global__ __launch_bounds__(256) void rows_reduce_kernel(const float* __restrict__ part,
                                                          int S, int C,
                                                          float* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = 0;
  for (; s + 4 <= S; s += 4) {
    a0 += part[static_cast<int64_t>(s) * C + c];
    a1 += part[static_cast<int64_t>(s + 1) * C + c];
    a2 += part[static_cast<int64_t>(s + 2) * C + c];
    a3 += part[static_cast<int64_t>(s + 3) * C + c];
  }
  for (; s < S; ++s) a0 += part[static_cast<int64_t>(s) * C + c];
  out[c] += (a0 + a1) + (a2 + a3);
}

// -------------------------------------------------------------- core input
// h_aug [N, ld] bf16 <- [h (c0 columns), clip(r), one_hot(a), 0...]: the
// core input row without the (empty) instruction encoding.
__global__ __launch_bounds__(256) void core_aug_fwd_kernel(
    bf16_t* __restrict__ h_aug, const bf16_t* __restrict__ h,
    const float* __restrict__ rewards, const int64_t* __restrict__ actions,
    int N, int ld, int c0, int clip_mode) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= static_cast<int64_t>(N) * ld) return;
  const int n = static_cast<int>(i / ld);
  const int j = static_cast<int>(i - static_cast<int64_t>(n) * ld);
  bf16_t out;
  if (j < c0) {
    out = h[static_cast<int64_t>(n) * c0 + j];
  } else {
    float v = 0.f;
    if (j == c0) v = clip_reward(rewards[n], clip_mode);
    else if (j - c0 - 1 == static_cast<int>(actions[n])) v = 1.f;
    out = f2bf(v);
  }
  h_aug[i] = out;
}

// out[c] += sum_r x[r, c] over an fp32 [N, C] matrix.  Block: 256 columns x
// kColRows rows, loads batched 16 deep; one atomic per column per block.
constexpr int kColRows = 64;
constexpr int kColBatch = 16;

__global__ __launch_bounds__(256) void colsum_f32_kernel(
    const float* __restrict__ x, int N, int C, float* __restrict__ part) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int r0 = blockIdx.y * kColRows;
  const int r1 = min(r0 + kColRows, N);
  if (c >= C) return;
  float s = 0.f;
  for (int base = r0; base < r1; base += kColBatch) {
    float v[kColBatch];
#pragma unroll
    for (int j = 0; j < kColBatch; ++j)
      v[j] = base + j < r1 ? x[static_cast<int64_t>(base + j) * C + c] : 0.f;
#pragma unroll
    for (int j = 0; j < kColBatch; ++j) s += v[j];
  }
  part[static_cast<int64_t>(blockIdx.y) * C + c] = s;  // slot of this row chunk
}

// dy [N, C] bf16 *= (y > 0); out[c] += sum_r dy[r, c] (after masking).
// C even: thread = (column pair, row lane); a block covers C/2 pairs x
// kRbRows rows (256 / (C/2) row lanes), every load of the block issued up
// front; row lanes are reduced through LDS, then one atomic per column.
constexpr int kRbRows = 32;

__global__ __launch_bounds__(256) void relu_bwd_colsum_kernel(
    bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, int N, int C,
    int ldy, float* __restrict__ part) {
  __shared__ float red[256][2];
  const int pairs = C >> 1;
  const int lanes = 256 / pairs;  // row lanes (host: C/2 divides 256)
  const int cp = threadIdx.x % pairs, rl = threadIdx.x / pairs;
  const int r0 = blockIdx.x * kRbRows;
  constexpr int kMaxPer = kRbRows;  // lanes >= 1
  const int per = kRbRows / lanes;
  unsigned dv[kMaxPer], yv[kMaxPer];
#pragma unroll
  for (int i = 0; i < kMaxPer; ++i) {
    const int r = r0 + rl + lanes * i;
    const bool in = i < per && r < N;
    dv[i] = in ? *reinterpret_cast<const unsigned*>(dy + static_cast<int64_t>(r) * C + 2 * cp) : 0u;
    yv[i] = in ? *reinterpret_cast<const unsigned*>(y + static_cast<int64_t>(r) * ldy + 2 * cp) : 0u;
  }
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPer; ++i) {
    const int r = r0 + rl + lanes * i;
    if (i < per && r < N) {
      const bool on0 = bf2f(static_cast<bf16_t>(yv[i] & 0xffffu)) > 0.f;
      const bool on1 = bf2f(static_cast<bf16_t>(yv[i] >> 16)) > 0.f;
      const unsigned m = (on0 ? 0xffffu : 0u) | (on1 ? 0xffff0000u : 0u);
      const unsigned d = dv[i] & m;
      if (m != 0xffffffffu)
        *reinterpret_cast<unsigned*>(dy + static_cast<int64_t>(r) * C + 2 * cp) = d;
      s0 += bf2f(static_cast<bf16_t>(d & 0xffffu));
      s1 += bf2f(static_cast<bf16_t>(d >> 16));
    }
  }
  red[threadIdx.x][0] = s0;
  red[threadIdx.x][1] = s1;
  __syncthreads();
  if (part && threadIdx.x < pairs) {
    float t0 = 0.f, t1 = 0.f;
    for (int l = 0; l < lanes; ++l) {
      t0 += red[l * pairs + threadIdx.x][0];
      t1 += red[l * pairs + threadIdx.x][1];
    }
    float* slot = part + static_cast<int64_t>(blockIdx.x) * C;  // this block's slot
    slot[2 * threadIdx.x] = t0;
    slot[2 * threadIdx.x + 1] = t1;
  }
}

// dx *= (x > 0), 8 bf16 per thread
__global__ __launch_bounds__(256) void relu_mask_bf16_kernel(
    uint4* __restrict__ dx, const uint4* __restrict__ x, int64_t n8) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n8) return;
  uint4 d = dx[i];
  const uint4 v = x[i];
  unsigned* dp = reinterpret_cast<unsigned*>(&d);
  const unsigned* vp = reinterpret_cast<const unsigned*>(&v);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    // bf16 > 0  <=>  sign bit clear and not (+)0
    const unsigned lo = vp[j] & 0xffffu, hi = vp[j] >> 16;
    const unsigned mlo = (lo != 0u && !(lo & 0x8000u)) ? 0xffffu : 0u;
    const unsigned mhi = (hi != 0u && !(hi & 0x8000u)) ? 0xffff0000u : 0u;
    dp[j] &= (mlo | mhi);
  }
  dx[i] = d;
}

}  // namespace

size_t learner_head_fwd_smem(int T, int A) {
  const int maxc = (A + 1 <= 16) ? 16 : 32;
  return sizeof(float) * (256 * maxc + 64 + (T + 1) * (A + 1) + T * A + 4 * T +
                          1 + 3 * T);
}

void learner_head_fwd_launch(const float* core, const float* wp, const float* bp,
                             const float* wb, const float* bb,
                             const float* behaviour, const int64_t* actions,
                             const float* rewards, const uint8_t* done, int T,
                             int B, int A, float discounting, int clip_mode,
                             float clip_rho, float clip_pg_rho,
                             float baseline_cost, float entropy_cost,
                             float* dlogits, float* dvalues, float* partial,
                             unsigned* ticket, float* loss, const HeadTasks& tk,
                             hipStream_t stream) {
  const size_t smem = learner_head_fwd_smem(T, A);
  auto k16 = learner_head_fwd_kernel<16>;
  auto k32 = learner_head_fwd_kernel<kMaxA + 1>;
  auto kern = (A + 1 <= 16) ? k16 : k32;
  if (smem > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(smem));
  hipLaunchKernelGGL(kern, dim3(B), dim3(kHeadThreads), smem, stream, core, wp,
                     bp, wb, bb, behaviour, actions, rewards, done, T, B, A,
                     discounting, clip_mode, clip_rho, clip_pg_rho,
                     baseline_cost, entropy_cost, dlogits, dvalues, partial,
                     ticket, loss, tk);
}

int head_bwd_maxc(int A1) { return A1 <= 16 ? 16 : (A1 <= 32 ? 32 : 64); }
int head_bwd_rows_for(int A1) {
  return head_bwd_maxc(A1) <= 32 ? head_bwd_rows<32>() : head_bwd_rows<64>();
}

int64_t learner_head_bwd_part_floats(int N1, int A, int K) {
  const int rows = head_bwd_rows_for(A + K);
  return static_cast<int64_t>((N1 + rows - 1) / rows) * 257 * (A + K);
}

void learner_head_bwd_launch(const float* gscale, const float* core,
                             const float* dlogits, const float* dvalues,
                             const float* wp, const float* wb, int N1, int Ng,
                             int A, int B, const int64_t* task, int K, float* dcore,
                             float* gwp, float* gbp, float* gwb, float* gbb,
                             float* part, hipStream_t stream) {
  const int A1 = A + K, maxc = head_bwd_maxc(A1), rows = head_bwd_rows_for(A1);
  const dim3 grid(256 / 16, (N1 + rows - 1) / rows);
  if (maxc == 16)
    hipLaunchKernelGGL(learner_head_bwd_kernel<16>, grid, dim3(256), 0, stream,
                       gscale, core, dlogits, dvalues, wp, wb, N1, Ng, A, B, task, K,
                       dcore, part);
  else if (maxc == 32)
    hipLaunchKernelGGL(learner_head_bwd_kernel<32>, grid, dim3(256), 0, stream,
                       gscale, core, dlogits, dvalues, wp, wb, N1, Ng, A, B, task, K,
                       dcore, part);
  else
    hipLaunchKernelGGL(learner_head_bwd_kernel<64>, grid, dim3(256), 0, stream,
                       gscale, core, dlogits, dvalues, wp, wb, N1, Ng, A, B, task, K,
                       dcore, part);
  hipLaunchKernelGGL(head_grad_reduce_kernel, dim3((257 * A1 + 255) / 256),
                     dim3(256), 0, stream, part, static_cast<int>(grid.y), A, K, gwp,
                     gbp, gwb, gbb);
}

void core_aug_fwd_launch(void* h_aug, const void* h, const float* rewards,
                         const int64_t* actions, int N, int ld, int c0,
                         int clip_mode, hipStream_t stream) {
  const int64_t n = static_cast<int64_t>(N) * ld;
  hipLaunchKernelGGL(core_aug_fwd_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     stream, static_cast<bf16_t*>(h_aug),
                     static_cast<const bf16_t*>(h), rewards, actions, N, ld, c0,
                     clip_mode);
}

int64_t colsum_f32_part_floats(int N, int C) {
  return static_cast<int64_t>((N + kColRows - 1) / kColRows) * C;
}

void colsum_f32_launch(const float* x, int N, int C, float* out, float* part,
                       hipStream_t stream) {
  dim3 grid((C + 255) / 256, (N + kColRows - 1) / kColRows);
  hipLaunchKernelGGL(colsum_f32_kernel, grid, dim3(256), 0, stream, x, N, C, part);
  hipLaunchKernelGGL(rows_reduce_kernel, dim3((C + 255) / 256), dim3(256), 0, stream,
                     part, static_cast<int>(grid.y), C, out);
}

int64_t relu_bwd_colsum_part_floats(int N, int C) {
  return static_cast<int64_t>((N + kRbRows - 1) / kRbRows) * C;
}

void relu_bwd_colsum_launch(void* dy, const void* y, int N, int C, int ldy,
                            float* out, float* part, hipStream_t stream) {
  const int nb = (N + kRbRows - 1) / kRbRows;
  hipLaunchKernelGGL(relu_bwd_colsum_kernel, dim3(nb), dim3(256), 0, stream,
                     static_cast<bf16_t*>(dy), static_cast<const bf16_t*>(y), N, C,
                     ldy, out ? part : nullptr);
  if (out)
    hipLaunchKernelGGL(rows_reduce_kernel, dim3((C + 255) / 256), dim3(256), 0, stream,
                       part, nb, C, out);
}

void relu_mask_bf16_launch(void* dx, const void* x, int64_t n,
                           hipStream_t stream) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(relu_mask_bf16_kernel, dim3((n8 + 255) / 256), dim3(256), 0,
                     stream, static_cast<uint4*>(dx), static_cast<const uint4*>(x),
                     n8);
}

}  // namespace sa
