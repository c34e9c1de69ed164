// Persistent LSTM-256 recurrence: ONE launch per direction for all T steps
// (same math as lstm.hip, reference experiment.py:228-235).
//
// Why: the per-step kernels of lstm.hip pay a dependent-launch boundary
// (~1.5 us) plus a cold L2 round trip and an end-of-kernel drain every step,
// ~4.9 us fwd / ~7 us bwd per step.  Here each workgroup keeps its W_h slice
// in registers and its cell state / carry in registers for the whole unroll,
// and the per-step all-to-all of h_t (fwd) or dG_t (bwd) goes through
// data-tagged 8-byte granules {tag, fp32 value} written with one sc1 store
// each and swept with sc1 loads until every tag matches (MI355X_MICROARCH.md
// "Workgroup dispatch, XCD placement & inter-workgroup visibility", the R2
// granule hand-off: no fences, correct at any workgroup->XCD placement).
//
// Layout of a step's exchange slot: [wave w][lane l][mt][s] granules, i.e.
// exactly the MFMA A operand of consumer wave w, lane l (row 16 mt + (l&15),
// k/n = KW w + 4 s + (l>>4)): every consumer lane sweeps 16 (fwd) / 32 (bwd)
// contiguous granules.  Two slots alternate (step parity); tag = processing
// step + 1, never 0.  The host zeroes both slots before every launch (memset
// node under hipGraph replay), so stale tags from a previous call never
// match.  Double buffering is safe: a workgroup can only publish step s+2
// into the slot of step s after it has swept step s+1, which every workgroup
// publishes only after it finished sweeping step s.
//
// Every wait is bounded: a sweep that does not complete within kSpinLimit
// passes sets the sticky error word and the whole grid leaves (the timeout
// is voted through the step's first barrier), so the grid always drains.
// Requires B <= 32 (one row tile) and all workgroups co-resident (64 x 512
// fwd, 16 x 1024 bwd threads: a quarter / sixteenth of the CUs).
//
// Measured (MI355X, T=101, B=32, tools/micro/lstm_probe.py): 9.0 us per fwd
// step and 27.6 us per bwd step, against 4.4 / 6.9 us for the per-step
// kernels.  Every consumer workgroup must sweep the whole h_t (64 KB of
// granules) or dG_t (256 KB) each step, and sc1 sweeps of freshly published
// remote lines run at ~10 GB/s per CU - the all-gather, not the launch
// boundary, sets the step time.  The path is therefore opt-in
// (SA_LSTM_PERSISTENT=1) and kept as the measured alternative.
#include "launchers.h"

#include <hip/hip_bf16.h>

namespace sa {
namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

constexpr unsigned kSpinLimit = 1u << 21;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ f4v mfma_f32(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void store_granule(unsigned long long* g, unsigned tag,
                                              float v) {
  __hip_atomic_store((gu64*)(g),
                     (static_cast<unsigned long long>(tag) << 32) | __float_as_uint(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One wave sweeps its 2*NS granules (contiguous: NS for row tile 0, NS for
// row tile 1) until every tag == `tag`; a row tile whose row is not live
// (>= B, never published) is skipped.  Returns false on timeout or when
// another workgroup already reported one (sticky error word).
template <int NS>
__device__ __forceinline__ bool sweep(const unsigned long long* g, unsigned tag,
                                      bool live0, bool live1, float (&v)[2 * NS],
                                      unsigned* err) {
  const gu64* p = (const gu64*)(g);
  const unsigned long long dummy = static_cast<unsigned long long>(tag) << 32;
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 2 * NS; ++k) {
      const bool live = k < NS ? live0 : live1;
      const unsigned long long x =
          live ? __hip_atomic_load(p + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
               : dummy;
      v[k] = __uint_as_float(static_cast<unsigned>(x));
      ok &= static_cast<unsigned>(x >> 32) == tag;
    }
    if (__all(ok)) return true;
    if ((spins & 63) == 63 &&
        __hip_atomic_load((gu32*)(err), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT) != 0u)
      return false;
    if (spins >= kSpinLimit) {
      __hip_atomic_store((gu32*)(err), 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// ---------------------------------------------------------------- forward
// 64 workgroups x 512 threads: workgroup j owns units [4j, 4j+4) (16 gate
// columns, packed n = 4u + g, the w4 layout of lstm.hip); wave w owns
// k in [32w, 32w+32).  Epilogue threads tid < 128: (row tid>>2, unit tid&3).
constexpr int kH = 256;
constexpr int kFwdWaves = 8;
constexpr int kFwdKW = kH / kFwdWaves;   // 32
constexpr int kFwdNS = kFwdKW / 4;       // 8 MFMA k-steps per wave
constexpr int kFwdSlot = kFwdWaves * 64 * 2 * kFwdNS;  // granules per slot

__global__ __launch_bounds__(512) void lstm_fwd_persistent_kernel(
    const float* __restrict__ xw, const float* __restrict__ h0,
    const float* __restrict__ c0, const uint8_t* __restrict__ done,
    const float* __restrict__ w4, float* __restrict__ hs, float* __restrict__ cs,
    float* __restrict__ acts, float* __restrict__ hpm,
    unsigned long long* __restrict__ xbuf, unsigned* __restrict__ err, int T,
    int B) {
  constexpr int H = kH, NW = kFwdWaves, KW = kFwdKW, NS = kFwdNS;
  __shared__ f4v red[NW][2][64];
  __shared__ float g_s[32][17];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int blk = blockIdx.x;
  const int kw0 = wave * KW;
  // B operand, resident for the whole unroll: W[k = kw0 + 4s + (l>>4)][n = l&15]
  float wb[NS];
  {
    const float* wsrc = w4 + (static_cast<int64_t>(blk) * H + kw0 + (lane >> 4)) * 16 + (lane & 15);
#pragma unroll
    for (int s = 0; s < NS; ++s) wb[s] = wsrc[s * 4 * 16];
  }
  // epilogue state: (row er, unit ej); c and h stay in registers
  const int er = tid >> 2, ej = blk * 4 + (tid & 3);
  const bool epi = tid < 128 && er < B;
  float c = 0.f, h = 0.f;
  if (epi) {
    c = c0[er * H + ej];
    h = h0[er * H + ej];
  }
  // producer granule index of (er, ej) inside a slot
  const int pw = ej / KW, ps = (ej % KW) >> 2;
  const int pl = ((ej & 3) << 4) | (er & 15);
  const int pidx = ((pw * 64 + pl) * 2 + (er >> 4)) * NS + ps;
  // prefetched step operands
  float xi = 0.f, xc = 0.f, xf = 0.f, xo = 0.f, ekeep = 0.f;
  auto fetch_epi = [&](int t) {
    if (epi) {
      const int64_t g0 = (static_cast<int64_t>(t) * B + er) * 4 * H + ej;
      xi = xw[g0];
      xc = xw[g0 + H];
      xf = xw[g0 + 2 * H];
      xo = xw[g0 + 3 * H];
      ekeep = done[t * B + er] ? 0.f : 1.f;
    }
  };
  const int arow0 = lane & 15;
  bool keep_a[2];
  auto fetch_keep = [&](int t) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int row = 16 * mt + arow0;
      keep_a[mt] = row < B && !done[t * B + (row < B ? row : 0)];
    }
  };
  fetch_epi(0);
  fetch_keep(0);
  for (int t = 0; t < T; ++t) {
    // ---- A operand: keep_t * h_{t-1}[row][k]
    float ha[2][NS];
    bool fail = false;
    if (t == 0) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int row = 16 * mt + arow0;
        const float* hr = h0 + (row < B ? row : 0) * H + kw0 + (lane >> 4);
#pragma unroll
        for (int s = 0; s < NS; ++s) ha[mt][s] = keep_a[mt] ? hr[4 * s] : 0.f;
      }
    } else {
      float v[2 * NS];
      const unsigned long long* src =
          xbuf + ((t - 1) & 1) * kFwdSlot + (wave * 64 + lane) * 2 * NS;
      // rows >= B are never published; sweep only live rows
      fail = !sweep<NS>(src, static_cast<unsigned>(t), arow0 < B, 16 + arow0 < B, v, err);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        ha[0][s] = keep_a[0] ? v[s] : 0.f;
        ha[1][s] = keep_a[1] ? v[NS + s] : 0.f;
      }
    }
    f4v acc[2] = {f4v{0.f, 0.f, 0.f, 0.f}, f4v{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      acc[0] = mfma_f32(ha[0][s], wb[s], acc[0]);
      acc[1] = mfma_f32(ha[1][s], wb[s], acc[1]);
    }
    red[wave][0][lane] = acc[0];
    red[wave][1][lane] = acc[1];
    if (__syncthreads_or(fail)) break;  // a timed-out sweep anywhere: leave
    {
      const int m = tid >> 4, n = tid & 15;  // 512 threads == 32 x 16 outputs
      const int mt = m >> 4, mm = m & 15;
      const int src_lane = ((mm >> 2) << 4) | n;
      const int i = mm & 3;
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) sum += red[w][mt][src_lane][i];
      g_s[m][n] = sum;
    }
    __syncthreads();
    if (epi) {
      const int eu = tid & 3;
      const float gi = sigm(g_s[er][eu * 4 + 0] + xi);
      const float gg = tanhf(g_s[er][eu * 4 + 1] + xc);
      const float gf = sigm(g_s[er][eu * 4 + 2] + xf + 1.0f);
      const float go = sigm(g_s[er][eu * 4 + 3] + xo);
      const float hprev = h;
      c = gf * ekeep * c + gi * gg;
      h = go * tanhf(c);
      store_granule(xbuf + (t & 1) * kFwdSlot + pidx, static_cast<unsigned>(t + 1), h);
      const int64_t hj = (static_cast<int64_t>(t) * B + er) * H + ej;
      const int64_t g0 = (static_cast<int64_t>(t) * B + er) * 4 * H + ej;
      hs[hj] = h;
      cs[hj] = c;
      hpm[hj] = ekeep * hprev;
      acts[g0] = gi;
      acts[g0 + H] = gg;
      acts[g0 + 2 * H] = gf;
      acts[g0 + 3 * H] = go;
    }
    if (t + 1 < T) {
      fetch_epi(t + 1);
      fetch_keep(t + 1);
    }
  }
}

// ---------------------------------------------------------------- backward
// 16 workgroups x 1024 threads: workgroup j owns units [16j, 16j+16);
// wave w owns gate columns n in [64w, 64w+64) of dG_{t+1} W_h^T.  Epilogue
// threads tid < 512: (row tid>>4, unit tid&15).
constexpr int kBwdWaves = 16;
constexpr int kBwdNW = 4 * kH / kBwdWaves;  // 64 gate columns per wave
constexpr int kBwdNS = kBwdNW / 4;          // 16
constexpr int kBwdSlot = kBwdWaves * 64 * 2 * kBwdNS;

__global__ __launch_bounds__(1024) void lstm_bwd_persistent_kernel(
    const float* __restrict__ dh_out, const uint8_t* __restrict__ done,
    const float* __restrict__ wt, const float* __restrict__ acts,
    const float* __restrict__ cs, const float* __restrict__ c0,
    const float* __restrict__ dc_last, float* __restrict__ dg,
    __hip_bfloat16* __restrict__ dg16, float* __restrict__ dc0,
    unsigned long long* __restrict__ xbuf, unsigned* __restrict__ err, int T,
    int B) {
  constexpr int H = kH, NW = kBwdWaves, NWID = kBwdNW, NS = kBwdNS;
  __shared__ f4v red[NW][2][64];
  __shared__ float r_s[32][17];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int blk = blockIdx.x;
  float wb[NS];
  {
    const float* wsrc = wt + (static_cast<int64_t>(blk) * NW + wave) * NS * 64 + lane;
#pragma unroll
    for (int s = 0; s < NS; ++s) wb[s] = wsrc[s * 64];
  }
  const int er = tid >> 4, eu = tid & 15, ej = blk * 16 + eu;
  const bool epi = tid < 512 && er < B;
  float carry = 0.f;  // dc_{t+1} f_{t+1} keep_{t+1}
  if (epi && dc_last) carry = dc_last[er * H + ej];
  // producer granule indices of (er, ej) for the 4 gates
  int pidx[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int n = g * H + ej;
    const int w = n / NWID, rem = n % NWID;
    const int l = ((rem & 3) << 4) | (er & 15);
    pidx[g] = ((w * 64 + l) * 2 + (er >> 4)) * NS + (rem >> 2);
  }
  float dho = 0.f, ai = 0.f, ag = 0.f, af = 0.f, ao = 0.f, cc = 0.f, cpv = 0.f,
        kf = 0.f, knext = 1.f;
  auto fetch = [&](int t) {
    if (epi) {
      const int64_t hj = (static_cast<int64_t>(t) * B + er) * H + ej;
      const int64_t g0 = (static_cast<int64_t>(t) * B + er) * 4 * H + ej;
      dho = dh_out[hj];
      ai = acts[g0];
      ag = acts[g0 + H];
      af = acts[g0 + 2 * H];
      ao = acts[g0 + 3 * H];
      cc = cs[hj];
      cpv = t > 0 ? cs[hj - static_cast<int64_t>(B) * H] : c0[er * H + ej];
      kf = done[t * B + er] ? 0.f : 1.f;
      knext = t + 1 < T ? (done[(t + 1) * B + er] ? 0.f : 1.f) : 1.f;
    }
  };
  fetch(T - 1);
  const int arow0 = lane & 15;
  for (int t = T - 1; t >= 0; --t) {
    const int p = T - 1 - t;  // processing step
    bool fail = false;
    if (t < T - 1) {
      float v[2 * NS];
      const unsigned long long* src =
          xbuf + ((t + 1) & 1) * kBwdSlot + (wave * 64 + lane) * 2 * NS;
      const bool live0 = arow0 < B, live1 = 16 + arow0 < B;
      fail = !sweep<NS>(src, static_cast<unsigned>(p), live0, live1, v, err);
      f4v acc[2] = {f4v{0.f, 0.f, 0.f, 0.f}, f4v{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        acc[0] = mfma_f32(live0 ? v[s] : 0.f, wb[s], acc[0]);
        acc[1] = mfma_f32(live1 ? v[NS + s] : 0.f, wb[s], acc[1]);
      }
      red[wave][0][lane] = acc[0];
      red[wave][1][lane] = acc[1];
    }
    if (__syncthreads_or(fail)) break;
    if (t < T - 1 && tid < 512) {
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
    if (epi) {
      const float rec = t < T - 1 ? r_s[er][eu] : 0.f;
      const float dh = dho + knext * rec;
      const float tc = tanhf(cc);
      const float dc = carry + dh * ao * (1.f - tc * tc);
      const float dgv[4] = {dc * ag * ai * (1.f - ai), dc * ai * (1.f - ag * ag),
                            dc * kf * cpv * af * (1.f - af),
                            dh * tc * ao * (1.f - ao)};
      unsigned long long* dst = xbuf + (t & 1) * kBwdSlot;
      const int64_t g0 = (static_cast<int64_t>(t) * B + er) * 4 * H + ej;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        store_granule(dst + pidx[g], static_cast<unsigned>(p + 1), dgv[g]);
        dg[g0 + g * H] = dgv[g];
        if (dg16) dg16[g0 + g * H] = __float2bfloat16(dgv[g]);
      }
      carry = dc * af * kf;
    }
    if (t > 0) fetch(t - 1);
  }
  if (epi && dc0) dc0[er * H + ej] = carry;
}

}  // namespace

size_t lstm_persistent_xbuf_granules(bool bwd) {
  return 2 * static_cast<size_t>(bwd ? kBwdSlot : kFwdSlot);
}

void lstm_fwd_persistent_launch(const float* xw, const float* h0, const float* c0,
                                const uint8_t* done, const float* w4, float* hs,
                                float* cs, float* acts, float* hpm, void* xbuf,
                                unsigned* err, int T, int B, hipStream_t stream) {
  hipLaunchKernelGGL(lstm_fwd_persistent_kernel, dim3(kH / 4), dim3(512), 0, stream,
                     xw, h0, c0, done, w4, hs, cs, acts, hpm,
                     static_cast<unsigned long long*>(xbuf), err, T, B);
}

void lstm_bwd_persistent_launch(const float* dh_out, const uint8_t* done,
                                const float* wt, const float* acts, const float* cs,
                                const float* c0, const float* dc_last, float* dg,
                                void* dg16, float* dc0, void* xbuf, unsigned* err,
                                int T, int B, hipStream_t stream) {
  hipLaunchKernelGGL(lstm_bwd_persistent_kernel, dim3(kH / 16), dim3(1024), 0, stream,
                     dh_out, done, wt, acts, cs, c0, dc_last, dg,
                     static_cast<__hip_bfloat16*>(dg16), dc0,
                     static_cast<unsigned long long*>(xbuf), err, T, B);
}

}  // namespace sa
