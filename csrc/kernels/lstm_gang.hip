// "Gang" LSTM-256 recurrence: one launch per direction for all T steps, run
// by a gang of EIGHT workgroups with the recurrent product on bf16 MFMA
// (v_mfma_f32_16x16x32_bf16, fp32 accumulate).  Same math and outputs as
// lstm.hip / lstm_persistent.hip (reference experiment.py:228-235).
//
// Why eight: lstm_persistent.hip (64 / 16 workgroups, exact fp32 MFMA) lost
// to the per-step kernels because every consumer workgroup swept the whole
// 64 KB (fwd) / 256 KB (bwd) exchange per step.  The exchange probe
// (tools/micro/xcd_sync_bench.hip, profiles/experiments.md) puts an 8-
// workgroup, 32 KB, all-loads-in-flight hand-off at ~1.9 us per step in any
// XCD placement, and with bf16 MFMA the whole 32x1024x256 step product is
// ~16 MFMAs per wave, so eight workgroups are enough and the exchange per
// consumer shrinks:
//   fwd: workgroup j owns units [32j, 32j+32) (128 gate columns); it
//        publishes its h_t as {tag, bf16 pair} granules and every workgroup
//        sweeps the whole h_t (4096 granules = 32 KB) into an LDS A image.
//   bwd: workgroup j owns units [32j, 32j+32); its dG_t slice stays in LDS
//        and its wave w computes the PARTIAL dG_t[:, own] W_h[32w.., own]^T
//        for destination workgroup w (a reduce-scatter): every workgroup
//        sweeps 8 sources x 32 x 32 partials as {tag, bf16 pair} granules
//        (32 KB) and sums them in fp32 in a fixed order (deterministic).
// Granule hand-off, tags, double-buffered slots, bounded spins and the
// sticky error word are those of lstm_persistent.hip (file header there).
// Numerics: the recurrent operand h_{t-1} / dG_{t+1} and W_h are rounded to
// bf16 for the product only (and the bwd partial sums for the exchange);
// the cell state, gates, carries and every output stay fp32.  Requires B <= 32 (rows >= B are computed as zeros and
// never stored).
#include "launchers.h"
#include "knobs.h"

#include <hip/hip_bf16.h>

#include <cstdlib>

namespace sa {
namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
typedef unsigned short bf16_t;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

constexpr unsigned kSpinLimit = 1u << 21;
constexpr int kH = 256;
constexpr int kGang = 8;              // workgroups
constexpr int kU = kH / kGang;        // 32 units per workgroup
constexpr int kThreads = 512;         // 8 waves
constexpr int kFSlot = 32 * kH / 2;   // fwd granules per slot: [row][unit pair]
constexpr int kBDest = 8 * 16 * kU;   // bwd granules per destination (4096)
constexpr int kBSlot = kGang * kBDest;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2v{lo, hi}, bf2v));
}
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, static_cast<__bf16>(f));
}
__device__ __forceinline__ f4v mfma(bf8v a, bf8v b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void publish(unsigned long long* g, unsigned tag,
                                        uint32_t bits) {
  __hip_atomic_store((gu64*)(g), (static_cast<unsigned long long>(tag) << 32) | bits,
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sweeps N contiguous granules until every tag == `tag` (all loads of a
// pass in flight together); v receives the low 32 bits.  false on timeout
// or when another workgroup already reported one (sticky error word).
// Granule k is read at g + (k / R) * S + k % R (R contiguous granules per
// run, runs S granules apart).
template <int N, int R = N, int S = 0>
__device__ __forceinline__ bool sweep(const unsigned long long* g, unsigned tag,
                                      uint32_t (&v)[N], unsigned* err, int nap = 1) {
  const gu64* p = (const gu64*)(g);
  if (nap < 0) {  // fault injection (lstm_gang_fault): behave as a timeout
    __hip_atomic_store((gu32*)(err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const unsigned long long x = __hip_atomic_load(
          p + (k / R) * S + k % R, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v[k] = static_cast<uint32_t>(x);
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
    for (int i = 0; i < nap; ++i) __builtin_amdgcn_s_sleep(1);
  }
}

// W_h [256, 1024] (k, n = g*256 + u) -> bf16 MFMA B fragments, 16 bytes per
// (workgroup j, wave w, step s, lane):
//   wf  (fwd): k = 32s + 8(l>>4) + e, column c = l&15 of wave w's n-tile:
//              unit 32j + 4w + (c>>2), gate c&3
//   wbk (bwd): row k = 32s + 8(l>>4) + e of the local dG image (gate s,
//              local unit 8(l>>4)+e of source j), column = unit
//              32w + 16a + (l&15) (a = n-tile), fragment index a*4 + s
__global__ __launch_bounds__(256) void lstm_gang_pack_kernel(
    const float* __restrict__ w, bf16_t* __restrict__ wf, bf16_t* __restrict__ wbk) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= kH * 4 * kH) return;
  const int k = idx >> 10, n = idx & 1023;
  const bf16_t v = f2bf(w[idx]);
  {
    const int g = n >> 8, u = n & 255;
    const int j = u >> 5, wv = (u & 31) >> 2, c = 4 * (u & 3) + g;
    const int s = k >> 5, lane = 16 * ((k & 31) >> 3) + c, e = k & 7;
    wf[((((j * 8 + wv) * 8 + s) * 64) + lane) * 8 + e] = v;
  }
  {
    const int g = n >> 8, rest = n & 255, j = rest >> 5, ul = rest & 31;
    const int wv = k >> 5, a = (k >> 4) & 1, lane = 16 * (ul >> 3) + (k & 15),
              e = ul & 7;
    wbk[((((j * 8 + wv) * 8 + a * 4 + g) * 64) + lane) * 8 + e] = v;
  }
}

// ---------------------------------------------------------------- forward
// Epilogue thread tid: row er = tid>>4, units 32j + 2q + {0,1} (q = tid&15);
// it publishes granule [er][16j + q] = {tag, bf16(h_u0), bf16(h_u1)}.  The
// sweep gives thread tid granules [8 tid, 8 tid + 8): row tid>>4, units
// 16(tid&15) .. +16, written keep-masked into the LDS A image.
__global__ __launch_bounds__(kThreads) void lstm_fwd_gang_kernel(
    const float* __restrict__ xw, const float* __restrict__ h0,
    const float* __restrict__ c0, const uint8_t* __restrict__ done,
    const bf16_t* __restrict__ wf, float* __restrict__ hs, float* __restrict__ cs,
    float* __restrict__ acts, float* __restrict__ hpm,
    unsigned long long* __restrict__ xbuf, unsigned* __restrict__ err, int T,
    int B, int nap) {
  constexpr int H = kH;
  __shared__ __attribute__((aligned(16))) bf16_t h_s[32][H + 8];
  __shared__ __attribute__((aligned(16))) float g_s[32][128 + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = blockIdx.x;
  bf8v wb[8];
  {
    const uint4* src = reinterpret_cast<const uint4*>(wf) + (j * 8 + wave) * 8 * 64 + lane;
#pragma unroll
    for (int s = 0; s < 8; ++s) wb[s] = __builtin_bit_cast(bf8v, src[s * 64]);
  }
  const int er = tid >> 4, q = tid & 15;
  const int ej = j * kU + 2 * q;  // first of the thread's two units
  const bool live = er < B;
  float c[2] = {0.f, 0.f}, h[2] = {0.f, 0.f};
  if (live) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      c[e] = c0[er * H + ej + e];
      h[e] = h0[er * H + ej + e];
    }
  }
  // The step's done byte is fetched raw with its xw operands one step ahead
  // and tested only where it is used: a test next to the load (or a fresh
  // done load per step) made the wave wait for the load - and, with one
  // vmcnt for loads and stores, for all of its step's output stores - before
  // its next sweep could start.  Nonzero default (B): rows >= B read as done.
  float xv[2][4] = {};
  uint32_t dnext = static_cast<uint32_t>(B);
  auto fetch = [&](int t) {
    if (live) {
      const int64_t g0 = (static_cast<int64_t>(t) * B + er) * 4 * H + ej;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float2 x2 = *reinterpret_cast<const float2*>(xw + g0 + g * H);
        xv[0][g] = x2.x;
        xv[1][g] = x2.y;
      }
      dnext = done[t * B + er];
    }
  };
  fetch(0);
  const int arow = lane & 15, ak = 8 * (lane >> 4);
  for (int t = 0; t < T; ++t) {
    // ---- LDS A image: keep_t * h_{t-1}, bf16 (the A-image row of this
    // thread is its epilogue row er: keep_t = live && !done[t][er])
    bool fail = false;
    const uint32_t dcur = dnext;
    {
      const int sr = tid >> 4, u0 = 16 * (tid & 15);
      uint32_t v[8];
      if (t == 0) {
        const bool keep = live && dcur == 0u;
        const float* hr = h0 + (sr < B ? sr : 0) * H + u0;
#pragma unroll
        for (int p = 0; p < 8; ++p)
          v[p] = keep ? pack2(hr[2 * p], hr[2 * p + 1]) : 0u;
      } else {
        fail = !sweep<8>(xbuf + ((t - 1) & 1) * kFSlot + 8 * tid,
                         static_cast<unsigned>(t), v, err, nap);
        if (!(live && dcur == 0u)) {
#pragma unroll
          for (int p = 0; p < 8; ++p) v[p] = 0u;
        }
      }
      uint4* dst = reinterpret_cast<uint4*>(&h_s[sr][u0]);
      dst[0] = uint4{v[0], v[1], v[2], v[3]};
      dst[1] = uint4{v[4], v[5], v[6], v[7]};
    }
    if (__syncthreads_or(fail)) break;  // a timed-out sweep anywhere: leave
    {
      f4v acc[2] = {f4v{0.f, 0.f, 0.f, 0.f}, f4v{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < 8; ++s) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const bf8v a = __builtin_bit_cast(
              bf8v, *reinterpret_cast<const uint4*>(&h_s[16 * mt + arow][32 * s + ak]));
          acc[mt] = mfma(a, wb[s], acc[mt]);
        }
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          g_s[16 * mt + 4 * (lane >> 4) + i][16 * wave + (lane & 15)] = acc[mt][i];
    }
    __syncthreads();
    {
      const float4 ga = *reinterpret_cast<const float4*>(&g_s[er][8 * q]);
      const float4 gb = *reinterpret_cast<const float4*>(&g_s[er][8 * q + 4]);
      const float gv[2][4] = {{ga.x, ga.y, ga.z, ga.w}, {gb.x, gb.y, gb.z, gb.w}};
      const float ekeep = dcur ? 0.f : 1.f;
      float hn[2], gi[2], gg[2], gf[2], go[2], hprev[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        gi[e] = sigm(gv[e][0] + xv[e][0]);
        gg[e] = tanhf(gv[e][1] + xv[e][1]);
        gf[e] = sigm(gv[e][2] + xv[e][2] + 1.0f);
        go[e] = sigm(gv[e][3] + xv[e][3]);
        hprev[e] = h[e];
        c[e] = gf[e] * ekeep * c[e] + gi[e] * gg[e];
        hn[e] = live ? go[e] * tanhf(c[e]) : 0.f;
        h[e] = hn[e];
      }
      publish(xbuf + (t & 1) * kFSlot + er * (H / 2) + j * (kU / 2) + q,
              static_cast<unsigned>(t + 1), pack2(hn[0], hn[1]));
      if (live) {
        const int64_t hj = (static_cast<int64_t>(t) * B + er) * H + ej;
        const int64_t g0 = (static_cast<int64_t>(t) * B + er) * 4 * H + ej;
        *reinterpret_cast<float2*>(hs + hj) = float2{hn[0], hn[1]};
        *reinterpret_cast<float2*>(cs + hj) = float2{c[0], c[1]};
        *reinterpret_cast<float2*>(hpm + hj) = float2{ekeep * hprev[0], ekeep * hprev[1]};
        *reinterpret_cast<float2*>(acts + g0) = float2{gi[0], gi[1]};
        *reinterpret_cast<float2*>(acts + g0 + H) = float2{gg[0], gg[1]};
        *reinterpret_cast<float2*>(acts + g0 + 2 * H) = float2{gf[0], gf[1]};
        *reinterpret_cast<float2*>(acts + g0 + 3 * H) = float2{go[0], go[1]};
      }
    }
    if (t + 1 < T) fetch(t + 1);
  }
}

// ---------------------------------------------------------------- backward
// Thread tid owns pairs idx = 2 tid + e (e = 0, 1) of the destination
// numbering idx = ((mt*2 + a)*64 + l)*4 + i4 (the MFMA D map of the
// producing wave): rows 16mt + 4(l>>4) + i4, local unit 16a + (l&15).  The
// producer of source j packs the partials of pairs 2 tid, 2 tid + 1 (rows
// i4 = 2(tid&1) + {0,1} of one D register quad) into granule j*512 + tid of
// the destination slot, so every 128-B line has ONE writer (a layout whose
// lines mixed 8 sources' granules timed out sporadically on MI355X), and
// consumer thread tid sweeps 8 granules, 512 apart.
__global__ __launch_bounds__(kThreads) void lstm_bwd_gang_kernel(
    const float* __restrict__ dh_out, const uint8_t* __restrict__ done,
    const bf16_t* __restrict__ wbk, const float* __restrict__ acts,
    const float* __restrict__ cs, const float* __restrict__ c0,
    const float* __restrict__ dc_last, float* __restrict__ dg,
    __hip_bfloat16* __restrict__ dg16, float* __restrict__ dc0,
    unsigned long long* __restrict__ xbuf, unsigned* __restrict__ err, int T,
    int B, int nap) {
  constexpr int H = kH;
  __shared__ __attribute__((aligned(16))) bf16_t d_s[2][32][4 * kU + 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = blockIdx.x;
  bf8v wb[8];  // [a*4 + s]
  {
    const uint4* src = reinterpret_cast<const uint4*>(wbk) + (j * 8 + wave) * 8 * 64 + lane;
#pragma unroll
    for (int f = 0; f < 8; ++f) wb[f] = __builtin_bit_cast(bf8v, src[f * 64]);
  }
  // this thread's two (row, unit) pairs
  const int pl = (tid >> 1) & 63, pa = (tid >> 7) & 1, pmt = tid >> 8;
  const int r0 = 16 * pmt + 4 * (pl >> 4) + 2 * (tid & 1);
  const int ul = 16 * pa + (pl & 15), ej = j * kU + ul;
  bool live[2];
  float carry[2] = {0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    live[e] = r0 + e < B;
    if (live[e] && dc_last) carry[e] = dc_last[(r0 + e) * H + ej];
  }
  // done bytes fetched raw and tested in the epilogue (see the forward)
  float dho[2] = {}, ai[2] = {}, ag[2] = {}, af[2] = {}, ao[2] = {}, cc[2] = {},
        cpv[2] = {};
  uint32_t kraw[2] = {0u, 0u}, nraw[2] = {0u, 0u};
  auto fetch = [&](int t) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      if (!live[e]) continue;
      const int r = r0 + e;
      const int64_t hj = (static_cast<int64_t>(t) * B + r) * H + ej;
      const int64_t g0 = (static_cast<int64_t>(t) * B + r) * 4 * H + ej;
      dho[e] = dh_out[hj];
      ai[e] = acts[g0];
      ag[e] = acts[g0 + H];
      af[e] = acts[g0 + 2 * H];
      ao[e] = acts[g0 + 3 * H];
      cc[e] = cs[hj];
      cpv[e] = t > 0 ? cs[hj - static_cast<int64_t>(B) * H] : c0[r * H + ej];
      kraw[e] = done[t * B + r];
      nraw[e] = t + 1 < T ? done[(t + 1) * B + r] : 0u;
    }
  };
  fetch(T - 1);
  const int arow = lane & 15, ak = 8 * (lane >> 4);
  for (int t = T - 1; t >= 0; --t) {
    const int p = T - 1 - t;  // processing step
    float rec[2] = {0.f, 0.f};
    bool fail = false;
    if (t < T - 1) {
      uint32_t v[8];
      fail = !sweep<8, 1, 16 * kU>(xbuf + ((t + 1) & 1) * kBSlot + j * kBDest + tid,
                                   static_cast<unsigned>(p), v, err, nap);
#pragma unroll
      for (int src = 0; src < kGang; ++src) {
        rec[0] += __uint_as_float(v[src] << 16);
        rec[1] += __uint_as_float(v[src] & 0xffff0000u);
      }
    }
    const int par = t & 1;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float dgv[4] = {0.f, 0.f, 0.f, 0.f};
      if (live[e]) {
        const float kf = kraw[e] ? 0.f : 1.f;
        const float knext = nraw[e] ? 0.f : 1.f;
        const float dh = dho[e] + knext * rec[e];
        const float tc = tanhf(cc[e]);
        const float dc = carry[e] + dh * ao[e] * (1.f - tc * tc);
        dgv[0] = dc * ag[e] * ai[e] * (1.f - ai[e]);
        dgv[1] = dc * ai[e] * (1.f - ag[e] * ag[e]);
        dgv[2] = dc * kf * cpv[e] * af[e] * (1.f - af[e]);
        dgv[3] = dh * tc * ao[e] * (1.f - ao[e]);
        const int64_t g0 = (static_cast<int64_t>(t) * B + r0 + e) * 4 * H + ej;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          dg[g0 + g * H] = dgv[g];
          if (dg16) dg16[g0 + g * H] = __float2bfloat16(dgv[g]);
        }
        carry[e] = dc * af[e] * kf;
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) d_s[par][r0 + e][g * kU + ul] = f2bf(dgv[g]);
    }
    if (__syncthreads_or(fail)) break;
    if (t > 0) {
      f4v acc[2][2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int a = 0; a < 2; ++a) acc[mt][a] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const bf8v av = __builtin_bit_cast(
              bf8v, *reinterpret_cast<const uint4*>(&d_s[par][16 * mt + arow][32 * s + ak]));
#pragma unroll
          for (int a = 0; a < 2; ++a) acc[mt][a] = mfma(av, wb[a * 4 + s], acc[mt][a]);
        }
      }
      // wave w's partial goes to destination workgroup w
      unsigned long long* dst = xbuf + par * kBSlot + wave * kBDest + j * 16 * kU;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int ip = 0; ip < 2; ++ip)
            publish(dst + ((mt * 2 + a) * 64 + lane) * 2 + ip, static_cast<unsigned>(p + 1),
                    pack2(acc[mt][a][2 * ip], acc[mt][a][2 * ip + 1]));
    }
    if (t > 0) fetch(t - 1);
  }
#pragma unroll
  for (int e = 0; e < 2; ++e)
    if (live[e] && dc0) dc0[(r0 + e) * H + ej] = carry[e];
}

// ------------------------------------------------- wave-specialised variants
// Same protocol, layouts and outputs as the kernels above, but the waves that
// POLL never have global stores in flight: on gfx950 one vmcnt counter covers
// loads and stores, so a sweep issued behind the epilogue's output stores and
// its own sc1 publish store could not retire a pass before those writes were
// acknowledged by memory.
//   fwd: waves 4-7 sweep h_{t-1} into the LDS A image; all 8 waves run the
//        MFMAs; waves 0-3 run the epilogue (thread: row tid>>3, units
//        32j + 4(tid&7) .. +4), publish and store the outputs.
//   bwd: waves 0-3 sweep the partials and run the epilogue (thread: unit
//        16a + (l&15), rows 16mt + 4(l>>4) + 0..3 for st = tid: l = st&63,
//        a = (st>>6)&1, mt = st>>7) and stage dG (bf16 A image + fp32 copy)
//        in LDS; waves 4-7 run the MFMAs for destinations 2w', 2w'+1,
//        publish, and store dg / dg16 from the fp32 LDS copy.
__global__ __launch_bounds__(kThreads) void lstm_fwd_gang_ws_kernel(
    const float* __restrict__ xw, const float* __restrict__ h0,
    const float* __restrict__ c0, const uint8_t* __restrict__ done,
    const bf16_t* __restrict__ wf, float* __restrict__ hs, float* __restrict__ cs,
    float* __restrict__ acts, float* __restrict__ hpm,
    unsigned long long* __restrict__ xbuf, unsigned* __restrict__ err, int T,
    int B, int nap) {
  constexpr int H = kH;
  __shared__ __attribute__((aligned(16))) bf16_t h_s[32][H + 8];
  __shared__ __attribute__((aligned(16))) float g_s[32][128 + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = blockIdx.x;
  const bool epi_wave = wave < 4;
  bf8v wb[8];
  {
    const uint4* src = reinterpret_cast<const uint4*>(wf) + (j * 8 + wave) * 8 * 64 + lane;
#pragma unroll
    for (int s = 0; s < 8; ++s) wb[s] = __builtin_bit_cast(bf8v, src[s * 64]);
  }
  // epilogue role
  const int er = (tid & 255) >> 3, uq = tid & 7;
  const int ej = j * kU + 4 * uq;
  const bool live = epi_wave && er < B;
  float c[4] = {0.f, 0.f, 0.f, 0.f}, h[4] = {0.f, 0.f, 0.f, 0.f};
  if (live) {
    const float4 c4 = *reinterpret_cast<const float4*>(c0 + er * H + ej);
    const float4 h4 = *reinterpret_cast<const float4*>(h0 + er * H + ej);
    c[0] = c4.x; c[1] = c4.y; c[2] = c4.z; c[3] = c4.w;
    h[0] = h4.x; h[1] = h4.y; h[2] = h4.z; h[3] = h4.w;
  }
  float4 xv[4] = {};
  float ekeep = 0.f;
  auto fetch = [&](int t) {
    if (live) {
      const int64_t g0 = (static_cast<int64_t>(t) * B + er) * 4 * H + ej;
#pragma unroll
      for (int g = 0; g < 4; ++g) xv[g] = *reinterpret_cast<const float4*>(xw + g0 + g * H);
      ekeep = done[t * B + er] ? 0.f : 1.f;
    }
  };
  fetch(0);
  // sweep role: granules [16 st, 16 st + 16) = row st>>3, units 32(st&7) .. +32
  const int st = tid & 255, sr = st >> 3, su0 = 32 * (st & 7);
  const int arow = lane & 15, ak = 8 * (lane >> 4);
  for (int t = 0; t < T; ++t) {
    bool fail = false;
    if (!epi_wave) {
      const bool keep = sr < B && !done[t * B + (sr < B ? sr : 0)];
      uint32_t v[16];
      if (t == 0) {
        const float* hr = h0 + (sr < B ? sr : 0) * H + su0;
#pragma unroll
        for (int p = 0; p < 16; ++p) v[p] = keep ? pack2(hr[2 * p], hr[2 * p + 1]) : 0u;
      } else {
        fail = !sweep<16>(xbuf + ((t - 1) & 1) * kFSlot + 16 * st,
                          static_cast<unsigned>(t), v, err, nap);
        if (!keep) {
#pragma unroll
          for (int p = 0; p < 16; ++p) v[p] = 0u;
        }
      }
      uint4* dst = reinterpret_cast<uint4*>(&h_s[sr][su0]);
#pragma unroll
      for (int q = 0; q < 4; ++q) dst[q] = uint4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
    }
    if (__syncthreads_or(fail)) break;
    {
      f4v acc[2] = {f4v{0.f, 0.f, 0.f, 0.f}, f4v{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < 8; ++s) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const bf8v a = __builtin_bit_cast(
              bf8v, *reinterpret_cast<const uint4*>(&h_s[16 * mt + arow][32 * s + ak]));
          acc[mt] = mfma(a, wb[s], acc[mt]);
        }
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          g_s[16 * mt + 4 * (lane >> 4) + i][16 * wave + (lane & 15)] = acc[mt][i];
    }
    __syncthreads();
    if (epi_wave) {
      float hn[4], gi[4], gg[4], gf[4], go[4], hp[4];
      const float* xg[4] = {&xv[0].x, &xv[1].x, &xv[2].x, &xv[3].x};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float4 gv = *reinterpret_cast<const float4*>(&g_s[er][16 * uq + 4 * e]);
        gi[e] = sigm(gv.x + xg[0][e]);
        gg[e] = tanhf(gv.y + xg[1][e]);
        gf[e] = sigm(gv.z + xg[2][e] + 1.0f);
        go[e] = sigm(gv.w + xg[3][e]);
        hp[e] = h[e];
        c[e] = gf[e] * ekeep * c[e] + gi[e] * gg[e];
        hn[e] = live ? go[e] * tanhf(c[e]) : 0.f;
        h[e] = hn[e];
      }
      unsigned long long* pub = xbuf + (t & 1) * kFSlot + er * (H / 2) + j * (kU / 2) + 2 * uq;
      publish(pub, static_cast<unsigned>(t + 1), pack2(hn[0], hn[1]));
      publish(pub + 1, static_cast<unsigned>(t + 1), pack2(hn[2], hn[3]));
      if (live) {
        const int64_t hj = (static_cast<int64_t>(t) * B + er) * H + ej;
        const int64_t g0 = (static_cast<int64_t>(t) * B + er) * 4 * H + ej;
        *reinterpret_cast<float4*>(hs + hj) = float4{hn[0], hn[1], hn[2], hn[3]};
        *reinterpret_cast<float4*>(cs + hj) = float4{c[0], c[1], c[2], c[3]};
        *reinterpret_cast<float4*>(hpm + hj) =
            float4{ekeep * hp[0], ekeep * hp[1], ekeep * hp[2], ekeep * hp[3]};
        *reinterpret_cast<float4*>(acts + g0) = float4{gi[0], gi[1], gi[2], gi[3]};
        *reinterpret_cast<float4*>(acts + g0 + H) = float4{gg[0], gg[1], gg[2], gg[3]};
        *reinterpret_cast<float4*>(acts + g0 + 2 * H) = float4{gf[0], gf[1], gf[2], gf[3]};
        *reinterpret_cast<float4*>(acts + g0 + 3 * H) = float4{go[0], go[1], go[2], go[3]};
      }
      if (t + 1 < T) fetch(t + 1);
    }
  }
}

__global__ __launch_bounds__(kThreads) void lstm_bwd_gang_ws_kernel(
    const float* __restrict__ dh_out, const uint8_t* __restrict__ done,
    const bf16_t* __restrict__ wbk, const float* __restrict__ acts,
    const float* __restrict__ cs, const float* __restrict__ c0,
    const float* __restrict__ dc_last, float* __restrict__ dg,
    __hip_bfloat16* __restrict__ dg16, float* __restrict__ dc0,
    unsigned long long* __restrict__ xbuf, unsigned* __restrict__ err, int T,
    int B, int nap) {
  constexpr int H = kH;
  __shared__ __attribute__((aligned(16))) bf16_t d_s[2][32][4 * kU + 8];
  __shared__ __attribute__((aligned(16))) float f_s[2][32][4 * kU + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = blockIdx.x;
  const bool epi_wave = wave < 4;
  const int mw = wave & 3;  // MFMA role: destinations 2mw, 2mw + 1
  bf8v wb[2][8];
  if (!epi_wave) {
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const uint4* src =
          reinterpret_cast<const uint4*>(wbk) + (j * 8 + 2 * mw + d) * 8 * 64 + lane;
#pragma unroll
      for (int f = 0; f < 8; ++f) wb[d][f] = __builtin_bit_cast(bf8v, src[f * 64]);
    }
  }
  // epilogue role: unit ul, rows r0 .. r0+3
  const int st = tid & 255, pl = st & 63, pa = (st >> 6) & 1, pmt = st >> 7;
  const int r0 = 16 * pmt + 4 * (pl >> 4);
  const int ul = 16 * pa + (pl & 15), ej = j * kU + ul;
  bool live[4];
  float carry[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    live[e] = epi_wave && r0 + e < B;
    if (live[e] && dc_last) carry[e] = dc_last[(r0 + e) * H + ej];
  }
  float dho[4] = {}, ai[4] = {}, ag[4] = {}, af[4] = {}, ao[4] = {}, cc[4] = {},
        cpv[4] = {}, kf[4] = {}, knext[4] = {1.f, 1.f, 1.f, 1.f};
  auto fetch = [&](int t) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (!live[e]) continue;
      const int r = r0 + e;
      const int64_t hj = (static_cast<int64_t>(t) * B + r) * H + ej;
      const int64_t g0 = (static_cast<int64_t>(t) * B + r) * 4 * H + ej;
      dho[e] = dh_out[hj];
      ai[e] = acts[g0];
      ag[e] = acts[g0 + H];
      af[e] = acts[g0 + 2 * H];
      ao[e] = acts[g0 + 3 * H];
      cc[e] = cs[hj];
      cpv[e] = t > 0 ? cs[hj - static_cast<int64_t>(B) * H] : c0[r * H + ej];
      kf[e] = done[t * B + r] ? 0.f : 1.f;
      knext[e] = t + 1 < T ? (done[(t + 1) * B + r] ? 0.f : 1.f) : 1.f;
    }
  };
  if (epi_wave) fetch(T - 1);
  const int arow = lane & 15, ak = 8 * (lane >> 4);
  for (int t = T - 1; t >= 0; --t) {
    const int p = T - 1 - t;
    const int par = t & 1;
    bool fail = false;
    if (epi_wave) {
      float rec[4] = {0.f, 0.f, 0.f, 0.f};
      if (t < T - 1) {
        uint32_t v[16];
        fail = !sweep<16, 2, 16 * kU>(xbuf + ((t + 1) & 1) * kBSlot + j * kBDest + 2 * st,
                                      static_cast<unsigned>(p), v, err, nap);
#pragma unroll
        for (int src = 0; src < kGang; ++src) {
          rec[0] += __uint_as_float(v[2 * src] << 16);
          rec[1] += __uint_as_float(v[2 * src] & 0xffff0000u);
          rec[2] += __uint_as_float(v[2 * src + 1] << 16);
          rec[3] += __uint_as_float(v[2 * src + 1] & 0xffff0000u);
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float dgv[4] = {0.f, 0.f, 0.f, 0.f};
        if (live[e]) {
          const float dh = dho[e] + knext[e] * rec[e];
          const float tc = tanhf(cc[e]);
          const float dc = carry[e] + dh * ao[e] * (1.f - tc * tc);
          dgv[0] = dc * ag[e] * ai[e] * (1.f - ai[e]);
          dgv[1] = dc * ai[e] * (1.f - ag[e] * ag[e]);
          dgv[2] = dc * kf[e] * cpv[e] * af[e] * (1.f - af[e]);
          dgv[3] = dh * tc * ao[e] * (1.f - ao[e]);
          carry[e] = dc * af[e] * kf[e];
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          d_s[par][r0 + e][g * kU + ul] = f2bf(dgv[g]);
          f_s[par][r0 + e][g * kU + ul] = dgv[g];
        }
      }
      if (t > 0) fetch(t - 1);
    }
    if (__syncthreads_or(fail)) break;
    if (!epi_wave) {
      if (t > 0) {
        f4v acc[2][2][2];
#pragma unroll
        for (int d = 0; d < 2; ++d)
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int a = 0; a < 2; ++a) acc[d][mt][a] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            const bf8v av = __builtin_bit_cast(
                bf8v, *reinterpret_cast<const uint4*>(&d_s[par][16 * mt + arow][32 * s + ak]));
#pragma unroll
            for (int d = 0; d < 2; ++d)
#pragma unroll
              for (int a = 0; a < 2; ++a)
                acc[d][mt][a] = mfma(av, wb[d][a * 4 + s], acc[d][mt][a]);
          }
        }
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          unsigned long long* dst =
              xbuf + par * kBSlot + (2 * mw + d) * kBDest + j * 16 * kU;
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
              for (int ip = 0; ip < 2; ++ip)
                publish(dst + ((mt * 2 + a) * 64 + lane) * 2 + ip,
                        static_cast<unsigned>(p + 1),
                        pack2(acc[d][mt][a][2 * ip], acc[d][mt][a][2 * ip + 1]));
        }
      }
      // outputs: 32 rows x 128 local columns, float4 per (row, gate, unit quad)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = st + 256 * k;  // 0..1023
        const int r = q >> 5, g = (q >> 3) & 3, u4 = (q & 7) * 4;
        if (r < B) {
          const float4 v = *reinterpret_cast<const float4*>(&f_s[par][r][g * kU + u4]);
          const int64_t g0 = (static_cast<int64_t>(t) * B + r) * 4 * H + g * H + j * kU + u4;
          *reinterpret_cast<float4*>(dg + g0) = v;
          if (dg16) {
            uint2 pk{pack2(v.x, v.y), pack2(v.z, v.w)};
            *reinterpret_cast<uint2*>(dg16 + g0) = pk;
          }
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (live[e] && dc0) dc0[(r0 + e) * H + ej] = carry[e];
}

}  // namespace

size_t lstm_gang_xbuf_granules(bool bwd) {
  return 2 * static_cast<size_t>(bwd ? kBSlot : kFSlot);
}

void lstm_gang_pack_launch(const float* w, void* wf, void* wbk, hipStream_t stream) {
  hipLaunchKernelGGL(lstm_gang_pack_kernel, dim3(kH * 4 * kH / 256), dim3(256), 0,
                     stream, w, static_cast<bf16_t*>(wf), static_cast<bf16_t*>(wbk));
}

// Uniform-role kernels by default; SA_LSTM_GANG_WS=1 selects the wave-
// specialised ones, measured slower (T=101, B=32: fwd 676-678 vs 446-448 us,
// bwd 823-839 vs 448-449 us; tools/micro/lstm_probe.py).
static int g_gang_ws = sa::measure_knob("SA_LSTM_GANG_WS", 0) == 1 ? 1 : 0;
// s_sleep(1) count between sweep passes (SA_LSTM_GANG_NAP, default 1).
static int g_gang_nap = [] {
  const int v = sa::measure_knob("SA_LSTM_GANG_NAP", 1);
  return v >= 0 && v <= 64 ? v : 1;
}();
int lstm_gang_nap(int v) {
  const int old = g_gang_nap;
  if (v >= 0 && v <= 64) g_gang_nap = v;
  return old;
}

// Fault injection for tests: every sweep reports a timeout (sticky error
// word set, unroll abandoned) so the learner-side guard can be exercised.
static int g_gang_fault = 0;
int lstm_gang_fault(int v) {
  const int old = g_gang_fault;
  if (v == 0 || v == 1) g_gang_fault = v;
  return old;
}

int lstm_gang_ws(int v) {
  const int old = g_gang_ws;
  if (v == 0 || v == 1) g_gang_ws = v;
  return old;
}

void lstm_fwd_gang_launch(const float* xw, const float* h0, const float* c0,
                          const uint8_t* done, const void* wf, float* hs, float* cs,
                          float* acts, float* hpm, void* xbuf, unsigned* err, int T,
                          int B, hipStream_t stream) {
  hipLaunchKernelGGL(g_gang_ws ? lstm_fwd_gang_ws_kernel : lstm_fwd_gang_kernel, dim3(kGang), dim3(kThreads), 0, stream, xw,
                     h0, c0, done, static_cast<const bf16_t*>(wf), hs, cs, acts, hpm,
                     static_cast<unsigned long long*>(xbuf), err, T, B,
                     g_gang_fault ? -1 : g_gang_nap);
}

void lstm_bwd_gang_launch(const float* dh_out, const uint8_t* done, const void* wbk,
                          const float* acts, const float* cs, const float* c0,
                          const float* dc_last, float* dg, void* dg16, float* dc0,
                          void* xbuf, unsigned* err, int T, int B, hipStream_t stream) {
  hipLaunchKernelGGL(g_gang_ws ? lstm_bwd_gang_ws_kernel : lstm_bwd_gang_kernel, dim3(kGang), dim3(kThreads), 0, stream,
                     dh_out, done, static_cast<const bf16_t*>(wbk), acts, cs, c0,
                     dc_last, dg, static_cast<__hip_bfloat16*>(dg16), dc0,
                     static_cast<unsigned long long*>(xbuf), err, T, B,
                     g_gang_fault ? -1 : g_gang_nap);
}

}  // namespace sa
