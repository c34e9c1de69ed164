// Actor-inference head: policy logits + baseline + categorical sample in ONE
// launch (reference experiment.py:200-210: Linear(A) policy, Linear(1)
// baseline, tf.multinomial(logits, 1); SURVEY.md §2.3 K10 + K11).
//
// One 64-lane wavefront per batch row.  Lane l holds h[4l..4l+3] (one 16-byte
// load), forms its 4-term partial dot product for every output column and the
// row's A+1 sums are finished with a butterfly (every lane ends with every
// logit; no LDS, no barriers).  Lane a < A then draws u_a from Philox4x32-10
// (key = seed, counter = (row, a, offset)) and the action is the Gumbel-max
// argmax_a (logit_a - log(-log u_a)), reduced across the wave with the lower
// index winning ties - an exact sample from softmax(logits), reproducible for
// a given (seed, offset) whatever the batch composition of the other rows.
// With offset_ptr the offset is read from device memory, so a captured
// inference graph draws fresh samples on every replay (the graph bumps it).
#include "launchers.h"

namespace sa {
namespace {

constexpr int kMaxA = 32;

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const unsigned lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// heads + Gumbel-max sample of one row (one wave)
__device__ __forceinline__ void sample_row(
    const float* __restrict__ h, const float* __restrict__ wp,
    const float* __restrict__ bp, const float* __restrict__ wb,
    const float* __restrict__ bb, float* __restrict__ logits,
    float* __restrict__ baseline, int64_t* __restrict__ action, int A,
    unsigned long long seed, unsigned long long offset, int row, int lane) {
  const float4 x = reinterpret_cast<const float4*>(h + (int64_t)row * 256)[lane];
  const float* w0 = wp + (4 * lane) * A;
  float acc[kMaxA + 1];
#pragma unroll
  for (int a = 0; a < kMaxA; ++a)
    acc[a] = a < A ? x.x * w0[a] + x.y * w0[A + a] + x.z * w0[2 * A + a] +
                         x.w * w0[3 * A + a]
                   : 0.f;
  const float4 wv = reinterpret_cast<const float4*>(wb)[lane];
  acc[kMaxA] = x.x * wv.x + x.y * wv.y + x.z * wv.z + x.w * wv.w;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
#pragma unroll
    for (int a = 0; a <= kMaxA; ++a)
      if (a < A || a == kMaxA) acc[a] += __shfl_xor(acc[a], m, 64);
  }
  float mine = -INFINITY;
#pragma unroll
  for (int a = 0; a < kMaxA; ++a)
    if (a == lane) mine = acc[a];
  float key = -INFINITY;
  if (lane < A) {
    mine += bp[lane];
    logits[(int64_t)row * A + lane] = mine;
    const uint4 r = philox4x32_10(
        make_uint4((unsigned)row, (unsigned)lane, (unsigned)offset,
                   (unsigned)(offset >> 32)),
        make_uint2((unsigned)seed, (unsigned)(seed >> 32)));
    const float u = ((r.x >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0,1)
    key = mine - __logf(-__logf(u));
  }
  int idx = lane;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const float ok = __shfl_xor(key, m, 64);
    const int oi = __shfl_xor(idx, m, 64);
    if (ok > key || (ok == key && oi < idx)) {
      key = ok;
      idx = oi;
    }
  }
  if (lane == 0) {
    baseline[row] = acc[kMaxA] + bb[0];
    action[row] = idx;
  }
}

__global__ __launch_bounds__(256) void actor_head_sample_kernel(
    const float* __restrict__ h, const float* __restrict__ wp,
    const float* __restrict__ bp, const float* __restrict__ wb,
    const float* __restrict__ bb, float* __restrict__ logits,
    float* __restrict__ baseline, int64_t* __restrict__ action, int B, int A,
    unsigned long long seed, unsigned long long offset,
    unsigned long long* __restrict__ offset_ptr, int advance) {
  const int lane = threadIdx.x & 63;
  if (offset_ptr != nullptr) offset = *offset_ptr;  // graph-replayed stream
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row < B) sample_row(h, wp, bp, wb, bb, logits, baseline, action, A, seed, offset, row, lane);
  // advance: the stream's counter pair {offset, waves done} moves to the next
  // offset in this launch (no separate add kernel in the board's graph).
  // Every wave counts itself once after its sampling (which consumed the
  // offset it read); the last one stores offset + 1 and re-arms the count.
  // Lane 0 only: divergent, so vector-memory atomics and stores.
  if (advance && lane == 0) {
    const unsigned long long waves = static_cast<unsigned long long>(gridDim.x) * 4;
    const unsigned long long done = __hip_atomic_fetch_add(
        offset_ptr + 1, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (done == waves - 1) {
      __hip_atomic_store(offset_ptr, offset + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(offset_ptr + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
// Inference-board epilogue (runtime/inference_board.py BoardServer._body):
// the per-row masked LSTM state update and the packing of every output field
// into the board's slot-major output block, in ONE launch instead of two
// compare + select + copy chains and one copy per field (12 dependent
// launches, ~57 us of each board launch: tools/micro/board_trace.py).
//   c[r] = mask[r] > 0 ? c2[r] : c[r], h likewise (r < R, H columns);
//   out[(r / M) * slot_bytes + off[f] + (r % M) * per[f] + b] = src_f[r][b]
// for every field f < nf (per-row byte counts multiples of 4).
// masked_only: rows whose mask is 0 are not packed (`out` may then be the
// device view of the board's registered HOST output region: a slot that did
// not ask may be being read by its worker right now), and each packing
// thread ends with a system-scope fence so the host sees the rows once the
// launch's completion event fires.  This replaces one D2H copy per ready
// slot (each ~6 us, but 40-150 us apart on the queue: profiles/r6_e2e.md).
constexpr int kBoardFields = 6;
struct BoardEpi {
  const uint32_t* src[kBoardFields];
  int per_dw[kBoardFields];  // dwords per row
  int off_dw[kBoardFields];  // dword offset of the field in a slot block
  int nf, R, M, slot_dw, H;
  int masked_only;
  const float* mask;         // [R]
  const float* c2;
  const float* h2;
  float* c;
  float* h;
  uint32_t* out;
};

__global__ __launch_bounds__(256) void board_epilogue_kernel(BoardEpi a) {
  const int r = blockIdx.x;  // one workgroup per row
  if (r >= a.R) return;
  const bool keep = a.mask[r] > 0.f;
  for (int j = threadIdx.x; j < a.H; j += blockDim.x) {
    const int64_t o = static_cast<int64_t>(r) * a.H + j;
    if (keep) {
      a.c[o] = a.c2[o];
      a.h[o] = a.h2[o];
    }
  }
  if (a.masked_only && !keep) return;  // uniform per workgroup
  const int s = r / a.M, m = r - s * a.M;
  uint32_t* dst = a.out + static_cast<int64_t>(s) * a.slot_dw;
  for (int f = 0; f < a.nf; ++f) {
    const int per = a.per_dw[f];
    const uint32_t* src = a.src[f] + static_cast<int64_t>(r) * per;
    uint32_t* d = dst + a.off_dw[f] + m * per;
    for (int j = threadIdx.x; j < per; j += blockDim.x) d[j] = src[j];
  }
  if (a.masked_only) __threadfence_system();
}

}  // namespace

int board_epilogue_max_fields() { return kBoardFields; }

void board_epilogue_launch(const void* const* src, const int* per_dw, const int* off_dw, int nf,
                           int R, int M, int slot_dw, int H, const float* mask, const float* c2,
                           const float* h2, float* c, float* h, void* out, int masked_only,
                           hipStream_t stream) {
  if (R <= 0) return;
  BoardEpi a{};
  a.masked_only = masked_only;
  for (int f = 0; f < nf && f < kBoardFields; ++f) {
    a.src[f] = static_cast<const uint32_t*>(src[f]);
    a.per_dw[f] = per_dw[f];
    a.off_dw[f] = off_dw[f];
  }
  a.nf = nf < kBoardFields ? nf : kBoardFields;
  a.R = R;
  a.M = M;
  a.slot_dw = slot_dw;
  a.H = H;
  a.mask = mask;
  a.c2 = c2;
  a.h2 = h2;
  a.c = c;
  a.h = h;
  a.out = static_cast<uint32_t*>(out);
  hipLaunchKernelGGL(board_epilogue_kernel, dim3(R), dim3(256), 0, stream, a);
}

int actor_head_max_actions() { return kMaxA; }

void actor_head_sample_launch(const float* h, const float* wp, const float* bp,
                              const float* wb, const float* bb, float* logits,
                              float* baseline, int64_t* action, int B, int A,
                              unsigned long long seed, unsigned long long offset,
                              unsigned long long* offset_ptr, int advance,
                              hipStream_t stream) {
  if (B <= 0) return;
  hipLaunchKernelGGL(actor_head_sample_kernel, dim3((B + 3) / 4), dim3(256), 0,
                     stream, h, wp, bp, wb, bb, logits, baseline, action, B, A,
                     seed, offset, offset_ptr, advance);
}

}  // namespace sa
