// Instruction encoder: embedding gather + LSTM(64) over the
// words of every frame's instruction + the output at the last valid word,
// forward and backward each in ONE launch, exact fp32 (v_mfma_f32_16x16x4).
//
// Reference: experiment.py:123-146 - hashed words -> snt.Embed(1000, 20) ->
// dynamic_rnn(LSTMBlockCell(64)) with sequence_length -> last valid output
// (zeros for an empty instruction).  Gate order i, c~, f, o; forget bias +1.
//
// The learner runs it for all T*B = 3232 frames of a batch; the per-word
// loop of the generic path (one LSTM step kernel per word and direction)
// cost +5.4 ms per fp32 learner step.  Here one workgroup owns 16 frames for
// the whole word loop: wave w computes gate type w (columns 64w..64w+63 of
// the 256 gates) with its kernel columns resident in registers as MFMA A
// fragments; the 16 x 84 [x_t, h_{t-1}] operand comes from the embedding
// table (global, L2-resident) and an LDS copy of h; the cell update runs
// thread-per-(frame, unit) with c in registers.
//
//   fwd saves: acts [L][N][256] (i, c~, f, o after their nonlinearities),
//              cs [L][N][64], xh [L][N][84] = [x_t, h_{t-1}] (the A operand of
//              the kernel-gradient GEMM)
//   bwd:       dgates [L][N][256] (the caller turns them into
//              dK = xh^T dgates, db = 1^T dgates with gemm_f32) and the
//              embedding gradient: with egrad, each valid word's dx row is
//              atomically added to its embedding row here; else dx [L][N][20]
//              is written for a deterministic one-hot product by the caller.
//              A scatter-add of all L*N rows of dx (torch index_add_) cost
//              0.43 ms per learner step: every word past an instruction's
//              length has dx = 0 and id 0, so half the adds hit row 0.
#include "launchers.h"

namespace sa {
namespace {

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kE = 20, kH = 64, kG = 256, kXH = kE + kH;  // 84 = 21 k-steps
constexpr int kRows = 16;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ f4v mfma4(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__global__ __launch_bounds__(256) void lang_lstm_fwd_kernel(
    const int64_t* __restrict__ ids, const int64_t* __restrict__ lengths,
    const float* __restrict__ embed, const float* __restrict__ kernel,
    const float* __restrict__ bias, int N, int L, int V, float* __restrict__ out,
    float* __restrict__ acts, float* __restrict__ cs, float* __restrict__ xh) {
  __shared__ float h_s[kRows][kH + 4];
  __shared__ float g_s[4][kRows][kH + 4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int r0 = blockIdx.x * kRows;
  // A fragments: kernel[k = 4s + g][col = 64w + 16ct + c16]
  float ka[4][21];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int s = 0; s < 21; ++s)
      ka[ct][s] = kernel[(4 * s + g) * kG + 64 * w + 16 * ct + c16];
  float bcol[4][4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) bcol[ct][r] = bias[64 * w + 16 * ct + 4 * g + r];
  // cell-update threads: row er, units 4 eq .. 4 eq + 3
  const int er = tid >> 4, eq = tid & 15;
  const int erow = r0 + er;
  const bool eok = erow < N;
  // lengths past the word dimension are clamped (the output is the last
  // step's h, as in the forward and backward of the torch path)
  const int elen = eok ? static_cast<int>(min<int64_t>(max<int64_t>(lengths[erow], 0), L)) : 0;
  float c[4] = {0.f, 0.f, 0.f, 0.f};
  for (int e = tid; e < kRows * (kH + 4); e += 256) (&h_s[0][0])[e] = 0.f;
  // B-operand row of this lane
  const int brow = r0 + c16;
  const bool bok = brow < N;
  __syncthreads();
  for (int t = 0; t < L; ++t) {
    // x_t of the lane's row (k = 4s + g, s < 5), h_{t-1} from LDS
    const int64_t id = bok ? ids[static_cast<int64_t>(brow) * L + t] : 0;
    const int vid = (id >= 0 && id < V) ? static_cast<int>(id) : 0;
    float bx[21];
#pragma unroll
    for (int s = 0; s < 5; ++s) bx[s] = embed[vid * kE + 4 * s + g];
#pragma unroll
    for (int s = 5; s < 21; ++s) bx[s] = h_s[c16][4 * (s - 5) + g];
    if (w == 0 && bok) {
      // the [x_t, h_{t-1}] row for the kernel-gradient GEMM
      float* xr = xh + (static_cast<int64_t>(t) * N + brow) * kXH;
#pragma unroll
      for (int s = 0; s < 21; ++s) xr[4 * s + g] = bx[s];
    }
    f4v acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[ct] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 21; ++s)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) acc[ct] = mfma4(ka[ct][s], bx[s], acc[ct]);
    // D[i = col 4g + r][j = row c16]
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) g_s[w][c16][16 * ct + 4 * g + r] = acc[ct][r] + bcol[ct][r];
    __syncthreads();
    if (eok) {
      float hv[4];
      float* ap = acts + (static_cast<int64_t>(t) * N + erow) * kG;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int u = 4 * eq + q;
        const float i = sigm(g_s[0][er][u]);
        const float cc = tanhf(g_s[1][er][u]);
        const float f = sigm(g_s[2][er][u] + 1.f);  // forget_bias = 1
        const float o = sigm(g_s[3][er][u]);
        c[q] = f * c[q] + i * cc;
        hv[q] = o * tanhf(c[q]);
        ap[u] = i;
        ap[kH + u] = cc;
        ap[2 * kH + u] = f;
        ap[3 * kH + u] = o;
        cs[(static_cast<int64_t>(t) * N + erow) * kH + u] = c[q];
      }
      if (t == elen - 1)
        *reinterpret_cast<f4v*>(out + static_cast<int64_t>(erow) * kH + 4 * eq) =
            f4v{hv[0], hv[1], hv[2], hv[3]};
#pragma unroll
      for (int q = 0; q < 4; ++q) h_s[er][4 * eq + q] = hv[q];
    }
    __syncthreads();
  }
  if (eok && elen <= 0)
    *reinterpret_cast<f4v*>(out + static_cast<int64_t>(erow) * kH + 4 * eq) =
        f4v{0.f, 0.f, 0.f, 0.f};
}

// Reverse word loop.  Step t (t < len): dh = [t == len-1] dout + dh_rec,
// dc = dc_carry + dh o (1 - tanh^2 c_t), gate gradients, dc_carry = dc f;
// then [dx_t, dh_rec] = dgates K^T (84 x 256 product, MFMA, K rows as A
// fragments in registers).  Steps t >= len carry no gradient.
__global__ __launch_bounds__(256) void lang_lstm_bwd_kernel(
    const int64_t* __restrict__ lengths, const float* __restrict__ kernel,
    const float* __restrict__ dout, const float* __restrict__ acts,
    const float* __restrict__ cs, int N, int L, float* __restrict__ dgates,
    float* __restrict__ dx, const int64_t* __restrict__ ids, int V,
    float* __restrict__ egrad) {
  __shared__ float dg_s[kRows][kG + 4];
  __shared__ float dr_s[kRows][96 + 4];  // [row][k]: dx (k < 20) | dh_rec
  __shared__ int len_s[kRows];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int r0 = blockIdx.x * kRows;
  // k tiles of 16 (84 rows padded to 96): wave w owns tiles w and w + 4
  constexpr int NKT = 2;
  // A fragments: A[i = k (16 per tile)][kk = col 4s + g] = kernel[k][col]
  float ka[NKT][64];
#pragma unroll
  for (int j = 0; j < NKT; ++j) {
    const int kt = w + 4 * j;
    const int k = 16 * kt + c16;
#pragma unroll
    for (int s = 0; s < 64; ++s)
      ka[j][s] = (kt < 6 && k < kXH) ? kernel[k * kG + 4 * s + g] : 0.f;
  }
  const int er = tid >> 4, eq = tid & 15;
  const int erow = r0 + er;
  const bool eok = erow < N;
  // lengths past the word dimension are clamped (the output is the last
  // step's h, as in the forward and backward of the torch path)
  const int elen = eok ? static_cast<int>(min<int64_t>(max<int64_t>(lengths[erow], 0), L)) : 0;
  float dcar[4] = {0.f, 0.f, 0.f, 0.f};
  float dout_v[4] = {0.f, 0.f, 0.f, 0.f};
  if (eok)
#pragma unroll
    for (int q = 0; q < 4; ++q) dout_v[q] = dout[static_cast<int64_t>(erow) * kH + 4 * eq + q];
  for (int e = tid; e < kRows * 100; e += 256) (&dr_s[0][0])[e] = 0.f;
  if (eq == 0) len_s[er] = elen;
  __syncthreads();
  for (int t = L - 1; t >= 0; --t) {
    if (eok) {
      const int64_t base = static_cast<int64_t>(t) * N + erow;
      const float* ap = acts + base * kG;
      float* dgp = dgates + base * kG;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int u = 4 * eq + q;
        float di = 0.f, dcc = 0.f, df = 0.f, dov = 0.f;
        if (t < elen) {
          const float dh = (t == elen - 1 ? dout_v[q] : 0.f) + dr_s[er][kE + u];
          const float i = ap[u], cc = ap[kH + u], f = ap[2 * kH + u], o = ap[3 * kH + u];
          const float ct = cs[base * kH + u];
          const float cp = t > 0 ? cs[(base - N) * kH + u] : 0.f;
          const float tc = tanhf(ct);
          const float dc = dcar[q] + dh * o * (1.f - tc * tc);
          di = dc * cc * i * (1.f - i);
          dcc = dc * i * (1.f - cc * cc);
          df = dc * cp * f * (1.f - f);
          dov = dh * tc * o * (1.f - o);
          dcar[q] = dc * f;
        } else {
          dcar[q] = 0.f;
        }
        dg_s[er][u] = di;
        dg_s[er][kH + u] = dcc;
        dg_s[er][2 * kH + u] = df;
        dg_s[er][3 * kH + u] = dov;
        dgp[u] = di;
        dgp[kH + u] = dcc;
        dgp[2 * kH + u] = df;
        dgp[3 * kH + u] = dov;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int u = 4 * eq + q;
        dg_s[er][u] = dg_s[er][kH + u] = dg_s[er][2 * kH + u] = dg_s[er][3 * kH + u] = 0.f;
      }
    }
    __syncthreads();
    // D[i = k][j = row] = sum_col kernel[k][col] dgates[row][col]
#pragma unroll
    for (int j = 0; j < NKT; ++j) {
      const int kt = w + 4 * j;
      if (kt >= 6) continue;
      f4v acc = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 64; ++s) acc = mfma4(ka[j][s], dg_s[c16][4 * s + g], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) dr_s[c16][16 * kt + 4 * g + r] = acc[r];
    }
    __syncthreads();
    // dx_t: into the embedding row of the word (valid words only; an
    // out-of-range id read row 0 in the forward, so its gradient goes there)
    // or out for the caller
    for (int e = tid; e < kRows * kE; e += 256) {
      const int rr = e / kE, k = e - (e / kE) * kE;
      const int row = r0 + rr;
      if (row >= N) continue;
      if (egrad != nullptr) {
        if (t < len_s[rr]) {
          const int64_t id = ids[static_cast<int64_t>(row) * L + t];
          const int vid = (id >= 0 && id < V) ? static_cast<int>(id) : 0;
          atomicAdd(egrad + vid * kE + k, dr_s[rr][k]);
        }
      } else {
        dx[(static_cast<int64_t>(t) * N + row) * kE + k] = dr_s[rr][k];
      }
    }
  }
}

}  // namespace

void lang_lstm_fwd_launch(const int64_t* ids, const int64_t* lengths, const float* embed,
                          const float* kernel, const float* bias, int N, int L, int V,
                          float* out, float* acts, float* cs, float* xh,
                          hipStream_t stream) {
  hipLaunchKernelGGL(lang_lstm_fwd_kernel, dim3((N + kRows - 1) / kRows), dim3(256), 0,
                     stream, ids, lengths, embed, kernel, bias, N, L, V, out, acts, cs, xh);
}

void lang_lstm_bwd_launch(const int64_t* lengths, const float* kernel, const float* dout,
                          const float* acts, const float* cs, int N, int L, float* dgates,
                          float* dx, const int64_t* ids, int V, float* egrad,
                          hipStream_t stream) {
  hipLaunchKernelGGL(lang_lstm_bwd_kernel, dim3((N + kRows - 1) / kRows), dim3(256), 0,
                     stream, lengths, kernel, dout, acts, cs, N, L, dgates, dx, ids, V,
                     egrad);
}

}  // namespace sa
