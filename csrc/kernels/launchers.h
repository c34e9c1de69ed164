// Host-side launcher declarations for the gfx950 kernels in csrc/kernels/.
// Kernels are plain HIP (no torch headers) so each .hip file compiles fast;
// csrc/bindings.cpp validates tensors and calls these with raw pointers and
// the current HIP stream (graph-capturable: no allocation, no sync).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sa {

// ---- rmsprop.hip -----------------------------------------------------------
// TF ApplyRMSProp over a flat fp32 buffer with lr = lr0*(1-min(f,F)/F) read
// from a device-side int64 frame counter.
void rmsprop_launch(float* w, const float* g, float* ms, float* mom,
                    const int64_t* frames, int64_t n, float lr0,
                    double total_frames, float decay, float momentum,
                    float eps, float gscale, int* guard, unsigned* lstm_err,
                    hipStream_t stream);

// NaN into *slot when err[0] | err[1] is set (the DP guard: one rank's
// fault makes every rank's finite check skip the same step).
void err_poison_launch(float* slot, unsigned* err, hipStream_t stream);

// ---- vtrace_loss.hip -------------------------------------------------------
// Fused V-trace (from logits) + IMPALA loss + analytic gradients.
// behaviour/target logits [T,B,A] f32, actions [T,B] i64, rewards/values
// [T,B] f32, done [T,B] u8, bootstrap [B] f32.
// Outputs: loss[4] = {total, pg, baseline, entropy} (sums), dlogits [T,B,A],
// dvalues [T,B]; optional vs/pg_adv [T,B] (may be null).
// work: scratch of 4*T*B floats.
void vtrace_loss_launch(const float* behaviour, const float* target,
                        const int64_t* actions, const float* rewards,
                        const uint8_t* done, const float* values,
                        const float* bootstrap, int T, int B, int A,
                        float discounting, int clip_mode, float clip_rho,
                        float clip_pg_rho, float baseline_cost,
                        float entropy_cost, float* loss, float* dlogits,
                        float* dvalues, float* vs_out, float* pg_adv_out,
                        float* work, hipStream_t stream);

// ---- lstm.hip --------------------------------------------------------------
// One LSTMBlockCell step over all B rows with done-reset (gate order i,c,f,o,
// forget bias +1).  xw_t [B,4H] = x_t W_x + b precomputed; w4 = W_h [H,4H]
// packed as [H/4 blocks][H k][4 units][4 gates]; h_pk = h_{t-1} in the fwd
// MFMA-operand order (see lstm.hip), written for the next step as h_pk_out;
// h_pk_in == nullptr reads h_prev [B,H] unpacked instead (first step).
// hpm_t (optional) = keep_t * h_prev for the dW_h GEMM.
void lstm_fwd_step_launch(const float* xw_t, const float* h_pk_in,
                          const float* h_prev, const float* c_prev,
                          const uint8_t* done_t, const float* w4, float* h_t,
                          float* h_pk_out, float* c_t, float* acts_t,
                          float* hpm_t, int B, int H, hipStream_t stream);
// Reverse step t: consumes dG_{t+1} (packed, null at t=T-1), writes dG_t
// (plain [B,4H] fp32, packed, and optionally bf16 for the bf16 dX GEMMs).
// wt = W_h^T packed [H/16][16][4H/64][64].
void lstm_bwd_step_launch(const float* dh_out_t, const float* dg_pk_in,
                          const uint8_t* done_next, const uint8_t* done_t,
                          const float* wt, const float* acts_t,
                          const float* c_t, const float* c_prev,
                          const float* dcarry_in, float* dcarry_out,
                          float* dg_t, float* dg_pk_out, void* dg16_t, int B,
                          int H, hipStream_t stream);
// Step-kernel placement knob: 1 = plain grid; 8 = launch 8x the blocks and let
// only every 8th work, i.e. all working blocks on one XCD (SA_LSTM_XPACK).
// v outside [1, 8] only queries.  Returns the previous value.
int lstm_xpack(int v);
// W_h [H,4H] -> fwd-packed w4 and bwd-packed wt (one launch per unroll).
// Instruction encoder (lang_lstm.hip): embedding + LSTM(64) over L words,
// output at the last valid word; fwd saves acts [L][N][256], cs [L][N][64],
// xh [L][N][84]; bwd -> dgates [L][N][256] and either dx [L][N][20] or,
// with egrad, dx added straight into the embedding rows of the valid words.
void lang_lstm_fwd_launch(const int64_t* ids, const int64_t* lengths, const float* embed,
                          const float* kernel, const float* bias, int N, int L, int V,
                          float* out, float* acts, float* cs, float* xh,
                          hipStream_t stream);
void lang_lstm_bwd_launch(const int64_t* lengths, const float* kernel, const float* dout,
                          const float* acts, const float* cs, int N, int L, float* dgates,
                          float* dx, const int64_t* ids, int V, float* egrad,
                          hipStream_t stream);

void lstm_pack_weights_launch(const float* w, float* w4, float* wt, int H,
                              hipStream_t stream);

// ---- lstm_persistent.hip -------------------------------------------------
// Whole-unroll LSTM-256 recurrence in one launch per direction (B <= 32).
// xbuf: lstm_persistent_xbuf_granules(bwd) zeroed 8-byte granules (zero it
// before EVERY launch); err: sticky timeout word (never reset by kernels).
// fwd: w4 packed as for lstm_fwd_step; outputs as lstm.hip (hs, cs, acts,
// hpm [T,B,...]).  bwd: wt packed W_h^T; dc_last may be null; dg16 / dc0
// may be null.
size_t lstm_persistent_xbuf_granules(bool bwd);
void lstm_fwd_persistent_launch(const float* xw, const float* h0, const float* c0,
                                const uint8_t* done, const float* w4, float* hs,
                                float* cs, float* acts, float* hpm, void* xbuf,
                                unsigned* err, int T, int B, hipStream_t stream);
void lstm_bwd_persistent_launch(const float* dh_out, const uint8_t* done,
                                const float* wt, const float* acts, const float* cs,
                                const float* c0, const float* dc_last, float* dg,
                                void* dg16, float* dc0, void* xbuf, unsigned* err,
                                int T, int B, hipStream_t stream);

// ---- lstm_gang.hip ---------------------------------------------------------
// Whole-unroll LSTM-256 recurrence on a gang of 8 workgroups with bf16 MFMA
// (B <= 32).  lstm_gang_pack_launch writes the bf16 fwd / bwd fragments (512
// KB each) of W_h [256,1024]; xbuf: lstm_gang_xbuf_granules(bwd) zeroed
// granules (zero before EVERY launch); err: the sticky timeout word.
size_t lstm_gang_xbuf_granules(bool bwd);
// 1 = wave-specialised kernels, 0 = uniform roles (default); other values
// only query.  Returns the previous value.
int lstm_gang_ws(int v);
// s_sleep(1) count between sweep passes (0..64; other values only query).
int lstm_gang_nap(int v);
// 1: every gang sweep reports a timeout (tests); v < 0 queries only.
int lstm_gang_fault(int v);
void lstm_gang_pack_launch(const float* w, void* wf, void* wbk, hipStream_t stream);
void lstm_fwd_gang_launch(const float* xw, const float* h0, const float* c0,
                          const uint8_t* done, const void* wf, float* hs, float* cs,
                          float* acts, float* hpm, void* xbuf, unsigned* err, int T,
                          int B, hipStream_t stream);
void lstm_bwd_gang_launch(const float* dh_out, const uint8_t* done, const void* wbk,
                          const float* acts, const float* cs, const float* c0,
                          const float* dc_last, float* dg, void* dg16, float* dc0,
                          void* xbuf, unsigned* err, int T, int B, hipStream_t stream);

// ---- learner_io.hip --------------------------------------------------------
// Fused heads + V-trace + loss (one workgroup per batch column; see the file
// header).  core [T+1,B,256]; behaviour/actions/rewards/done point at row 1
// of the [T+1,B,...] batch tensors; dlogits [T,B,A], dvalues [T,B];
// partial [B*3] scratch; ticket: zero-initialised persistent counter.
// Multi-task value heads (PopArt): task [B] int64 head index per batch
// column (null: one head), K heads (wb [256, K], bb [K]); mu / nu [K] the
// PopArt first / second moments (null: no normalisation); vs_out [T, B] the
// de-normalised V-trace targets (null: not written).
struct HeadTasks {
  const int64_t* task = nullptr;
  int K = 1;
  const float* mu = nullptr;
  const float* nu = nullptr;
  float* vs_out = nullptr;
};
size_t learner_head_fwd_smem(int T, int A);
void learner_head_fwd_launch(const float* core, const float* wp, const float* bp,
                             const float* wb, const float* bb,
                             const float* behaviour, const int64_t* actions,
                             const float* rewards, const uint8_t* done, int T,
                             int B, int A, float discounting, int clip_mode,
                             float clip_rho, float clip_pg_rho,
                             float baseline_cost, float entropy_cost,
                             float* dlogits, float* dvalues, float* partial,
                             unsigned* ticket, float* loss, const HeadTasks& tk,
                             hipStream_t stream);
// dcore [N1,256] = g (dlogits Wp^T + dv Wb[:, task]^T) (rows >= Ng zero;
// row r = t B + b reads head task[r % B], task null = head 0); heads'
// gradients accumulated into gwp [256,A], gbp [A], gwb [256,K], gbb [K]
// through per-row-chunk slots `part` (learner_head_bwd_part_floats) summed in
// a fixed order (bitwise reproducible).  A + K <= 64.
int64_t learner_head_bwd_part_floats(int N1, int A, int K);
void learner_head_bwd_launch(const float* gscale, const float* core,
                             const float* dlogits, const float* dvalues,
                             const float* wp, const float* wb, int N1, int Ng,
                             int A, int B, const int64_t* task, int K, float* dcore,
                             float* gwp, float* gbp, float* gwb, float* gbb,
                             float* part, hipStream_t stream);
// h_aug (bf16 [N, ld]) <- [h (bf16 [N, c0]), clip(r), one_hot(a), 0...]
void core_aug_fwd_launch(void* h_aug, const void* h, const float* rewards,
                         const int64_t* actions, int N, int ld, int c0,
                         int clip_mode, hipStream_t stream);
// out[c] += sum_r x[r,c], x fp32 [N,C]; per-row-chunk slots in `part`
// (colsum_f32_part_floats), added in a fixed order
int64_t colsum_f32_part_floats(int N, int C);
void colsum_f32_launch(const float* x, int N, int C, float* out, float* part,
                       hipStream_t stream);
// dy bf16 [N,C] *= (y > 0) (y bf16 with row stride ldy); out[c] += colsum
// (slots in `part`: relu_bwd_colsum_part_floats)
int64_t relu_bwd_colsum_part_floats(int N, int C);
void relu_bwd_colsum_launch(void* dy, const void* y, int N, int C, int ldy,
                            float* out, float* part, hipStream_t stream);
// dx bf16 *= (x > 0), n % 8 == 0
void relu_mask_bf16_launch(void* dx, const void* x, int64_t n,
                           hipStream_t stream);

// ---- actor_io.hip ----------------------------------------------------------
// Actor inference head: logits [B,A] = h Wp + bp, baseline [B] = h Wb + bb,
// action [B] ~ Categorical(softmax(logits)) by Gumbel-max over Philox4x32-10
// (key = seed, counter = (row, a, offset)).  h fp32 [B,256], A <= 32.
int actor_head_max_actions();
// inference-board epilogue (actor_io.hip): masked state update + slot-major
// output packing in one launch
int board_epilogue_max_fields();
void board_epilogue_launch(const void* const* src, const int* per_dw, const int* off_dw, int nf,
                           int R, int M, int slot_dw, int H, const float* mask, const float* c2,
                           const float* h2, float* c, float* h, void* out, int masked_only,
                           hipStream_t stream);
void actor_head_sample_launch(const float* h, const float* wp, const float* bp,
                              const float* wb, const float* bb, float* logits,
                              float* baseline, int64_t* action, int B, int A,
                              unsigned long long seed, unsigned long long offset,
                              unsigned long long* offset_ptr, int advance,
                              hipStream_t stream);

// ---- calibration ----------------------------------------------------------
void noop_launch(int blocks, int threads, int* p, hipStream_t s);

}  // namespace sa
