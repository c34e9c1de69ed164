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
                    float eps, int* guard, hipStream_t stream);

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
// MFMA-operand order (see lstm.hip), written for the next step as h_pk_out.
void lstm_fwd_step_launch(const float* xw_t, const float* h_pk_in,
                          const float* c_prev, const uint8_t* done_t,
                          const float* w4, float* h_t, float* h_pk_out,
                          float* c_t, float* acts_t, int B, int H,
                          hipStream_t stream);
// Reverse step t: consumes dG_{t+1} (packed, null at t=T-1), writes dG_t
// (plain [B,4H] and packed).  wt = W_h^T packed [H/16][16][4H/64][64].
void lstm_bwd_step_launch(const float* dh_out_t, const float* dg_pk_in,
                          const uint8_t* done_next, const uint8_t* done_t,
                          const float* wt, const float* acts_t,
                          const float* c_t, const float* c_prev,
                          const float* dcarry_in, float* dcarry_out,
                          float* dg_t, float* dg_pk_out, int B, int H,
                          hipStream_t stream);

// ---- calibration ----------------------------------------------------------
void noop_launch(int blocks, int threads, int* p, hipStream_t s);

}  // namespace sa
