// Launchers for the NHWC bf16 conv torso kernels (conv_torso.hip).
// Activations are NHWC bf16 (void* = raw bf16 bits), weights fp32 TF HWIO
// [3][3][CIN][COUT], weight/bias gradients fp32 and ACCUMULATED (zero first).
// pb_h/pb_w: TF-SAME pad_before of the 3x3/2 max-pool.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sa {
namespace conv {

int res_conv_rows(int H, int W);
// Sets a launch knob (value < 0: query only); returns the previous value or
// -1 for an unknown key.
int conv_tune_set(const char* key, int value);

// C = 3 (RGB) or 4 (stacked Atari frames) uint8 channels per pixel.
void conv1_pool_fwd_launch(const uint8_t* x, const float* w, const float* b,
                           void* pooled, uint8_t* argmax, int N, int H, int W,
                           int C, int pb_h, int pb_w, hipStream_t s);
void conv_pool_fwd_launch(const void* x, const float* w, const float* b,
                          void* pooled, uint8_t* argmax, int N, int H, int W,
                          int CIN, int COUT, int pb_h, int pb_w, hipStream_t s);
void res_conv_fwd_launch(const void* x, const float* w, const float* b,
                         const void* resid, void* y, int N, int H, int W,
                         int C, bool post_relu, bool relu_in, hipStream_t s);
// Whole residual block: t = relu(conv1(relu(x)) + b1) (written, for the
// backward), y = conv2(t) + b2 + x [then relu].
void res_block_fwd_launch(const void* x, const float* w1, const float* b1,
                          const float* w2, const float* b2, void* t, void* y,
                          int N, int H, int W, int C, bool post_relu,
                          hipStream_t s);
void res_conv_bwd_launch(const void* dy, const void* act, const void* skip,
                         const float* w, void* dx, float* dw, float* db, int N,
                         int H, int W, int C, bool relu_act, hipStream_t s,
                         float* part = nullptr);
void pool_conv_bwd_launch(const void* dP, const uint8_t* argmax, const void* x,
                          const float* w, void* dx, float* dw, float* db, int N,
                          int H, int W, int CIN, int COUT, int pb_h, int pb_w,
                          hipStream_t s, float* part = nullptr);
void conv1_pool_bwd_launch(const void* dP, const uint8_t* argmax,
                           const uint8_t* x, float* dw, float* db, int N,
                           int H, int W, int C, int pb_h, int pb_w, hipStream_t s,
                           float* part = nullptr);
// Deterministic mode (conv_tune("deterministic", 1)): the wgrad launches
// above take a slot workspace of this many floats (0 = mode off) and add the
// per-workgroup slots in a fixed order instead of with float atomics.
int64_t wgrad_part_floats(int cin, int cout, bool conv1);

}  // namespace conv
}  // namespace sa
