// Reference-precision (exact fp32) conv kernels for gfx950: NHWC fp32
// implicit GEMM on v_mfma_f32_16x16x4_f32 (f32 inputs, f32 accumulate, one
// rounding per product - bit-for-bit an fmaf chain, no xf32/TF32 shortcut).
//
// One templated forward kernel covers every conv the agent needs
// (reference experiment.py:153-189): the shallow torso's 8x8/4, 4x4/2, 3x3/2
// (TF-SAME, incl. the asymmetric W pad 0/1 of the third layer), the deep
// ResNet's 3x3/1 convs, uint8 frames (x/255 on load, any C <= 4 so RGB and
// Atari-style 4-frame stacks share the path) and, with flipped/transposed
// weights over a zero-dilated source, the data gradient.  Weight gradients
// are a pixel-reduction GEMM with a fixed-order two-stage reduction
// (deterministic: per-workgroup partials, then one summing pass).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sa {

// The current device's sticky error words, int32[4] zero-initialised device
// memory (bindings.cpp): [0] the LSTM recurrence's timeout word, [1] the
// conv kernels' hand-off timeout word.  The RMSProp guard consumes both.
unsigned* device_error_words();

namespace cf32 {

// kSrcPoolGrad: the source is the gradient of a 3x3/2 SAME max-pool's
// OUTPUT (dP [N, Hp, Wp, C] + its argmax codes); the kernel gathers the
// pre-pool gradient on load (sum of dP over the windows whose argmax is the
// position, windows in ascending order: bitwise the maxpool_bwd result), so
// the pre-pool gradient is never materialised.
enum SrcKind { kSrcF32 = 0, kSrcU8 = 1, kSrcPoolGrad = 2 };

// Max-pool geometry for the gather (pre-pool dims come from the caller).
struct PoolGeom {
  const uint8_t* arg;  // [N, Hp, Wp, C] first-max tap codes dy*3+dx
  int Hp, Wp, pbh, pbw;
};

// Forward conv / data gradient.  The kernel computes
//   out[n, oy, ox, co] = sum_{ky,kx,i} L[n, oy*S + ky, ox*S + kx, i] * Wk[ky,kx,i,co]
// over the LDS image L of the source: source pixel (j, i) sits at image
// position (j*D + pt, i*D + pl), zeros elsewhere (padding and dilation).
//   forward : D = 1, S = stride, Wk = W (HWIO), pads = TF-SAME pad_before
//   dgrad   : D = stride, S = 1, Wk = W flipped in (ky, kx) and transposed in
//             (ci, co) (flip = true), pads = K - 1 - pad_before
// Epilogue: v = acc [+ bias]; [v = mask > 0 ? v : 0]; [v += add]; [relu].
struct ConvArgs {
  const void* src;     // [N, Hs, Ws, Cs] fp32 (or uint8 frames, Cs <= 4)
  const float* w;      // HWIO [K, K, wcin, wcout]
  const float* bias;   // [Cout] or null
  const float* mask;   // [N, Ho, Wo, Cout] or null (ReLU derivative source)
  const float* add;    // [N, Ho, Wo, Cout] or null (residual / skip)
  float* out;          // [N, Ho, Wo, Cout]
  int N, Hs, Ws, Cs;   // source dims
  int Ho, Wo, Cout;    // output dims
  int pt, pl, D;       // image placement of the source
  int wcin, wcout;
  int relu_in, relu_out;
  PoolGeom pool;       // src_kind == kSrcPoolGrad: src is dP, (Hs, Ws) pre-pool
  // strided output placement (0 = identity): launch output (oy, ox) lands at
  // out[n, oy*ostr + ooy, ox*ostr + oox] of an [N, Hf, Wf, Cout] array (and
  // mask / add are read there): one phase of a phase-decomposed dgrad
  int ostr, ooy, oox, Hf, Wf;
  // phase-stacked dgrad (phase_c > 0): output channel co of the launch is
  // channel co % phase_c of phase k = co / phase_c = (ry, rx) (S = ostr);
  // launch output (oy, ox) lands at dX[ostr*(oy+ooy) + ry - pt_ph,
  // ostr*(ox+oox) + rx - pl_ph] when inside [0,Hf) x [0,Wf), else dropped
  int phase_c, pt_ph, pl_ph;
};

// Weight gradient of the FORWARD conv (stride S, pads pt/pl):
//   dW[ky,kx,ci,co] += sum_{n,oy,ox} X[n, oy*S+ky-pt, ox*S+kx-pl, ci] * dY[n,oy,ox,co]
//   db[co]          += sum dY[n,oy,ox,co]          (when db != null)
// X is the layer input (optionally ReLU'd on load, or uint8 frames / 255).
struct WgradArgs {
  const void* src;     // [N, H, W, Cin]
  const float* dy;     // [N, Ho, Wo, Cout]
  float* dw;           // [K, K, Cin, Cout], accumulated
  float* db;           // [Cout] or null, accumulated
  int N, H, W, Cin;
  int Ho, Wo, Cout;
  int pt, pl;
  int relu_in;
  PoolGeom pool;       // pool.arg != null: dy is dP, (Ho, Wo) pre-pool dims
  int dw_cin = 0;      // > 0: dw has this many input channels (<= Cin; the
                       // stage-0 weights of an RGB frame staged as 4 channels)
};

// Winograd F(2x2,3x3) fp32 path (conv_wino.hip) for 3x3/1 SAME convs with
// 16/32 channels in and out (forward and data gradient); false when the
// shape is not covered.  SA_F32_WINO=0 disables it (direct implicit GEMM).
bool wino_enabled();

// Deferred weight-gradient slot reductions: while on, every fixed-order
// slot sum (wgrad_reduce / wgrad_reduce_slots) is queued instead of
// launched, and wgrad_flush launches all queued sums as ONE kernel (the
// torso backward's ~15 reductions become one launch).  The caller keeps the
// slot workspaces alive until the flush.  Per host thread.
void wgrad_set_defer(bool on);
int wgrad_flush(hipStream_t s);  // -> number of reductions launched

// Fault injection (tests): 1 = every bounded intra-workgroup hand-off wait of
// the fused Winograd backward reports a timeout.  Returns the old setting.
int conv_wino_fault(int v);
// Compile-time-geometry Winograd instances on (1) / off (0); returns the old
// setting (tests compare both forms bitwise).
int conv_wino_geo(int v);
// CUs the persistent conv grids are sized for: 256 - 8 R, where R CUs per
// XCD are left to a concurrently running stream (the time-chunked LSTM
// pipeline).  conv_cu_reserve(R) sets R (0..16; -1 reads) and returns the
// previous value; the default comes from SA_CU_RESERVE (0).  Launch-time
// state: a captured graph keeps the grids it was captured with.
int conv_cu_reserve(int r);
// CUs the persistent grids are sized for now: 256 - 8 * conv_cu_reserve(-1).
int conv_cus();
bool wino_conv_launch(const ConvArgs& a, bool flip, hipStream_t s);
// Stage head with the 3x3/2 SAME max-pool fused (conv_wino.hip): x [N,H,W,Cin]
// -> pooled [N,H/2,W/2,Cout] + argmax codes, the 3x3/1 conv + bias in
// Winograd form, the pre-pool map only in LDS.  (Cin, Cout) = (16, 32) with
// W in {32, 48, 64} and H % 4 == 0 (stage 1), (4, 16) with W in {64, 96} and
// H % 4 == 0 (stage 0 on the 4-channel image), (32, 32) at 18x24 (stage 2,
// whole-image ranges); `side` holds >= wino_conv_pool_side_floats floats of
// scratch.  False (nothing launched) when the shape is not covered.
// `stages` (or SA_F32_WINO_POOL when < 0): bit 0 stage 1, bit 1 stage 0,
// bit 2 stage 2 (default 7).
int64_t wino_conv_pool_side_floats(int W, int Cout);
bool wino_conv_pool_launch(const float* x, const float* w, const float* b, float* pooled,
                           uint8_t* arg, float* side, int64_t side_floats, int N, int H, int W,
                           int Cin, int Cout, int stages, hipStream_t s);
// Winograd weight gradient (3x3/1 SAME, 16/32 channels; SA_F32_WINO_WG=0
// disables): per-workgroup partials in the wgrad slot layout of `ws`, then
// the same fixed-order slot reduction as the direct kernel.
bool wino_wgrad_enabled();
bool wino_wgrad_launch(const WgradArgs& a, float* ws, hipStream_t s);
// Fused backward of a 3x3/1 SAME conv (x: C channels, dY: Cy): dX =
// dgrad(dY) [* (x > 0) when mask_x: the residual convs, whose input is the
// mask] [+ add]; dW += sum relu?(x) (x) dY, db += sum dY (accumulated); dY
// and x read once.  `ws` holds >= ws_floats floats of slot workspace.
// False when the shape is not covered (then nothing ran).
bool wino_bwd_fused_enabled();
bool wino_bwd_fused_launch(const float* dy, const float* w, const float* x, const float* add,
                           float* out, int relu_x, int mask_x, int N, int H, int W, int C,
                           int Cy, float* ws, int64_t ws_floats, float* dw, float* db,
                           hipStream_t s);
// Fixed-order sum of G slot partials [G][rows16][Cout] (rows tap*Cin + ci,
// row 9*Cin = bias) accumulated into dW (HWIO 3x3) / db.
void wgrad_reduce_slots(const float* part, int G, int rows16, int Cout, int Cin, float* dw,
                        float* db, hipStream_t s);

// Returns false (and launches nothing) when no instance matches the shape;
// the bindings turn that into an error naming the shape.
bool conv_launch(const ConvArgs& a, int K, int S, int src_kind, bool flip,
                 hipStream_t s);
// Workgroup slots of one wgrad launch (partial-sum rows in the workspace).
int64_t wgrad_slots(int K, int cinp, int cout);
// `ws` must hold wgrad_workspace_floats(K, Cin, Cout) floats.
int64_t wgrad_workspace_floats(int K, int Cin, int Cout);
bool wgrad_launch(const WgradArgs& a, int K, int S, int src_kind, float* ws,
                  hipStream_t s);

// Fused conv3x3/1 (SAME) + bias + 3x3/2 SAME max-pool: y [N, Hp, Wp, Cout]
// and argmax codes; the pre-pool conv output only ever lives in LDS.
bool conv_pool_fwd_launch(const ConvArgs& a, int src_kind, int pbh, int pbw,
                          float* pooled, uint8_t* arg, hipStream_t s);

// 3x3/2 max-pool, TF SAME (pads pb_h/pb_w before, -inf padding):
// y [N, Hp, Wp, C] and the first maximal tap dy*3+dx per element.  C / 4
// must be a power of two (false otherwise).
bool maxpool_fwd_launch(const float* x, float* y, uint8_t* arg, int N, int H,
                        int W, int C, int Hp, int Wp, int pb_h, int pb_w,
                        hipStream_t s);
// dx[n, y, x, c] = sum of dy over the windows whose argmax is (y, x).
bool maxpool_bwd_launch(const float* dy, const uint8_t* arg, float* dx, int N,
                        int H, int W, int C, int Hp, int Wp, int pb_h, int pb_w,
                        hipStream_t s);
// uint8 frames [P pixels][Cs <= 4] -> fp32 [P][4] (x / 255, zero-padded)
void frames_f32_launch(const uint8_t* x, float* y, int64_t P, int Cs, hipStream_t s);
// dy *= (ref > 0), fp32, n % 4 == 0
void relu_mask_launch(float* dy, const float* ref, int64_t n, hipStream_t s);

}  // namespace cf32
}  // namespace sa
