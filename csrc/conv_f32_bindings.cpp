// Torch bindings for the exact-fp32 conv kernels (kernels/conv_f32.hip).
// Every op validates shapes on the host, allocates through the caching
// allocator and launches on the current stream (graph-capturable); a shape
// with no compiled instance raises instead of falling back.
#include <torch/extension.h>

#include <cstdlib>
#include <climits>
#include <algorithm>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "kernels/conv_f32.h"
#include "kernels/knobs.h"

namespace {

// Slot workspaces of the deferred weight-gradient reductions (see
// wgrad_set_defer): kept alive until cf32_wgrad_flush launches their sums.
thread_local bool t_defer = false;
thread_local std::vector<at::Tensor> t_keep;

at::Tensor slot_workspace(int64_t floats, const at::Tensor& like) {
  auto ws = at::empty({floats}, like.options().dtype(at::kFloat));
  if (t_defer) t_keep.push_back(ws);
  return ws;
}


hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

// A launch that fails (e.g. an LDS request the device refuses) must not
// leave its output uninitialised silently.
void check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  TORCH_CHECK(e == hipSuccess, what, ": kernel launch failed: ", hipGetErrorString(e));
}

int src_kind(const at::Tensor& x) {
  if (x.scalar_type() == at::kByte) return sa::cf32::kSrcU8;
  TORCH_CHECK(x.scalar_type() == at::kFloat, "conv source must be uint8 frames or float32");
  return sa::cf32::kSrcF32;
}

// Every activation / gradient tensor these kernels touch stays under 4 GB:
// the kernels and their tile schedules are validated up to that size (the
// Winograd stagers address one tensor with 32-bit buffer offsets).  Larger
// learner batches run the torso in frame chunks (ops/conv_f32.py
// MAX_FRAMES); an oversized call fails here instead of computing garbage.
void check_size(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.numel() * static_cast<int64_t>(t.element_size()) < (int64_t{1} << 32), name,
              " is ", t.numel() * t.element_size(),
              " bytes: fp32 conv tensors must stay under 4 GB (chunk the frames: "
              "ops/conv_f32.py MAX_FRAMES)");
}

void check_nhwc(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.dim() == 4, name,
              " must be a contiguous NHWC GPU tensor");
  check_size(t, name);
}

const float* opt_f32(const c10::optional<at::Tensor>& t, const at::Tensor& like,
                     const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->sizes() == like.sizes(),
              name, " must be a contiguous float32 tensor shaped like the output");
  return t->data_ptr<float>();
}

void check_w(const at::Tensor& w) {
  TORCH_CHECK(w.is_cuda() && w.is_contiguous() && w.scalar_type() == at::kFloat && w.dim() == 4 &&
                  w.size(0) == w.size(1),
              "weights must be contiguous float32 HWIO [K,K,Cin,Cout]");
}

// y = conv(relu_in ? relu(x) : x, w, stride, pads) [+ b] [* (mask > 0)] [+ add] [relu]
at::Tensor conv_fwd(at::Tensor x, at::Tensor w, c10::optional<at::Tensor> b, int64_t stride,
                    int64_t pt, int64_t pl, int64_t Ho, int64_t Wo, bool relu_in,
                    c10::optional<at::Tensor> add, bool relu_out) {
  check_nhwc(x, "x");
  check_w(w);
  const int kind = src_kind(x);
  TORCH_CHECK(w.size(2) == x.size(3), "weights Cin ", w.size(2), " != input channels ", x.size(3));
  const int64_t Cout = w.size(3);
  const c10::DeviceGuard g(x.device());
  auto y = at::empty({x.size(0), Ho, Wo, Cout}, x.options().dtype(at::kFloat));
  check_size(y, "y");
  sa::cf32::ConvArgs a{};
  a.src = x.data_ptr();
  a.w = w.data_ptr<float>();
  if (b.has_value() && b->defined()) {
    TORCH_CHECK(b->numel() == Cout && b->scalar_type() == at::kFloat && b->is_contiguous(), "bias");
    a.bias = b->data_ptr<float>();
  }
  a.add = opt_f32(add, y, "add");
  a.out = y.data_ptr<float>();
  a.N = x.size(0); a.Hs = x.size(1); a.Ws = x.size(2); a.Cs = x.size(3);
  a.Ho = Ho; a.Wo = Wo; a.Cout = Cout;
  a.pt = pt; a.pl = pl; a.D = 1;
  a.wcin = w.size(2); a.wcout = Cout;
  a.relu_in = relu_in; a.relu_out = relu_out;
  TORCH_CHECK(sa::cf32::conv_launch(a, w.size(0), stride, kind, false, stream()),
              "conv_f32: no kernel instance for K=", w.size(0), " stride=", stride, " Cin=",
              x.size(3), " Cout=", Cout, " src=", kind == sa::cf32::kSrcU8 ? "uint8" : "f32");
  check_launch("cf32_conv_fwd");
  return y;
}

// dx [N,H,W,Cin] of y = conv(x, w, stride, pads): correlation of the
// stride-dilated dy with the flipped, transposed weights; then
// [* (mask > 0)] [+ add].
sa::cf32::PoolGeom pool_geom(const c10::optional<at::Tensor>& arg, const at::Tensor& dP,
                             int64_t Hc, int64_t Wc, int64_t pbh, int64_t pbw) {
  sa::cf32::PoolGeom pg{};
  if (!arg.has_value() || !arg->defined()) return pg;
  TORCH_CHECK(arg->sizes() == dP.sizes() && arg->scalar_type() == at::kByte &&
                  arg->is_contiguous(), "pool argmax must be uint8 shaped like dP");
  TORCH_CHECK(dP.size(1) == (Hc + 1) / 2 && dP.size(2) == (Wc + 1) / 2 && dP.size(3) % 4 == 0,
              "dP must be the 3x3/2 pool of a ", Hc, "x", Wc, " map");
  pg.arg = arg->data_ptr<uint8_t>();
  pg.Hp = dP.size(1); pg.Wp = dP.size(2); pg.pbh = pbh; pg.pbw = pbw;
  return pg;
}

// SA_F32_DGRAD_STACK=1: one phase-stacked launch instead of S*S phase
// launches (measured equal: shallow2 391 vs 361-381 us, shallow3 611 vs
// 584-618 us - the per-tile work stays one tiny image either way)
bool phase_stacked() {
  static const bool on = sa::env_knob("SA_F32_DGRAD_STACK", 0) == 1;
  return on;
}

at::Tensor conv_dgrad(at::Tensor dy, at::Tensor w, int64_t stride, int64_t pt, int64_t pl,
                      int64_t H, int64_t W, c10::optional<at::Tensor> mask,
                      c10::optional<at::Tensor> add, c10::optional<at::Tensor> pool_arg,
                      int64_t pool_pbh, int64_t pool_pbw) {
  check_nhwc(dy, "dy");
  check_w(w);
  TORCH_CHECK(dy.scalar_type() == at::kFloat, "dy must be float32");
  TORCH_CHECK(w.size(3) == dy.size(3), "weights Cout != dy channels");
  const int64_t K = w.size(0), Cin = w.size(2);
  const c10::DeviceGuard g(dy.device());
  auto dx = at::empty({dy.size(0), H, W, Cin}, dy.options());
  check_size(dx, "dx");
  static const bool phase = sa::env_knob("SA_F32_DGRAD_PHASE", 1) != 0;
  if (stride > 1 && !(pool_arg.has_value() && pool_arg->defined()) && phase) {
    // Phase decomposition: dX rows i = S q + r - pt get the taps k = r + S j
    // only, so each of the S x S output phases is a stride-1 correlation of
    // the UNDILATED dY with a ceil(K/S)^2 sub-kernel (missing taps zero) -
    // no MFMA work on the dilation zeros (1/S^2 of the dilated form's).
    const int64_t S = stride, Kq = (K + S - 1) / S;
    const int64_t Hy = dy.size(1), Wy = dy.size(2);
    if (Cin % 16 == 0 && phase_stacked()) {
      // ONE launch for all S*S phases: their sub-kernels stacked along the
      // output channels (Cout = S*S*Cin), the epilogue routes each 16-channel
      // block to its phase's pixels - dY staged once, S*S times the MFMA
      // columns per tile (tiny 9x12 / 18x24 outputs fill the waves)
      int64_t qy0 = INT64_MAX, qy1 = INT64_MIN, qx0 = INT64_MAX, qx1 = INT64_MIN;
      for (int64_t r = 0; r < S; ++r) {
        qy0 = std::min(qy0, (pt - r + S - 1) / S);
        qy1 = std::max(qy1, (H - 1 + pt - r) / S);
        qx0 = std::min(qx0, (pl - r + S - 1) / S);
        qx1 = std::max(qx1, (W - 1 + pl - r) / S);
      }
      auto wst = at::zeros({Kq, Kq, S * S * Cin, w.size(3)}, w.options());
      for (int64_t ry = 0; ry < S; ++ry)
        for (int64_t rx = 0; rx < S; ++rx) {
          const int64_t ny = (K - ry + S - 1) / S, nx = (K - rx + S - 1) / S;
          const int64_t k = ry * S + rx;
          wst.narrow(0, 0, ny).narrow(1, 0, nx).narrow(2, k * Cin, Cin).copy_(
              w.slice(0, ry, K, S).slice(1, rx, K, S));
        }
      sa::cf32::ConvArgs a{};
      a.src = dy.data_ptr();
      a.w = wst.data_ptr<float>();
      a.mask = opt_f32(mask, dx, "mask");
      a.add = opt_f32(add, dx, "add");
      a.out = dx.data_ptr<float>();
      a.N = dy.size(0); a.Hs = Hy; a.Ws = Wy; a.Cs = dy.size(3);
      a.Ho = qy1 - qy0 + 1; a.Wo = qx1 - qx0 + 1; a.Cout = S * S * Cin;
      a.pt = Kq - 1 - qy0; a.pl = Kq - 1 - qx0; a.D = 1;
      a.wcin = S * S * Cin; a.wcout = w.size(3);
      a.ostr = S; a.ooy = qy0; a.oox = qx0; a.Hf = H; a.Wf = W;
      a.phase_c = Cin; a.pt_ph = pt; a.pl_ph = pl;
      TORCH_CHECK(sa::cf32::conv_launch(a, Kq, 1, sa::cf32::kSrcF32, true, stream()),
                  "conv_f32 dgrad: no phase-stacked kernel for K=", Kq, " dy channels=",
                  dy.size(3), " dx channels=", S * S * Cin);
      check_launch("cf32_conv_dgrad(stacked)");
      return dx;
    }
    // every phase's sub-kernel at once: w zero-padded to Kq * S taps per
    // axis, tap k = S j + r -> wall[r_y][r_x][j_y][j_x] (missing taps zero);
    // a pad and one copy instead of a fill and a copy per phase
    auto wall = at::constant_pad_nd(w, {0, 0, 0, 0, 0, Kq * S - K, 0, Kq * S - K})
                    .view({Kq, S, Kq, S, Cin, w.size(3)})
                    .permute({1, 3, 0, 2, 4, 5})
                    .contiguous();
    for (int64_t ry = 0; ry < S; ++ry) {
      // q range with 0 <= S q + ry - pt < H
      const int64_t qy0 = (pt - ry + S - 1) >= 0 ? (pt - ry + S - 1) / S : 0;
      const int64_t qy1 = (H - 1 + pt - ry) / S;
      if (qy1 < qy0) continue;
      for (int64_t rx = 0; rx < S; ++rx) {
        const int64_t qx0 = (pl - rx + S - 1) >= 0 ? (pl - rx + S - 1) / S : 0;
        const int64_t qx1 = (W - 1 + pl - rx) / S;
        if (qx1 < qx0) continue;
        auto wsub = wall.select(0, ry).select(0, rx);  // [Kq, Kq, Cin, Cout]
        sa::cf32::ConvArgs a{};
        a.src = dy.data_ptr();
        a.w = wsub.data_ptr<float>();
        a.mask = opt_f32(mask, dx, "mask");
        a.add = opt_f32(add, dx, "add");
        a.out = dx.data_ptr<float>();
        a.N = dy.size(0); a.Hs = Hy; a.Ws = Wy; a.Cs = dy.size(3);
        a.Ho = qy1 - qy0 + 1; a.Wo = qx1 - qx0 + 1; a.Cout = Cin;
        // out[q] = sum_j dy[q - j] wsub[j]: flipped taps, Kq - 1 rows above
        a.pt = Kq - 1 - qy0; a.pl = Kq - 1 - qx0; a.D = 1;
        a.wcin = Cin; a.wcout = w.size(3);
        a.ostr = S; a.ooy = S * qy0 + ry - pt; a.oox = S * qx0 + rx - pl;
        a.Hf = H; a.Wf = W;
        TORCH_CHECK(sa::cf32::conv_launch(a, Kq, 1, sa::cf32::kSrcF32, true, stream()),
                    "conv_f32 dgrad: no phase kernel for K=", Kq, " dy channels=",
                    dy.size(3), " dx channels=", Cin);
        check_launch("cf32_conv_dgrad(phase)");
      }
    }
    return dx;
  }
  // dy is the conv output's gradient, or (pool_arg) the gradient of its
  // 3x3/2 max-pool, gathered on load
  const int64_t Hc = (H + stride - 1) / stride, Wc = (W + stride - 1) / stride;
  const auto pg = pool_geom(pool_arg, dy, Hc, Wc, pool_pbh, pool_pbw);
  sa::cf32::ConvArgs a{};
  a.pool = pg;
  a.src = dy.data_ptr();
  a.w = w.data_ptr<float>();
  a.mask = opt_f32(mask, dx, "mask");
  a.add = opt_f32(add, dx, "add");
  a.out = dx.data_ptr<float>();
  a.N = dy.size(0); a.Hs = pg.arg ? Hc : dy.size(1); a.Ws = pg.arg ? Wc : dy.size(2);
  a.Cs = dy.size(3);
  a.Ho = H; a.Wo = W; a.Cout = Cin;
  a.pt = K - 1 - pt; a.pl = K - 1 - pl; a.D = stride;
  a.wcin = Cin; a.wcout = w.size(3);
  const int kind = pg.arg ? sa::cf32::kSrcPoolGrad : sa::cf32::kSrcF32;
  TORCH_CHECK(sa::cf32::conv_launch(a, K, 1, kind, true, stream()),
              "conv_f32 dgrad: no kernel instance for K=", K, " dy channels=", dy.size(3),
              " dx channels=", Cin);
  check_launch("cf32_conv_dgrad");
  return dx;
}

// dw += sum x^T dy (HWIO), db += sum dy; x: the layer input (uint8 frames
// or float32, optionally ReLU'd on load).  Deterministic (no atomics).
void conv_wgrad(at::Tensor x, at::Tensor dy, int64_t stride, int64_t pt, int64_t pl,
                bool relu_in, at::Tensor dw, c10::optional<at::Tensor> db,
                c10::optional<at::Tensor> pool_arg, int64_t pool_pbh, int64_t pool_pbw) {
  check_nhwc(x, "x");
  check_nhwc(dy, "dy");
  TORCH_CHECK(dy.scalar_type() == at::kFloat, "dy must be float32");
  check_w(dw);
  const int kind = src_kind(x);
  const int64_t K = dw.size(0);
  // dw may have fewer input channels than x (RGB weights, 4-channel image)
  TORCH_CHECK(dw.size(2) <= x.size(3) && dw.size(3) == dy.size(3), "dw shape");
  const c10::DeviceGuard g(x.device());
  auto ws = slot_workspace(sa::cf32::wgrad_workspace_floats(K, x.size(3), dy.size(3)), dy);
  sa::cf32::WgradArgs a{};
  a.src = x.data_ptr();
  a.dy = dy.data_ptr<float>();
  a.dw = dw.data_ptr<float>();
  if (db.has_value() && db->defined()) {
    TORCH_CHECK(db->numel() == dy.size(3) && db->scalar_type() == at::kFloat &&
                    db->is_contiguous(), "db");
    a.db = db->data_ptr<float>();
  }
  a.N = x.size(0); a.H = x.size(1); a.W = x.size(2); a.Cin = x.size(3);
  a.Ho = dy.size(1); a.Wo = dy.size(2); a.Cout = dy.size(3);
  if (pool_arg.has_value() && pool_arg->defined()) {
    // dy is the gradient of the conv output's 3x3/2 max-pool
    a.Ho = (x.size(1) + stride - 1) / stride;
    a.Wo = (x.size(2) + stride - 1) / stride;
    a.pool = pool_geom(pool_arg, dy, a.Ho, a.Wo, pool_pbh, pool_pbw);
  }
  a.pt = pt; a.pl = pl; a.relu_in = relu_in;
  a.dw_cin = dw.size(2);
  TORCH_CHECK(sa::cf32::wgrad_launch(a, K, stride, kind, ws.data_ptr<float>(), stream()),
              "conv_f32 wgrad: no kernel instance for K=", K, " stride=", stride, " Cin=",
              x.size(3), " Cout=", dy.size(3));
  check_launch("cf32_conv_wgrad");
}

// Backward of a 3x3/1 SAME conv: returns dX = dgrad(dy, w) [* (x > 0) when
// mask: the deep torso's residual convs, whose input is also the data
// gradient's ReLU mask] [+ add] and accumulates dw += relu?(x)^T dy, db +=
// sum dy.  One fused pass (dY and x read once) where a kernel covers the
// shape (residual convs, the stage heads' 16 -> 32 and 32 -> 32), else the
// separate data-gradient and weight-gradient kernels.
at::Tensor conv_bwd_fused(at::Tensor dy, at::Tensor w, at::Tensor x, bool relu_x,
                          at::Tensor dw, c10::optional<at::Tensor> db,
                          c10::optional<at::Tensor> add, bool mask) {
  check_nhwc(dy, "dy");
  check_nhwc(x, "x");
  check_w(w);
  check_w(dw);
  TORCH_CHECK(dy.scalar_type() == at::kFloat && x.scalar_type() == at::kFloat, "float32");
  TORCH_CHECK(w.size(0) == 3 && w.size(2) == x.size(3) && w.size(3) == dy.size(3) &&
                  dy.size(0) == x.size(0) && dy.size(1) == x.size(1) && dy.size(2) == x.size(2),
              "conv_bwd_fused: 3x3/1 SAME conv (x and dy of one spatial shape)");
  TORCH_CHECK(dw.sizes() == w.sizes(), "dw shape");
  const c10::DeviceGuard g(dy.device());
  auto dx = at::empty(x.sizes(), x.options());
  const float* addp = opt_f32(add, dx, "add");
  float* dbp = nullptr;
  if (db.has_value() && db->defined()) {
    TORCH_CHECK(db->numel() == dy.size(3) && db->scalar_type() == at::kFloat && db->is_contiguous(),
                "db");
    dbp = db->data_ptr<float>();
  }
  const int C = x.size(3), Cy = dy.size(3);
  if (sa::cf32::wino_bwd_fused_enabled()) {
    const int64_t wsf = sa::cf32::wgrad_workspace_floats(3, C, Cy);
    auto ws = slot_workspace(wsf, dy);
    if (sa::cf32::wino_bwd_fused_launch(dy.data_ptr<float>(), w.data_ptr<float>(),
                                        x.data_ptr<float>(), addp, dx.data_ptr<float>(),
                                        relu_x ? 1 : 0, mask ? 1 : 0, x.size(0), x.size(1),
                                        x.size(2), C, Cy, ws.data_ptr<float>(), wsf,
                                        dw.data_ptr<float>(), dbp, stream())) {
      check_launch("cf32_conv_bwd_fused");
      return dx;
    }
  }
  // separate kernels: weight gradient, then the (masked) data gradient
  conv_wgrad(x, dy, 1, 1, 1, relu_x, dw, db, c10::nullopt, 0, 0);
  return conv_dgrad(dy, w, 1, 1, 1, x.size(1), x.size(2),
                    mask ? c10::optional<at::Tensor>(x) : c10::nullopt, add, c10::nullopt, 0, 0);
}

// Fused stage head: maxpool3x3/2(conv3x3/1(x) + b) -> {pooled, argmax}
std::vector<at::Tensor> conv_pool_fwd(at::Tensor x, at::Tensor w, at::Tensor b, int64_t pbh,
                                      int64_t pbw) {
  check_nhwc(x, "x");
  check_w(w);
  const int kind = src_kind(x);
  TORCH_CHECK(w.size(0) == 3 && w.size(2) == x.size(3), "conv_pool_fwd: 3x3 weights");
  TORCH_CHECK(b.numel() == w.size(3) && b.scalar_type() == at::kFloat && b.is_contiguous(), "bias");
  const c10::DeviceGuard g(x.device());
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), Cout = w.size(3);
  auto y = at::empty({N, (H + 1) / 2, (W + 1) / 2, Cout}, x.options().dtype(at::kFloat));
  check_size(y, "y");
  auto arg = at::empty(y.sizes(), x.options().dtype(at::kByte));
  sa::cf32::ConvArgs a{};
  a.src = x.data_ptr();
  a.w = w.data_ptr<float>();
  a.bias = b.data_ptr<float>();
  a.N = N; a.Hs = H; a.Ws = W; a.Cs = x.size(3);
  a.Ho = H; a.Wo = W; a.Cout = Cout;
  a.pt = 1; a.pl = 1; a.D = 1;
  a.wcin = w.size(2); a.wcout = Cout;
  TORCH_CHECK(sa::cf32::conv_pool_fwd_launch(a, kind, pbh, pbw, y.data_ptr<float>(),
                                             arg.data_ptr<uint8_t>(), stream()),
              "conv_pool_fwd: no kernel instance for Cin=", x.size(3), " Cout=", Cout);
  check_launch("cf32_conv_pool_fwd");
  return {y, arg};
}

// Deep stage head (16 -> 32, or 4 -> 16 on the stage-0 image) with the
// max-pool fused into the Winograd conv (conv_wino.hip wino_conv_pool_kernel):
// {pooled, argmax}, or {} when the shape is not covered (nothing ran; the
// caller takes the other kernels)
std::vector<at::Tensor> wino_conv_pool_fwd(at::Tensor x, at::Tensor w, at::Tensor b,
                                           int64_t stages) {
  check_nhwc(x, "x");
  check_w(w);
  TORCH_CHECK(x.scalar_type() == at::kFloat, "x must be float32");
  TORCH_CHECK(b.scalar_type() == at::kFloat && b.is_contiguous() && b.numel() == w.size(3), "bias");
  const int64_t Cin = x.size(3), Cout = w.size(3);
  if (w.size(0) != 3 || w.size(2) != Cin ||
      !((Cin == 16 && Cout == 32) || (Cin == 4 && Cout == 16) || (Cin == 32 && Cout == 32)))
    return {};
  const c10::DeviceGuard g(x.device());
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2);
  if (H % 2 != 0 || W % 2 != 0) return {};
  auto y = at::empty({N, H / 2, W / 2, Cout}, x.options());
  check_size(y, "y");
  auto arg = at::empty(y.sizes(), x.options().dtype(at::kByte));
  const int64_t sf = sa::cf32::wino_conv_pool_side_floats(static_cast<int>(W), static_cast<int>(Cout));
  auto side = at::empty({sf}, x.options());
  if (!sa::cf32::wino_conv_pool_launch(x.data_ptr<float>(), w.data_ptr<float>(),
                                       b.data_ptr<float>(), y.data_ptr<float>(),
                                       arg.data_ptr<uint8_t>(), side.data_ptr<float>(), sf,
                                       static_cast<int>(N), static_cast<int>(H),
                                       static_cast<int>(W), static_cast<int>(Cin),
                                       static_cast<int>(Cout), static_cast<int>(stages),
                                       stream()))
    return {};
  check_launch("cf32_wino_conv_pool_fwd");
  return {y, arg};
}

std::vector<at::Tensor> maxpool_fwd(at::Tensor x, int64_t pb_h, int64_t pb_w) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.size(3) % 4 == 0, "maxpool: float32, C % 4 == 0");
  const c10::DeviceGuard g(x.device());
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t Hp = (H + 1) / 2, Wp = (W + 1) / 2;
  auto y = at::empty({N, Hp, Wp, C}, x.options());
  auto arg = at::empty({N, Hp, Wp, C}, x.options().dtype(at::kByte));
  TORCH_CHECK(sa::cf32::maxpool_fwd_launch(x.data_ptr<float>(), y.data_ptr<float>(),
                                           arg.data_ptr<uint8_t>(), N, H, W, C, Hp, Wp,
                                           pb_h, pb_w, stream()),
              "maxpool: C / 4 must be a power of two");
  check_launch("cf32_maxpool_fwd");
  return {y, arg};
}

at::Tensor maxpool_bwd(at::Tensor dy, at::Tensor arg, int64_t H, int64_t W, int64_t pb_h,
                       int64_t pb_w) {
  check_nhwc(dy, "dy");
  TORCH_CHECK(dy.scalar_type() == at::kFloat && dy.size(3) % 4 == 0, "dy float32, C % 4 == 0");
  TORCH_CHECK(arg.sizes() == dy.sizes() && arg.scalar_type() == at::kByte && arg.is_contiguous(),
              "argmax");
  TORCH_CHECK(dy.size(1) == (H + 1) / 2 && dy.size(2) == (W + 1) / 2, "pooled shape");
  const c10::DeviceGuard g(dy.device());
  auto dx = at::empty({dy.size(0), H, W, dy.size(3)}, dy.options());
  check_size(dx, "dx");
  TORCH_CHECK(sa::cf32::maxpool_bwd_launch(dy.data_ptr<float>(), arg.data_ptr<uint8_t>(),
                                           dx.data_ptr<float>(), dy.size(0), H, W,
                                           dy.size(3), dy.size(1), dy.size(2), pb_h, pb_w,
                                           stream()),
              "maxpool: C / 4 must be a power of two");
  check_launch("cf32_maxpool_bwd");
  return dx;
}

at::Tensor frames_f32(at::Tensor x) {
  check_nhwc(x, "frames");
  TORCH_CHECK(x.scalar_type() == at::kByte && x.size(3) >= 1 && x.size(3) <= 4,
              "frames must be uint8 NHWC with 1..4 channels");
  const c10::DeviceGuard g(x.device());
  auto y = at::empty({x.size(0), x.size(1), x.size(2), 4}, x.options().dtype(at::kFloat));
  check_size(y, "y");
  sa::cf32::frames_f32_launch(x.data_ptr<uint8_t>(), y.data_ptr<float>(),
                              x.size(0) * x.size(1) * x.size(2), x.size(3), stream());
  check_launch("cf32_frames_f32");
  return y;
}

void relu_mask_(at::Tensor dy, at::Tensor ref) {
  TORCH_CHECK(dy.is_cuda() && dy.is_contiguous() && dy.scalar_type() == at::kFloat, "dy");
  TORCH_CHECK(ref.is_contiguous() && ref.scalar_type() == at::kFloat &&
                  ref.numel() == dy.numel() && dy.numel() % 4 == 0, "ref");
  const c10::DeviceGuard g(dy.device());
  sa::cf32::relu_mask_launch(dy.data_ptr<float>(), ref.data_ptr<float>(), dy.numel(), stream());
}

}  // namespace

void register_conv_f32_ops(pybind11::module& m) {
  using pybind11::arg;
  m.def("cf32_conv_fwd", &conv_fwd, arg("x"), arg("w"), arg("b"), arg("stride"), arg("pt"),
        arg("pl"), arg("Ho"), arg("Wo"), arg("relu_in") = false, arg("add") = pybind11::none(),
        arg("relu_out") = false);
  m.def("cf32_conv_dgrad", &conv_dgrad, arg("dy"), arg("w"), arg("stride"), arg("pt"), arg("pl"),
        arg("H"), arg("W"), arg("mask") = pybind11::none(), arg("add") = pybind11::none(),
        arg("pool_arg") = pybind11::none(), arg("pool_pbh") = 0, arg("pool_pbw") = 0);
  m.def("cf32_conv_wgrad", &conv_wgrad, arg("x"), arg("dy"), arg("stride"), arg("pt"), arg("pl"),
        arg("relu_in"), arg("dw"), arg("db") = pybind11::none(),
        arg("pool_arg") = pybind11::none(), arg("pool_pbh") = 0, arg("pool_pbw") = 0);
  m.def("cf32_conv_bwd_fused", &conv_bwd_fused, arg("dy"), arg("w"), arg("x"), arg("relu_x"),
        arg("dw"), arg("db") = pybind11::none(), arg("add") = pybind11::none(),
        arg("mask") = true);
  m.def("cf32_conv_pool_fwd", &conv_pool_fwd);
  m.def("cf32_wino_conv_pool_fwd", &wino_conv_pool_fwd, arg("x"), arg("w"), arg("b"),
        arg("stages") = -1);
  m.def("cf32_maxpool_fwd", &maxpool_fwd);
  m.def("cf32_maxpool_bwd", &maxpool_bwd);
  m.def("cf32_relu_mask_", &relu_mask_);
  m.def("cf32_frames_f32", &frames_f32);
  m.def("cf32_wino_fault", [](int v) { return sa::cf32::conv_wino_fault(v); });
  // 1: compile-time-geometry Winograd instances where the map has one
  // (default), 0: runtime geometry everywhere; returns the previous setting
  m.def("cf32_wino_geo", [](int v) { return sa::cf32::conv_wino_geo(v); });
  // R CUs per XCD left out of every persistent conv grid (-1 reads)
  m.def("cf32_cu_reserve", [](int r) { return sa::cf32::conv_cu_reserve(r); });
  // deferred weight-gradient reductions: defer(True) ... flush() -> one launch
  m.def("cf32_wgrad_defer", [](bool on) {
    t_defer = on;
    sa::cf32::wgrad_set_defer(on);
  });
  m.def("cf32_wgrad_flush", []() {
    const int n = sa::cf32::wgrad_flush(stream());
    t_keep.clear();
    return n;
  });
}
