// Torch bindings for the conv torso kernels (see kernels/conv_torso.hip).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "kernels/conv_launchers.h"

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_act(const at::Tensor& t, const char* name, int64_t C) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), name, " must be a contiguous GPU tensor");
  TORCH_CHECK(t.dim() == 4 && t.size(3) == C, name, " must be NHWC with C=", C);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
  // validated sizes (and the largest learner chunk: ops/conv_f32.py
  // MAX_FRAMES); an oversized call fails here instead of computing garbage
  TORCH_CHECK(t.numel() * 2 < (int64_t{1} << 32), name, " is ", t.numel() * 2,
              " bytes: bf16 conv tensors must stay under 4 GB (chunk the frames)");
}
void check_w(const at::Tensor& w, const at::Tensor& b, int64_t cin, int64_t cout) {
  TORCH_CHECK(w.is_cuda() && w.is_contiguous() && w.scalar_type() == at::kFloat,
              "weights must be contiguous fp32 GPU");
  TORCH_CHECK(w.dim() == 4 && w.size(0) == 3 && w.size(1) == 3 && w.size(2) == cin &&
              w.size(3) == cout, "weights must be [3,3,", cin, ",", cout, "]");
  TORCH_CHECK(b.numel() == cout && b.scalar_type() == at::kFloat && b.is_contiguous(),
              "bias must be fp32 [cout]");
}
void check_grad(const at::Tensor& dw, const at::Tensor& db, int64_t cin, int64_t cout) {
  TORCH_CHECK(dw.is_contiguous() && dw.scalar_type() == at::kFloat &&
              dw.numel() == 9 * cin * cout, "dw must be fp32 [3,3,cin,cout]");
  TORCH_CHECK(db.is_contiguous() && db.scalar_type() == at::kFloat && db.numel() == cout,
              "db must be fp32 [cout]");
}
bool supported(int64_t c) { return c == 16 || c == 32; }

// Deterministic mode: a stream-ordered slot workspace for the wgrad flush
// (empty when the mode is off).
at::Tensor wgrad_part(const at::Tensor& like, int64_t cin, int64_t cout, bool conv1) {
  const int64_t n = sa::conv::wgrad_part_floats((int)cin, (int)cout, conv1);
  return n ? at::empty({n}, like.options()) : at::Tensor();
}
float* ptr_or_null(const at::Tensor& t) { return t.defined() ? t.data_ptr<float>() : nullptr; }

std::vector<at::Tensor> conv1_pool_fwd(at::Tensor x, at::Tensor w, at::Tensor b,
                                       int64_t pb_h, int64_t pb_w) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.scalar_type() == at::kByte &&
              x.dim() == 4 && (x.size(3) == 3 || x.size(3) == 4),
              "frames must be uint8 NHWC with C = 3 or 4");
  const int64_t C = x.size(3);
  check_w(w, b, C, 16);
  const c10::DeviceGuard g(x.device());
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2);
  const int64_t Hp = (H + 1) / 2, Wo = (W + 1) / 2;
  auto pooled = at::empty({N, Hp, Wo, 16}, x.options().dtype(at::kBFloat16));
  auto arg = at::empty({N, Hp, Wo, 16}, x.options());
  sa::conv::conv1_pool_fwd_launch(x.data_ptr<uint8_t>(), w.data_ptr<float>(),
                                  b.data_ptr<float>(), pooled.data_ptr(),
                                  arg.data_ptr<uint8_t>(), N, H, W, C, pb_h, pb_w,
                                  stream());
  return {pooled, arg};
}

std::vector<at::Tensor> conv_pool_fwd(at::Tensor x, at::Tensor w, at::Tensor b,
                                      int64_t pb_h, int64_t pb_w) {
  const int64_t CIN = x.size(3), COUT = w.size(3);
  TORCH_CHECK(supported(CIN) && supported(COUT), "channels must be 16/32");
  check_act(x, "x", CIN);
  check_w(w, b, CIN, COUT);
  TORCH_CHECK(!(CIN == 32 && COUT == 16), "32->16 not instantiated");
  const c10::DeviceGuard g(x.device());
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2);
  const int64_t Hp = (H + 1) / 2, Wo = (W + 1) / 2;
  auto pooled = at::empty({N, Hp, Wo, COUT}, x.options());
  auto arg = at::empty({N, Hp, Wo, COUT}, x.options().dtype(at::kByte));
  sa::conv::conv_pool_fwd_launch(x.data_ptr(), w.data_ptr<float>(), b.data_ptr<float>(),
                                 pooled.data_ptr(), arg.data_ptr<uint8_t>(), N, H, W,
                                 CIN, COUT, pb_h, pb_w, stream());
  return {pooled, arg};
}

// y = conv(relu_in ? relu(x) : x) + b [+ resid] [then relu]
at::Tensor res_conv_fwd(at::Tensor x, at::Tensor w, at::Tensor b,
                        c10::optional<at::Tensor> resid, bool post_relu,
                        bool relu_in) {
  const int64_t C = x.size(3);
  TORCH_CHECK(supported(C), "channels must be 16/32");
  check_act(x, "x", C);
  check_w(w, b, C, C);
  const void* rp = nullptr;
  if (resid.has_value() && resid->defined()) {
    check_act(*resid, "resid", C);
    TORCH_CHECK(resid->sizes() == x.sizes(), "resid shape");
    rp = resid->data_ptr();
  }
  const c10::DeviceGuard g(x.device());
  auto y = at::empty_like(x);
  sa::conv::res_conv_fwd_launch(x.data_ptr(), w.data_ptr<float>(), b.data_ptr<float>(),
                                rp, y.data_ptr(), x.size(0), x.size(1), x.size(2), C,
                                post_relu, relu_in, stream());
  return y;
}

// -> {t, y}: t = relu(conv1(relu(x)) + b1), y = conv2(t) + b2 + x [+ relu]
std::vector<at::Tensor> res_block_fwd(at::Tensor x, at::Tensor w1, at::Tensor b1,
                                      at::Tensor w2, at::Tensor b2, bool post_relu) {
  const int64_t C = x.size(3);
  TORCH_CHECK(supported(C), "channels must be 16/32");
  check_act(x, "x", C);
  check_w(w1, b1, C, C);
  check_w(w2, b2, C, C);
  const c10::DeviceGuard g(x.device());
  auto t = at::empty_like(x);
  auto y = at::empty_like(x);
  sa::conv::res_block_fwd_launch(x.data_ptr(), w1.data_ptr<float>(), b1.data_ptr<float>(),
                                 w2.data_ptr<float>(), b2.data_ptr<float>(), t.data_ptr(),
                                 y.data_ptr(), x.size(0), x.size(1), x.size(2), C,
                                 post_relu, stream());
  return {t, y};
}

// dx = [skip +] dgrad(dy) * (act > 0); dW += relu?(act)^T dy; db += sum dy
at::Tensor res_conv_bwd(at::Tensor dy, at::Tensor act, c10::optional<at::Tensor> skip,
                        at::Tensor w, at::Tensor dw, at::Tensor db, bool relu_act) {
  const int64_t C = act.size(3);
  TORCH_CHECK(supported(C), "channels must be 16/32");
  check_act(dy, "dy", C);
  check_act(act, "act", C);
  TORCH_CHECK(dy.sizes() == act.sizes(), "dy/act shape");
  TORCH_CHECK(w.is_contiguous() && w.scalar_type() == at::kFloat && w.numel() == 9 * C * C,
              "w");
  check_grad(dw, db, C, C);
  const void* sp = nullptr;
  if (skip.has_value() && skip->defined()) {
    check_act(*skip, "skip", C);
    sp = skip->data_ptr();
  }
  const c10::DeviceGuard g(dy.device());
  auto dx = at::empty_like(act);
  auto part = wgrad_part(dw, C, C, false);
  sa::conv::res_conv_bwd_launch(dy.data_ptr(), act.data_ptr(), sp, w.data_ptr<float>(),
                                dx.data_ptr(), dw.data_ptr<float>(), db.data_ptr<float>(),
                                act.size(0), act.size(1), act.size(2), C, relu_act,
                                stream(), ptr_or_null(part));
  return dx;
}

c10::optional<at::Tensor> pool_conv_bwd(at::Tensor dP, at::Tensor arg, at::Tensor x,
                                        at::Tensor w, at::Tensor dw, at::Tensor db,
                                        bool need_dx, int64_t pb_h, int64_t pb_w) {
  const int64_t CIN = x.size(3), COUT = dP.size(3);
  TORCH_CHECK(supported(CIN) && supported(COUT), "channels must be 16/32");
  TORCH_CHECK(!(CIN == 32 && COUT == 16), "32->16 not instantiated");
  check_act(x, "x", CIN);
  check_act(dP, "dP", COUT);
  TORCH_CHECK(arg.sizes() == dP.sizes() && arg.scalar_type() == at::kByte &&
              arg.is_contiguous(), "argmax");
  TORCH_CHECK(dP.size(1) == (x.size(1) + 1) / 2 && dP.size(2) == (x.size(2) + 1) / 2,
              "pooled shape");
  TORCH_CHECK(w.numel() == 9 * CIN * COUT && w.scalar_type() == at::kFloat, "w");
  check_grad(dw, db, CIN, COUT);
  const c10::DeviceGuard g(x.device());
  c10::optional<at::Tensor> dx;
  void* dxp = nullptr;
  if (need_dx) {
    dx = at::empty_like(x);
    dxp = dx->data_ptr();
  }
  auto part = wgrad_part(dw, CIN, COUT, false);
  sa::conv::pool_conv_bwd_launch(dP.data_ptr(), arg.data_ptr<uint8_t>(), x.data_ptr(),
                                 w.data_ptr<float>(), dxp, dw.data_ptr<float>(),
                                 db.data_ptr<float>(), x.size(0), x.size(1), x.size(2),
                                 CIN, COUT, pb_h, pb_w, stream(), ptr_or_null(part));
  return dx;
}

void conv1_pool_bwd(at::Tensor dP, at::Tensor arg, at::Tensor x, at::Tensor dw,
                    at::Tensor db, int64_t pb_h, int64_t pb_w) {
  TORCH_CHECK(x.scalar_type() == at::kByte && x.dim() == 4 &&
              (x.size(3) == 3 || x.size(3) == 4) && x.is_contiguous(), "frames");
  const int64_t C = x.size(3);
  check_act(dP, "dP", 16);
  TORCH_CHECK(arg.sizes() == dP.sizes() && arg.scalar_type() == at::kByte, "argmax");
  TORCH_CHECK(dP.size(1) == (x.size(1) + 1) / 2 && dP.size(2) == (x.size(2) + 1) / 2,
              "pooled shape");
  check_grad(dw, db, C, 16);
  const c10::DeviceGuard g(x.device());
  auto part = wgrad_part(dw, C, 16, true);
  sa::conv::conv1_pool_bwd_launch(dP.data_ptr(), arg.data_ptr<uint8_t>(),
                                  x.data_ptr<uint8_t>(), dw.data_ptr<float>(),
                                  db.data_ptr<float>(), x.size(0), x.size(1),
                                  x.size(2), C, pb_h, pb_w, stream(), ptr_or_null(part));
}

}  // namespace

void register_conv_ops(pybind11::module& m) {
  m.def("conv1_pool_fwd", &conv1_pool_fwd);
  m.def("conv_pool_fwd", &conv_pool_fwd);
  m.def("res_block_fwd", &res_block_fwd);
  m.def("res_conv_fwd", &res_conv_fwd, pybind11::arg("x"), pybind11::arg("w"),
        pybind11::arg("b"), pybind11::arg("resid") = pybind11::none(),
        pybind11::arg("post_relu") = false, pybind11::arg("relu_in") = true);
  m.def("res_conv_bwd", &res_conv_bwd, pybind11::arg("dy"), pybind11::arg("act"),
        pybind11::arg("skip"), pybind11::arg("w"), pybind11::arg("dw"),
        pybind11::arg("db"), pybind11::arg("relu_act") = true);
  m.def("pool_conv_bwd", &pool_conv_bwd);
  m.def("conv1_pool_bwd", &conv1_pool_bwd);
  m.def("conv_tune", [](const std::string& key, int64_t value) {
          return sa::conv::conv_tune_set(key.c_str(), static_cast<int>(value));
        }, pybind11::arg("key"), pybind11::arg("value") = -1);
}
