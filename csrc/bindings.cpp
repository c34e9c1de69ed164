// PyTorch bindings for the gfx950 kernels (module scalable_agent_amd._C).
// Validates shapes/dtypes on the host, allocates outputs through the caching
// allocator and launches on the current HIP stream, so every op can be
// captured into a hipGraph (torch.cuda.CUDAGraph).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

#include "kernels/launchers.h"
#include "kernels/knobs.h"
#include "kernels/conv_launchers.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define SA_CHECK_CUDA(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define SA_CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define SA_CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define SA_CHECK(t) SA_CHECK_CUDA(t); SA_CHECK_CONTIG(t)

const uint8_t* u8ptr(const at::Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBool || t.scalar_type() == at::kByte,
              "mask must be bool/uint8");
  return reinterpret_cast<const uint8_t*>(t.data_ptr());
}

void rmsprop(at::Tensor w, at::Tensor g, at::Tensor ms, at::Tensor mom,
             at::Tensor frames, double lr0, double total_frames, double decay,
             double momentum, double eps, c10::optional<at::Tensor> guard,
             c10::optional<at::Tensor> lstm_err, double gscale) {
  SA_CHECK(w); SA_CHECK(g); SA_CHECK(ms); SA_CHECK(mom); SA_CHECK_CUDA(frames);
  SA_CHECK_F32(w); SA_CHECK_F32(g); SA_CHECK_F32(ms); SA_CHECK_F32(mom);
  TORCH_CHECK(frames.scalar_type() == at::kLong, "frames must be int64");
  TORCH_CHECK(w.numel() % 4 == 0, "flat buffer must be a multiple of 4");
  TORCH_CHECK(g.numel() == w.numel() && ms.numel() == w.numel() &&
              mom.numel() == w.numel(), "size mismatch");
  int* gp = nullptr;
  if (guard.has_value()) {
    SA_CHECK_CUDA(*guard);
    TORCH_CHECK(guard->scalar_type() == at::kInt && guard->numel() >= 4,
                "guard must be int32[4] (flag, skipped, lstm_timeouts, -)");
    gp = guard->data_ptr<int>();
  }
  unsigned* ep = nullptr;
  if (lstm_err.has_value() && lstm_err->defined()) {
    TORCH_CHECK(gp != nullptr, "lstm_err needs a guard");
    SA_CHECK_CUDA(*lstm_err);
    TORCH_CHECK(lstm_err->scalar_type() == at::kInt, "lstm_err must be int32");
    ep = reinterpret_cast<unsigned*>(lstm_err->data_ptr<int>());
  }
  const c10::DeviceGuard dguard(w.device());
  sa::rmsprop_launch(w.data_ptr<float>(), g.data_ptr<float>(),
                     ms.data_ptr<float>(), mom.data_ptr<float>(),
                     frames.data_ptr<int64_t>(), w.numel(), (float)lr0,
                     total_frames, (float)decay, (float)momentum, (float)eps,
                     (float)gscale, gp, ep, cur_stream());
}

void err_poison(at::Tensor slot, at::Tensor err) {
  SA_CHECK(slot); SA_CHECK_F32(slot); SA_CHECK_CUDA(err);
  TORCH_CHECK(slot.numel() >= 1, "sentinel slot must hold one element");
  TORCH_CHECK(err.scalar_type() == at::kInt && err.numel() >= 2,
              "err must be the int32 error words");
  TORCH_CHECK(slot.device() == err.device(), "slot and err on one device");
  const c10::DeviceGuard dguard(slot.device());
  sa::err_poison_launch(slot.data_ptr<float>(),
                        reinterpret_cast<unsigned*>(err.data_ptr<int>()),
                        cur_stream());
}

std::vector<at::Tensor> vtrace_loss(at::Tensor behaviour, at::Tensor target,
                                    at::Tensor actions, at::Tensor rewards,
                                    at::Tensor done, at::Tensor values,
                                    at::Tensor bootstrap, double discounting,
                                    int64_t clip_mode, double clip_rho,
                                    double clip_pg_rho, double baseline_cost,
                                    double entropy_cost, bool want_targets) {
  SA_CHECK(behaviour); SA_CHECK(target); SA_CHECK(actions); SA_CHECK(rewards);
  SA_CHECK(done); SA_CHECK(values); SA_CHECK(bootstrap);
  SA_CHECK_F32(behaviour); SA_CHECK_F32(target); SA_CHECK_F32(rewards);
  SA_CHECK_F32(values); SA_CHECK_F32(bootstrap);
  TORCH_CHECK(actions.scalar_type() == at::kLong, "actions must be int64");
  TORCH_CHECK(target.dim() == 3, "logits must be [T,B,A]");
  const int T = target.size(0), B = target.size(1), A = target.size(2);
  TORCH_CHECK(behaviour.sizes() == target.sizes(), "logit shape mismatch");
  TORCH_CHECK(actions.numel() == T * B && rewards.numel() == T * B &&
              done.numel() == T * B && values.numel() == T * B &&
              bootstrap.numel() == B, "[T,B] shape mismatch");
  const c10::DeviceGuard guard(target.device());
  auto f32 = target.options();
  auto loss = at::empty({4}, f32);
  auto dlogits = at::empty_like(target);
  auto dvalues = at::empty({T, B}, f32);
  auto work = at::empty({4 * T * B}, f32);
  at::Tensor vs, pg;
  if (want_targets) {
    vs = at::empty({T, B}, f32);
    pg = at::empty({T, B}, f32);
  }
  sa::vtrace_loss_launch(
      behaviour.data_ptr<float>(), target.data_ptr<float>(),
      actions.data_ptr<int64_t>(), rewards.data_ptr<float>(), u8ptr(done),
      values.data_ptr<float>(), bootstrap.data_ptr<float>(), T, B, A,
      (float)discounting, (int)clip_mode, (float)clip_rho, (float)clip_pg_rho,
      (float)baseline_cost, (float)entropy_cost, loss.data_ptr<float>(),
      dlogits.data_ptr<float>(), dvalues.data_ptr<float>(),
      want_targets ? vs.data_ptr<float>() : nullptr,
      want_targets ? pg.data_ptr<float>() : nullptr, work.data_ptr<float>(),
      cur_stream());
  if (want_targets) return {loss, dlogits, dvalues, vs, pg};
  return {loss, dlogits, dvalues};
}

// Persistent whole-unroll LSTM kernels (lstm_persistent.hip) for H == 256,
// B <= 32 when enabled (SA_LSTM_PERSISTENT=1 or lstm_set_persistent(True)).
// OFF by default: measured on MI355X (tools/micro/lstm_probe.py, T=101,
// B=32) the granule all-gather of h / dG costs 9 / 27.6 us per step against
// 4.4 / 6.9 us for the graph-replayed per-step kernels, whose operand loads
// ride the normal L2/MALL path.
bool g_lstm_persistent = sa::measure_knob("SA_LSTM_PERSISTENT", 0) == 1;

bool use_persistent(int H, int B) { return g_lstm_persistent && H == 256 && B <= 32; }

// Gang kernels (lstm_gang.hip: 8 workgroups, bf16 recurrent product) for
// H == 256, B <= 32: the DEFAULT (SA_LSTM_GANG=0 or lstm_set_gang(False)
// selects the exact-fp32 per-step kernels); they take precedence over the
// fp32 persistent kernels.  Measured at T=101, B=32 (tools/micro/
// lstm_probe.py): fwd 446 vs 446-460 us, bwd 448 vs 724 us per unroll.
bool g_lstm_gang = sa::env_knob("SA_LSTM_GANG", 1) != 0;

// T == 1 (actor inference steps) stays on the per-step kernels: one step
// gains nothing from the gang and the inference graphs keep their layout.
bool use_gang(int H, int B, int T) { return g_lstm_gang && H == 256 && B <= 32 && T >= 2; }

// Recurrence implementation, resolved ONCE per unroll by the caller and
// passed to both lstm_fwd and lstm_bwd (the packed weights differ between
// them): 2 = gang (bf16 recurrent product), 1 = persistent (fp32),
// 0 = per-step kernels (fp32).  exact: the caller needs fp32 (reference
// precision), so the bf16 gang is never chosen.
enum LstmMode { kStep = 0, kPersistent = 1, kGang = 2 };
int64_t lstm_mode(int64_t H, int64_t B, int64_t T, bool exact) {
  if (!exact && use_gang(H, B, T)) return kGang;
  if (use_persistent(H, B)) return kPersistent;
  return kStep;
}

// Sticky per-device timeout word of the persistent kernels (0 = healthy).
at::Tensor lstm_err_word(const at::Device& dev) {
  // called from the learner and from actor-inference threads
  static std::mutex mu;
  std::lock_guard<std::mutex> lock(mu);
  static std::map<int, at::Tensor> words;
  auto it = words.find(dev.index());
  if (it != words.end()) return it->second;
  auto w = at::zeros({4}, at::TensorOptions().dtype(at::kInt).device(dev));
  words[dev.index()] = w;
  return w;
}

at::Tensor lstm_xbuf(bool bwd, const at::TensorOptions& o) {
  // zeroed before EVERY launch (a memset node under graph replay): stale
  // tags of an earlier call can never match
  return at::zeros({(int64_t)sa::lstm_persistent_xbuf_granules(bwd)}, o.dtype(at::kLong));
}

// Returns {hs, cs, acts, hpm, wt}: hpm[t] = keep_t * h_{t-1} (A operand of
// the dW_h GEMM), wt = W_h^T packed for lstm_bwd.  w4 (optional, per-step /
// persistent modes): W_h already packed by lstm_pack_fwd - an inference
// agent packs once per weight publish instead of on every step; wt is then
// empty (no backward).
std::vector<at::Tensor> lstm_fwd(at::Tensor xw, at::Tensor done, at::Tensor c0,
                                 at::Tensor h0, at::Tensor w_h, int64_t mode,
                                 c10::optional<at::Tensor> w4_in) {
  SA_CHECK(xw); SA_CHECK(done); SA_CHECK(c0); SA_CHECK(h0); SA_CHECK(w_h);
  SA_CHECK_F32(xw); SA_CHECK_F32(c0); SA_CHECK_F32(h0); SA_CHECK_F32(w_h);
  const int T = xw.size(0), B = xw.size(1), H4 = xw.size(2), H = H4 / 4;
  TORCH_CHECK(H == 256 || H == 64, "hidden size must be 256 or 64");
  TORCH_CHECK(w_h.size(0) == H && w_h.size(1) == H4, "W_h must be [H,4H]");
  TORCH_CHECK(c0.numel() == B * H && h0.numel() == B * H, "state shape");
  TORCH_CHECK(done.numel() == T * B, "done shape");
  const c10::DeviceGuard guard(xw.device());
  auto hs = at::empty({T, B, H}, xw.options());
  auto cs = at::empty({T, B, H}, xw.options());
  auto acts = at::empty({T, B, H4}, xw.options());
  auto hpm = at::empty({T, B, H}, xw.options());
  const bool packed = w4_in.has_value();
  if (packed) {
    SA_CHECK(*w4_in); SA_CHECK_F32(*w4_in);
    TORCH_CHECK(w4_in->numel() == static_cast<int64_t>(H) * H4 && mode != kGang,
                "w4: the per-step packing of W_h (not for the gang)");
  }
  auto w4 = packed ? *w4_in : at::empty({H * H4}, xw.options());
  auto wt = at::empty({packed ? 0 : H * H4}, xw.options());
  const int64_t RT = (B + 31) / 32;
  auto hpk = at::empty({2, RT * 32 * H}, xw.options());
  auto s = cur_stream();
  const uint8_t* dn = u8ptr(done);
  TORCH_CHECK(mode >= kStep && mode <= kGang, "lstm mode");
  TORCH_CHECK(mode == kStep || (H == 256 && B <= 32 && (mode != kGang || T >= 2)),
              "lstm mode ", mode, " does not cover H=", H, " B=", B, " T=", T);
  if (mode == kGang) {
    // w4 / wt carry the bf16 gang fragments instead (512 KB of their 1 MB)
    sa::lstm_gang_pack_launch(w_h.data_ptr<float>(), w4.data_ptr(), wt.data_ptr(), s);
    auto xbuf = at::zeros({(int64_t)sa::lstm_gang_xbuf_granules(false)},
                          xw.options().dtype(at::kLong));
    sa::lstm_fwd_gang_launch(
        xw.data_ptr<float>(), h0.data_ptr<float>(), c0.data_ptr<float>(), dn,
        w4.data_ptr(), hs.data_ptr<float>(), cs.data_ptr<float>(),
        acts.data_ptr<float>(), hpm.data_ptr<float>(), xbuf.data_ptr(),
        reinterpret_cast<unsigned*>(lstm_err_word(xw.device()).data_ptr<int>()), T, B, s);
    return {hs, cs, acts, hpm, wt};
  }
  if (!packed)
    sa::lstm_pack_weights_launch(w_h.data_ptr<float>(), w4.data_ptr<float>(),
                                 wt.data_ptr<float>(), H, s);
  if (mode == kPersistent) {
    auto xbuf = lstm_xbuf(false, xw.options());
    sa::lstm_fwd_persistent_launch(
        xw.data_ptr<float>(), h0.data_ptr<float>(), c0.data_ptr<float>(), dn,
        w4.data_ptr<float>(), hs.data_ptr<float>(), cs.data_ptr<float>(),
        acts.data_ptr<float>(), hpm.data_ptr<float>(), xbuf.data_ptr(),
        reinterpret_cast<unsigned*>(lstm_err_word(xw.device()).data_ptr<int>()), T, B, s);
    return {hs, cs, acts, hpm, wt};
  }
  for (int t = 0; t < T; ++t) {
    const float* cp = t == 0 ? c0.data_ptr<float>() : cs[t - 1].data_ptr<float>();
    const float* hp = t == 0 ? h0.data_ptr<float>() : hs[t - 1].data_ptr<float>();
    sa::lstm_fwd_step_launch(xw[t].data_ptr<float>(),
                             t == 0 ? nullptr : hpk[t & 1].data_ptr<float>(), hp,
                             cp, dn + t * B, w4.data_ptr<float>(),
                             hs[t].data_ptr<float>(), hpk[(t + 1) & 1].data_ptr<float>(),
                             cs[t].data_ptr<float>(), acts[t].data_ptr<float>(),
                             hpm[t].data_ptr<float>(), B, H, s);
  }
  return {hs, cs, acts, hpm, wt};
}

// W_h [H, 4H] -> w4 (the per-step / persistent kernels' packing, H*4H
// floats) in place; the backward packing goes to a scratch buffer.
void lstm_pack_fwd(at::Tensor w_h, at::Tensor w4) {
  SA_CHECK(w_h); SA_CHECK(w4); SA_CHECK_F32(w_h); SA_CHECK_F32(w4);
  const int H = w_h.size(0);
  TORCH_CHECK((H == 256 || H == 64) && w_h.size(1) == 4 * H && w4.numel() == H * 4 * H,
              "W_h [H,4H] and w4 of H*4H floats");
  const c10::DeviceGuard guard(w_h.device());
  auto scratch = at::empty({H * 4 * H}, w_h.options());
  sa::lstm_pack_weights_launch(w_h.data_ptr<float>(), w4.data_ptr<float>(),
                               scratch.data_ptr<float>(), H, cur_stream());
}

// Returns {dG [T,B,4H] f32, dc0 [B,H], dG bf16 (or an empty tensor)}.
// wt: the packed W_h^T from lstm_fwd.  dc_last (optional) is the gradient
// w.r.t. the final cell state (a later time chunk's dc0); dc0 is the gradient
// w.r.t. the initial cell state (already masked by keep_0).
std::vector<at::Tensor> lstm_bwd(at::Tensor dh_out, at::Tensor done, at::Tensor wt,
                                 at::Tensor acts, at::Tensor cs, at::Tensor c0,
                                 c10::optional<at::Tensor> dc_last, bool want_bf16,
                                 int64_t mode) {
  SA_CHECK(dh_out); SA_CHECK(done); SA_CHECK(wt); SA_CHECK(acts);
  SA_CHECK(cs); SA_CHECK(c0);
  SA_CHECK_F32(dh_out);
  const int T = acts.size(0), B = acts.size(1), H4 = acts.size(2), H = H4 / 4;
  TORCH_CHECK(wt.numel() == H * H4, "packed W_h^T size");
  TORCH_CHECK(dh_out.numel() == T * B * H, "dh shape");
  if (dc_last.has_value()) {
    SA_CHECK(*dc_last); SA_CHECK_F32(*dc_last);
    TORCH_CHECK(dc_last->numel() == c0.numel(), "dc_last shape");
  }
  const c10::DeviceGuard guard(acts.device());
  auto dg = at::empty({T, B, H4}, acts.options());
  at::Tensor dg16;
  if (want_bf16) dg16 = at::empty({T, B, H4}, acts.options().dtype(at::kBFloat16));
  // every step writes its carry / packed dG before the next one reads it
  auto carry = at::empty({2, B, H}, acts.options());
  const int64_t RT = (B + 31) / 32;
  auto dgpk = at::empty({2, RT * 32 * H4}, acts.options());
  auto s = cur_stream();
  const uint8_t* dn = u8ptr(done);
  TORCH_CHECK(mode >= kStep && mode <= kGang, "lstm mode");
  TORCH_CHECK(mode == kStep || (H == 256 && B <= 32), "lstm mode ", mode,
              " does not cover H=", H, " B=", B);
  if (mode == kGang) {
    auto dc0 = at::empty({B, H}, acts.options());
    auto xbuf = at::zeros({(int64_t)sa::lstm_gang_xbuf_granules(true)},
                          acts.options().dtype(at::kLong));
    sa::lstm_bwd_gang_launch(
        dh_out.data_ptr<float>(), dn, wt.data_ptr(), acts.data_ptr<float>(),
        cs.data_ptr<float>(), c0.data_ptr<float>(),
        dc_last.has_value() ? dc_last->data_ptr<float>() : nullptr,
        dg.data_ptr<float>(), want_bf16 ? dg16.data_ptr() : nullptr,
        dc0.data_ptr<float>(), xbuf.data_ptr(),
        reinterpret_cast<unsigned*>(lstm_err_word(acts.device()).data_ptr<int>()), T, B, s);
    if (!want_bf16) dg16 = at::empty({0}, acts.options());
    return {dg, dc0, dg16};
  }
  if (mode == kPersistent) {
    auto dc0 = at::empty({B, H}, acts.options());
    auto xbuf = lstm_xbuf(true, acts.options());
    sa::lstm_bwd_persistent_launch(
        dh_out.data_ptr<float>(), dn, wt.data_ptr<float>(), acts.data_ptr<float>(),
        cs.data_ptr<float>(), c0.data_ptr<float>(),
        dc_last.has_value() ? dc_last->data_ptr<float>() : nullptr,
        dg.data_ptr<float>(), want_bf16 ? dg16.data_ptr() : nullptr,
        dc0.data_ptr<float>(), xbuf.data_ptr(),
        reinterpret_cast<unsigned*>(lstm_err_word(acts.device()).data_ptr<int>()), T, B, s);
    if (!want_bf16) dg16 = at::empty({0}, acts.options());
    return {dg, dc0, dg16};
  }
  for (int t = T - 1; t >= 0; --t) {
    const float* dgn = t == T - 1 ? nullptr : dgpk[(t + 1) & 1].data_ptr<float>();
    const uint8_t* dnext = t == T - 1 ? nullptr : dn + (t + 1) * B;
    const float* cp = t == 0 ? c0.data_ptr<float>() : cs[t - 1].data_ptr<float>();
    const float* cin = t == T - 1
        ? (dc_last.has_value() ? dc_last->data_ptr<float>() : nullptr)
        : carry[(t + 1) & 1].data_ptr<float>();
    sa::lstm_bwd_step_launch(dh_out[t].data_ptr<float>(), dgn, dnext, dn + t * B,
                             wt.data_ptr<float>(), acts[t].data_ptr<float>(),
                             cs[t].data_ptr<float>(), cp, cin,
                             carry[t & 1].data_ptr<float>(), dg[t].data_ptr<float>(),
                             dgpk[t & 1].data_ptr<float>(),
                             want_bf16 ? dg16[t].data_ptr() : nullptr, B, H, s);
  }
  if (!want_bf16) dg16 = at::empty({0}, acts.options());
  return {dg, carry[0], dg16};
}

void lstm_set_persistent(bool on) { g_lstm_persistent = on; }
bool lstm_get_persistent() { return g_lstm_persistent; }
void lstm_set_gang(bool on) { g_lstm_gang = on; }
bool lstm_get_gang() { return g_lstm_gang; }
at::Tensor lstm_error(at::Tensor like) { return lstm_err_word(like.device()); }

void noop(int64_t blocks, int64_t threads, at::Tensor counter) {
  sa::noop_launch(blocks, threads, counter.data_ptr<int>(), cur_stream());
}

}  // namespace

namespace sa {
unsigned* device_error_words() {
  int d = 0;
  (void)hipGetDevice(&d);
  return reinterpret_cast<unsigned*>(
      lstm_err_word(at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(d))).data_ptr<int>());
}
}  // namespace sa

void register_conv_ops(pybind11::module& m);     // conv_bindings.cpp
void register_learner_ops(pybind11::module& m);  // learner_bindings.cpp
void register_conv_f32_ops(pybind11::module& m); // conv_f32_bindings.cpp
void register_board_server(pybind11::module& m); // board_server.cpp

PYBIND11_MODULE(_C, m) {
  m.doc() = "scalable_agent_amd gfx950 HIP kernels";
  m.def("rmsprop", &rmsprop, pybind11::arg("w"), pybind11::arg("g"),
        pybind11::arg("ms"), pybind11::arg("mom"), pybind11::arg("frames"),
        pybind11::arg("lr0"), pybind11::arg("total_frames"),
        pybind11::arg("decay"), pybind11::arg("momentum"), pybind11::arg("eps"),
        pybind11::arg("guard") = pybind11::none(),
        pybind11::arg("lstm_err") = pybind11::none(), pybind11::arg("gscale") = 1.0);
  m.def("err_poison", &err_poison);
  m.def("vtrace_loss", &vtrace_loss);
  m.def("lstm_fwd", &lstm_fwd, pybind11::arg("xw"), pybind11::arg("done"),
        pybind11::arg("c0"), pybind11::arg("h0"), pybind11::arg("w_h"),
        pybind11::arg("mode"), pybind11::arg("w4") = pybind11::none());
  m.def("lstm_pack_fwd", &lstm_pack_fwd, pybind11::arg("w_h"), pybind11::arg("w4"));
  m.def("lstm_bwd", &lstm_bwd, pybind11::arg("dh_out"), pybind11::arg("done"),
        pybind11::arg("wt"), pybind11::arg("acts"), pybind11::arg("cs"),
        pybind11::arg("c0"), pybind11::arg("dc_last") = pybind11::none(),
        pybind11::arg("want_bf16") = false, pybind11::arg("mode"));
  m.def("lstm_set_persistent", &lstm_set_persistent);
  m.def("lstm_get_persistent", &lstm_get_persistent);
  m.def("lstm_set_gang", &lstm_set_gang);
  m.def("lstm_get_gang", &lstm_get_gang);
  m.def("lstm_gang_ws", [](int v) { return sa::lstm_gang_ws(v); });
  m.def("lstm_gang_nap", [](int v) { return sa::lstm_gang_nap(v); });
  m.def("lstm_gang_fault", [](int v) { return sa::lstm_gang_fault(v); });
  m.def("lstm_mode", &lstm_mode);
  m.def("lstm_error_word", &lstm_error);
  m.def("lstm_xpack", &sa::lstm_xpack);
  m.def("noop", &noop);
  register_conv_ops(m);
  register_learner_ops(m);
  register_conv_f32_ops(m);
  register_board_server(m);
}
