// Torch bindings for the learner glue kernels (csrc/kernels/learner_io.hip).
// Host-side shape/dtype checks; outputs come from the caching allocator and
// everything launches on the current stream (hipGraph-capturable).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "kernels/launchers.h"
#include "kernels/gemm_f32.h"
#include "kernels/gemm_bf16.h"

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define LB_CHECK(t) TORCH_CHECK((t).is_cuda() && (t).is_contiguous(), #t " must be a contiguous GPU tensor")
#define LB_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define LB_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bfloat16")

const uint8_t* mask_ptr(const at::Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBool || t.scalar_type() == at::kByte,
              "done must be bool/uint8");
  return reinterpret_cast<const uint8_t*>(t.data_ptr());
}

// core [T1,B,256]; behaviour [T1,B,A]; actions/rewards/done [T1,B] (full
// batch tensors: the kernel reads rows 1..T).  ticket: persistent int32[1],
// zero between launches.  Multi-task value heads: wb [256, K], bb [K] with
// task [B] (int64 head per batch column; required when K > 1); PopArt:
// mu / nu [K] statistics (both or neither), want_vs returns the V-trace
// targets.  -> {loss[4], dlogits [T,B,A], dvalues [T,B][, vs [T,B]]}
std::vector<at::Tensor> learner_head_fwd(
    at::Tensor core, at::Tensor wp, at::Tensor bp, at::Tensor wb, at::Tensor bb,
    at::Tensor behaviour, at::Tensor actions, at::Tensor rewards, at::Tensor done,
    at::Tensor ticket, double discounting, int64_t clip_mode, double clip_rho,
    double clip_pg_rho, double baseline_cost, double entropy_cost,
    c10::optional<at::Tensor> task, c10::optional<at::Tensor> mu,
    c10::optional<at::Tensor> nu, bool want_vs) {
  LB_CHECK(core); LB_CHECK(wp); LB_CHECK(bp); LB_CHECK(wb); LB_CHECK(bb);
  LB_CHECK(behaviour); LB_CHECK(actions); LB_CHECK(rewards); LB_CHECK(done);
  LB_CHECK(ticket);
  LB_F32(core); LB_F32(wp); LB_F32(bp); LB_F32(wb); LB_F32(bb);
  LB_F32(behaviour); LB_F32(rewards);
  TORCH_CHECK(actions.scalar_type() == at::kLong, "actions must be int64");
  TORCH_CHECK(ticket.scalar_type() == at::kInt && ticket.numel() >= 1, "ticket");
  TORCH_CHECK(core.dim() == 3 && core.size(2) == 256, "core must be [T+1,B,256]");
  const int T1 = core.size(0), B = core.size(1), T = T1 - 1;
  const int A = wp.size(1);
  TORCH_CHECK(T >= 1, "need T >= 1");
  TORCH_CHECK(wp.dim() == 2 && wp.size(0) == 256, "policy w must be [256,A]");
  TORCH_CHECK(A >= 1 && A + 1 <= 32, "1 <= num_actions <= 31");
  TORCH_CHECK(wb.numel() % 256 == 0, "value w must be [256, K]");
  const int K = wb.numel() / 256;
  TORCH_CHECK(bp.numel() == A && bb.numel() == K && K >= 1 && A + K <= 64,
              "value heads: b [K], A + K <= 64");
  TORCH_CHECK(K == 1 || task.has_value(), "K > 1 value heads need the task ids");
  TORCH_CHECK(mu.has_value() == nu.has_value(), "PopArt needs mu and nu");
  TORCH_CHECK(behaviour.numel() == (int64_t)T1 * B * A, "behaviour logits shape");
  TORCH_CHECK(actions.numel() == (int64_t)T1 * B && rewards.numel() == (int64_t)T1 * B &&
              done.numel() == (int64_t)T1 * B, "[T+1,B] shape mismatch");
  TORCH_CHECK(sa::learner_head_fwd_smem(T, A) <= 160 * 1024, "unroll too long");
  sa::HeadTasks tk;
  tk.K = K;
  if (task.has_value()) {
    LB_CHECK(*task);
    TORCH_CHECK(task->scalar_type() == at::kLong && task->numel() == B, "task ids [B] int64");
    tk.task = task->data_ptr<int64_t>();
  }
  if (mu.has_value()) {
    LB_CHECK(*mu); LB_CHECK(*nu); LB_F32(*mu); LB_F32(*nu);
    TORCH_CHECK(mu->numel() == K && nu->numel() == K, "PopArt statistics [K]");
    tk.mu = mu->data_ptr<float>();
    tk.nu = nu->data_ptr<float>();
  }
  const c10::DeviceGuard guard(core.device());
  auto f32 = core.options();
  auto loss = at::empty({4}, f32);
  auto dlogits = at::empty({T, B, A}, f32);
  auto dvalues = at::empty({T, B}, f32);
  auto partial = at::empty({B * 3}, f32);
  at::Tensor vs;
  if (want_vs) {
    vs = at::empty({T, B}, f32);
    tk.vs_out = vs.data_ptr<float>();
  }
  sa::learner_head_fwd_launch(
      core.data_ptr<float>(), wp.data_ptr<float>(), bp.data_ptr<float>(),
      wb.data_ptr<float>(), bb.data_ptr<float>(),
      behaviour.data_ptr<float>() + (int64_t)B * A,
      actions.data_ptr<int64_t>() + B, rewards.data_ptr<float>() + B,
      mask_ptr(done) + B, T, B, A, (float)discounting, (int)clip_mode,
      (float)clip_rho, (float)clip_pg_rho, (float)baseline_cost,
      (float)entropy_cost, dlogits.data_ptr<float>(), dvalues.data_ptr<float>(),
      partial.data_ptr<float>(), reinterpret_cast<unsigned*>(ticket.data_ptr<int>()),
      loss.data_ptr<float>(), tk, stream());
  if (want_vs) return {loss, dlogits, dvalues, vs};
  return {loss, dlogits, dvalues};
}

// -> dcore [T1,B,256]; the heads' gradients are ACCUMULATED into gwp/gbp/gwb/gbb
// (gwb [256, K], gbb [K]; task [B] selects each column's value head)
at::Tensor learner_head_bwd(at::Tensor gscale, at::Tensor core, at::Tensor dlogits,
                            at::Tensor dvalues, at::Tensor wp, at::Tensor wb,
                            at::Tensor gwp, at::Tensor gbp, at::Tensor gwb,
                            at::Tensor gbb, c10::optional<at::Tensor> task) {
  LB_CHECK(gscale); LB_CHECK(core); LB_CHECK(dlogits); LB_CHECK(dvalues);
  LB_CHECK(wp); LB_CHECK(wb); LB_CHECK(gwp); LB_CHECK(gbp); LB_CHECK(gwb);
  LB_CHECK(gbb);
  LB_F32(gscale); LB_F32(core); LB_F32(dlogits); LB_F32(dvalues); LB_F32(gwp);
  LB_F32(gbp); LB_F32(gwb); LB_F32(gbb);
  const int T1 = core.size(0), B = core.size(1), A = wp.size(1);
  const int K = wb.numel() / 256;
  TORCH_CHECK(wb.numel() == 256 * K && K >= 1 && A + K <= 64, "value heads");
  TORCH_CHECK(K == 1 || task.has_value(), "K > 1 value heads need the task ids");
  TORCH_CHECK(dlogits.numel() == (int64_t)(T1 - 1) * B * A, "dlogits shape");
  TORCH_CHECK(gwp.numel() == wp.numel() && gbp.numel() == A &&
              gwb.numel() == 256 * K && gbb.numel() == K, "gradient sink shapes");
  const int64_t* tp = nullptr;
  if (task.has_value()) {
    LB_CHECK(*task);
    TORCH_CHECK(task->scalar_type() == at::kLong && task->numel() == B, "task ids [B] int64");
    tp = task->data_ptr<int64_t>();
  }
  const c10::DeviceGuard guard(core.device());
  auto dcore = at::empty_like(core);
  auto part = at::empty({sa::learner_head_bwd_part_floats(T1 * B, A, K)}, core.options());
  sa::learner_head_bwd_launch(
      gscale.data_ptr<float>(), core.data_ptr<float>(), dlogits.data_ptr<float>(),
      dvalues.data_ptr<float>(), wp.data_ptr<float>(), wb.data_ptr<float>(),
      T1 * B, (T1 - 1) * B, A, B, tp, K, dcore.data_ptr<float>(), gwp.data_ptr<float>(),
      gbp.data_ptr<float>(), gwb.data_ptr<float>(), gbb.data_ptr<float>(),
      part.data_ptr<float>(), stream());
  return dcore;
}

// -> h_aug bf16 [N, ld] = [h (bf16 [N, c0]), clip(r), one_hot(a), 0...]
at::Tensor core_aug_fwd(at::Tensor h, at::Tensor rewards, at::Tensor actions,
                        int64_t ld, int64_t clip_mode) {
  LB_CHECK(h); LB_CHECK(rewards); LB_CHECK(actions);
  LB_BF16(h); LB_F32(rewards);
  TORCH_CHECK(actions.scalar_type() == at::kLong, "actions must be int64");
  const int N = h.size(0), c0 = h.size(1);
  TORCH_CHECK(rewards.numel() == N && actions.numel() == N, "row count");
  TORCH_CHECK(ld > c0, "aug width");
  const c10::DeviceGuard guard(h.device());
  auto h_aug = at::empty({N, ld}, h.options());
  sa::core_aug_fwd_launch(h_aug.data_ptr(), h.data_ptr(), rewards.data_ptr<float>(),
                          actions.data_ptr<int64_t>(), N, (int)ld, c0,
                          (int)clip_mode, stream());
  return h_aug;
}

void colsum_f32_(at::Tensor x, at::Tensor out) {
  LB_CHECK(x); LB_CHECK(out); LB_F32(x); LB_F32(out);
  const int C = x.size(-1);
  const int64_t N = x.numel() / C;
  TORCH_CHECK(out.numel() == C, "out must have one entry per column");
  const c10::DeviceGuard guard(x.device());
  auto part = at::empty({sa::colsum_f32_part_floats((int)N, C)}, x.options());
  sa::colsum_f32_launch(x.data_ptr<float>(), (int)N, C, out.data_ptr<float>(),
                        part.data_ptr<float>(), stream());
}

// dy bf16 [N,C] *= (y > 0); y may be a column slice (row stride >= C)
void relu_bwd_colsum_(at::Tensor dy, at::Tensor y, c10::optional<at::Tensor> out) {
  LB_CHECK(dy); LB_BF16(dy); LB_BF16(y);
  TORCH_CHECK(y.is_cuda() && y.dim() == 2 && y.stride(1) == 1, "y must be row-major 2-D");
  const int N = dy.size(0), C = dy.size(1);
  TORCH_CHECK(y.size(0) == N && y.size(1) == C, "shape mismatch");
  TORCH_CHECK(C % 2 == 0 && C <= 512 && 256 % (C / 2) == 0 && (C / 2) * 32 >= 256,
              "relu_bwd_colsum_: C/2 must divide 256 and C >= 16");
  float* op = nullptr;
  if (out.has_value()) {
    LB_CHECK(*out); LB_F32(*out);
    TORCH_CHECK(out->numel() == C, "out size");
    op = out->data_ptr<float>();
  }
  const c10::DeviceGuard guard(dy.device());
  at::Tensor part;
  if (op)
    part = at::empty({sa::relu_bwd_colsum_part_floats(N, C)},
                     dy.options().dtype(at::kFloat));
  sa::relu_bwd_colsum_launch(dy.data_ptr(), y.data_ptr(), N, C, (int)y.stride(0),
                             op, op ? part.data_ptr<float>() : nullptr, stream());
}

void relu_mask_bf16_(at::Tensor dx, at::Tensor x) {
  LB_CHECK(dx); LB_CHECK(x); LB_BF16(dx); LB_BF16(x);
  TORCH_CHECK(dx.numel() == x.numel() && dx.numel() % 8 == 0, "size");
  const c10::DeviceGuard guard(dx.device());
  sa::relu_mask_bf16_launch(dx.data_ptr(), x.data_ptr(), dx.numel(), stream());
}

// Actor inference head + sampler: h [B,256] f32 -> {logits [B,A], baseline
// [B], action [B] int64}.  (seed, offset) select the Philox stream; the
// caller advances offset once per call.
std::vector<at::Tensor> actor_head_sample(at::Tensor h, at::Tensor wp, at::Tensor bp,
                                          at::Tensor wb, at::Tensor bb, int64_t seed,
                                          int64_t offset,
                                          c10::optional<at::Tensor> offset_dev) {
  LB_CHECK(h); LB_CHECK(wp); LB_CHECK(bp); LB_CHECK(wb); LB_CHECK(bb);
  LB_F32(h); LB_F32(wp); LB_F32(bp); LB_F32(wb); LB_F32(bb);
  TORCH_CHECK(h.dim() == 2 && h.size(1) == 256, "h must be [B,256]");
  TORCH_CHECK(wp.dim() == 2 && wp.size(0) == 256, "policy w must be [256,A]");
  const int B = h.size(0), A = wp.size(1);
  TORCH_CHECK(A >= 1 && A <= sa::actor_head_max_actions(), "1 <= num_actions <= 32");
  TORCH_CHECK(bp.numel() == A && wb.numel() == 256 && bb.numel() == 1,
              "one value head");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(h.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(wb.data_ptr()) % 16 == 0,
              "h / baseline w must be 16-byte aligned");
  // offset_dev: one int64 (the caller advances it), or the pair {offset,
  // waves done} the kernel advances itself (zero-initialised, then owned by
  // the kernel)
  unsigned long long* op = nullptr;
  int advance = 0;
  if (offset_dev.has_value()) {
    LB_CHECK(*offset_dev);
    TORCH_CHECK(offset_dev->scalar_type() == at::kLong &&
                    (offset_dev->numel() == 1 || offset_dev->numel() == 2) &&
                    offset_dev->is_contiguous(),
                "offset_dev must be one int64 or a contiguous pair");
    op = reinterpret_cast<unsigned long long*>(offset_dev->data_ptr());
    advance = offset_dev->numel() == 2;
  }
  const c10::DeviceGuard guard(h.device());
  auto logits = at::empty({B, A}, h.options());
  auto baseline = at::empty({B}, h.options());
  auto action = at::empty({B}, h.options().dtype(at::kLong));
  sa::actor_head_sample_launch(h.data_ptr<float>(), wp.data_ptr<float>(),
                               bp.data_ptr<float>(), wb.data_ptr<float>(),
                               bb.data_ptr<float>(), logits.data_ptr<float>(),
                               baseline.data_ptr<float>(),
                               action.data_ptr<int64_t>(), B, A,
                               static_cast<unsigned long long>(seed),
                               static_cast<unsigned long long>(offset), op, advance,
                               stream());
  return {logits, baseline, action};
}

// Inference-board epilogue: c / h [R, H] f32 updated in place where mask [R]
// (or [R, 1]) > 0 from c2 / h2, and every tensor of `fields` ([R, ...], any
// dtype, 4-byte multiple per row) packed into `out` (uint8, S slot blocks of
// slot_bytes) at byte offset offs[f] + (r % M) * row_bytes(f) of slot r / M.
// out_addr != 0: pack into that device-accessible address instead of `out`
// (the board's registered host output region, out.numel() bytes long; only
// the rows whose mask is set are written, then fenced at system scope).
void board_epilogue(std::vector<at::Tensor> fields, std::vector<int64_t> offs, at::Tensor out,
                    int64_t M, int64_t slot_bytes, at::Tensor mask, at::Tensor c2,
                    at::Tensor h2, at::Tensor c, at::Tensor h, int64_t out_addr) {
  const int nf = static_cast<int>(fields.size());
  TORCH_CHECK(nf >= 1 && nf <= sa::board_epilogue_max_fields() &&
              static_cast<int>(offs.size()) == nf, "board_epilogue: 1..6 fields with offsets");
  LB_CHECK(out); LB_CHECK(mask); LB_CHECK(c2); LB_CHECK(h2); LB_CHECK(c); LB_CHECK(h);
  LB_F32(mask); LB_F32(c2); LB_F32(h2); LB_F32(c); LB_F32(h);
  TORCH_CHECK(out.scalar_type() == at::kByte, "out must be uint8");
  TORCH_CHECK(c.dim() == 2 && c.sizes() == h.sizes() && c.sizes() == c2.sizes() &&
              c.sizes() == h2.sizes(), "c / h / c2 / h2 must be [R, H]");
  const int64_t R = c.size(0), H = c.size(1);
  TORCH_CHECK(mask.numel() == R, "mask must have R elements");
  TORCH_CHECK(M >= 1 && R % M == 0 && slot_bytes % 4 == 0 &&
              out.numel() >= (R / M) * slot_bytes, "board geometry");
  void* dst = out_addr ? reinterpret_cast<void*>(out_addr) : out.data_ptr();
  TORCH_CHECK(reinterpret_cast<uintptr_t>(dst) % 4 == 0, "out 4-byte aligned");
  const void* src[8];
  int per[8], off[8];
  for (int f = 0; f < nf; ++f) {
    LB_CHECK(fields[f]);
    TORCH_CHECK(fields[f].dim() >= 1 && fields[f].size(0) == R, "field rows != R");
    const int64_t rb = fields[f].numel() / R * fields[f].element_size();
    TORCH_CHECK(rb % 4 == 0 && offs[f] % 4 == 0 && offs[f] + M * rb <= slot_bytes &&
                reinterpret_cast<uintptr_t>(fields[f].data_ptr()) % 4 == 0,
                "field rows / offsets must be 4-byte multiples inside the slot block");
    src[f] = fields[f].data_ptr();
    per[f] = static_cast<int>(rb / 4);
    off[f] = static_cast<int>(offs[f] / 4);
  }
  const c10::DeviceGuard guard(c.device());
  sa::board_epilogue_launch(src, per, off, nf, static_cast<int>(R), static_cast<int>(M),
                            static_cast<int>(slot_bytes / 4), static_cast<int>(H),
                            mask.data_ptr<float>(), c2.data_ptr<float>(), h2.data_ptr<float>(),
                            c.data_ptr<float>(), h.data_ptr<float>(), dst, out_addr != 0,
                            stream());
}

// C[:, :N] (+)= op(A) op(B) with the fused epilogue of kernels/gemm_f32.h.
// A / B / C / mask may be row slices of wider row-major matrices (row stride
// = stride(0), unit column stride).  op(A) = A^T when ta (A is [K, M]),
// op(B) = B^T when tb (B is [N, K]).  colsum: ones-row column sums of op(B)
// accumulated into it; aug_*: the core-input columns [clip(r), one_hot(a),
// 0...] written at C[:, aug_c0:] (aug_c0 = N).
void gemm_f32(at::Tensor A, at::Tensor B, bool ta, bool tb, at::Tensor C,
              c10::optional<at::Tensor> bias, c10::optional<at::Tensor> mask, bool relu,
              bool accumulate, c10::optional<at::Tensor> colsum,
              c10::optional<at::Tensor> aug_reward, c10::optional<at::Tensor> aug_action) {
  auto rm = [](const at::Tensor& t, const char* n) {
    TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.stride(1) == 1 && t.scalar_type() == at::kFloat,
                n, " must be a row-major float32 GPU matrix");
    TORCH_CHECK(t.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, n,
                " rows must be 16-byte aligned");
  };
  rm(A, "A"); rm(B, "B"); rm(C, "C");
  const int64_t M = ta ? A.size(1) : A.size(0), K = ta ? A.size(0) : A.size(1);
  const int64_t Kb = tb ? B.size(1) : B.size(0), N = tb ? B.size(0) : B.size(1);
  TORCH_CHECK(K == Kb, "gemm_f32: inner dimensions ", K, " vs ", Kb);
  TORCH_CHECK(C.size(0) == M && C.size(1) >= N, "gemm_f32: C must be [M, >= N]");
  TORCH_CHECK(K % 4 == 0 || (ta && !tb),
              "gemm_f32: K must be a multiple of 4 unless op(A) = A^T and op(B) = B");
  sa::GemmEpilogue ep{};
  ep.C = C.data_ptr<float>();
  ep.ldc = C.stride(0);
  if (bias.has_value() && bias->defined()) {
    LB_CHECK(*bias); LB_F32(*bias);
    TORCH_CHECK(bias->numel() == N, "bias size");
    ep.bias = bias->data_ptr<float>();
  }
  if (mask.has_value() && mask->defined()) {
    rm(*mask, "mask");
    TORCH_CHECK(mask->size(0) == M && mask->size(1) >= N, "mask shape");
    ep.mask = mask->data_ptr<float>();
    ep.ldm = mask->stride(0);
  }
  ep.relu = relu;
  ep.accumulate = accumulate;
  const bool ones = colsum.has_value() && colsum->defined();
  if (ones) {
    LB_CHECK(*colsum); LB_F32(*colsum);
    TORCH_CHECK(colsum->numel() == N, "colsum size");
    ep.colsum = colsum->data_ptr<float>();
  }
  if (aug_reward.has_value() && aug_reward->defined()) {
    TORCH_CHECK(aug_action.has_value() && aug_action->defined(), "aug needs actions");
    LB_CHECK(*aug_reward); LB_F32(*aug_reward); LB_CHECK(*aug_action);
    TORCH_CHECK(aug_action->scalar_type() == at::kLong, "actions must be int64");
    TORCH_CHECK(aug_reward->numel() == M && aug_action->numel() == M, "aug rows");
    TORCH_CHECK(C.size(1) > N && C.size(1) == C.stride(0), "aug: C must be [M, ld > N]");
    ep.aug_reward = aug_reward->data_ptr<float>();
    ep.aug_action = aug_action->data_ptr<int64_t>();
    ep.aug_c0 = N;
  }
  const c10::DeviceGuard guard(A.device());
  const int splits = sa::gemm_f32_splits(M, N, K, ones);
  at::Tensor part;
  if (splits > 1)
    part = at::empty({sa::gemm_f32_part_floats(M, N, K, ones, splits)}, A.options());
  TORCH_CHECK(sa::gemm_f32_launch(A.data_ptr<float>(), B.data_ptr<float>(), M, N, K,
                                  A.stride(0), B.stride(0), ta, tb, ones, splits,
                                  splits > 1 ? part.data_ptr<float>() : nullptr, ep, stream()),
              "gemm_f32: launch refused");
}


// C[:, :N] (+)= op(A) op(B) over bf16 A / B (fp32 accumulate), the fused
// epilogue of kernels/gemm_bf16.h: C fp32 or bf16, mask bf16.  Same
// conventions as gemm_f32 (row slices of wider matrices; op(A) = A^T when
// ta, A is [K, M]; op(B) = B^T when tb, B is [N, K]).
void gemm_bf16(at::Tensor A, at::Tensor B, bool ta, bool tb, at::Tensor C,
               c10::optional<at::Tensor> bias, c10::optional<at::Tensor> mask, bool relu,
               bool accumulate, c10::optional<at::Tensor> colsum,
               c10::optional<at::Tensor> aug_reward, c10::optional<at::Tensor> aug_action) {
  auto rm = [](const at::Tensor& t, const char* n, bool want_bf16) {
    TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.stride(1) == 1, n,
                " must be a row-major GPU matrix");
    TORCH_CHECK(!want_bf16 || t.scalar_type() == at::kBFloat16, n, " must be bf16");
    TORCH_CHECK(t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, n,
                " rows must be 16-byte aligned");
  };
  rm(A, "A", true); rm(B, "B", true);
  TORCH_CHECK(C.is_cuda() && C.dim() == 2 && C.stride(1) == 1 &&
              (C.scalar_type() == at::kFloat || C.scalar_type() == at::kBFloat16),
              "C must be a row-major fp32 / bf16 GPU matrix");
  const int64_t M = ta ? A.size(1) : A.size(0), K = ta ? A.size(0) : A.size(1);
  const int64_t Kb = tb ? B.size(1) : B.size(0), N = tb ? B.size(0) : B.size(1);
  TORCH_CHECK(K == Kb, "gemm_bf16: inner dimensions ", K, " vs ", Kb);
  TORCH_CHECK(C.size(0) == M && C.size(1) >= N, "gemm_bf16: C must be [M, >= N]");
  TORCH_CHECK(K % 8 == 0 || (ta && !tb),
              "gemm_bf16: K must be a multiple of 8 unless op(A) = A^T and op(B) = B");
  sa::GemmBf16Epilogue ep{};
  ep.C = C.data_ptr();
  ep.ldc = C.stride(0);
  ep.c_bf16 = C.scalar_type() == at::kBFloat16;
  TORCH_CHECK(!(accumulate && ep.c_bf16), "gemm_bf16: accumulate needs an fp32 C");
  if (bias.has_value() && bias->defined()) {
    LB_CHECK(*bias); LB_F32(*bias);
    TORCH_CHECK(bias->numel() == N, "bias size");
    ep.bias = bias->data_ptr<float>();
  }
  if (mask.has_value() && mask->defined()) {
    rm(*mask, "mask", true);
    TORCH_CHECK(mask->size(0) == M && mask->size(1) >= N, "mask shape");
    ep.mask = reinterpret_cast<const uint16_t*>(mask->data_ptr());
    ep.ldm = mask->stride(0);
  }
  ep.relu = relu;
  ep.accumulate = accumulate;
  const bool ones = colsum.has_value() && colsum->defined();
  if (ones) {
    LB_CHECK(*colsum); LB_F32(*colsum);
    TORCH_CHECK(colsum->numel() == N, "colsum size");
    ep.colsum = colsum->data_ptr<float>();
  }
  if (aug_reward.has_value() && aug_reward->defined()) {
    TORCH_CHECK(aug_action.has_value() && aug_action->defined(), "aug needs actions");
    LB_CHECK(*aug_reward); LB_F32(*aug_reward); LB_CHECK(*aug_action);
    TORCH_CHECK(aug_action->scalar_type() == at::kLong, "actions must be int64");
    TORCH_CHECK(aug_reward->numel() == M && aug_action->numel() == M, "aug rows");
    TORCH_CHECK(C.size(1) > N && C.size(1) == C.stride(0), "aug: C must be [M, ld > N]");
    ep.aug_reward = aug_reward->data_ptr<float>();
    ep.aug_action = aug_action->data_ptr<int64_t>();
    ep.aug_c0 = N;
  }
  const c10::DeviceGuard guard(A.device());
  const int splits = sa::gemm_bf16_splits(M, N, K, ones);
  at::Tensor part;
  if (splits > 1)
    part = at::empty({sa::gemm_bf16_part_floats(M, N, K, ones, splits)},
                     A.options().dtype(at::kFloat));
  TORCH_CHECK(sa::gemm_bf16_launch(reinterpret_cast<const uint16_t*>(A.data_ptr()),
                                   reinterpret_cast<const uint16_t*>(B.data_ptr()), M, N, K,
                                   A.stride(0), B.stride(0), ta, tb, ones, splits,
                                   splits > 1 ? part.data_ptr<float>() : nullptr, ep,
                                   stream()),
              "gemm_bf16: launch refused");
}

// Instruction encoder: ids [N, L] int64, lengths [N] int64, embed [V, 20],
// kernel [84, 256], bias [256] -> {out [N, 64], acts, cs, xh} (saved for the
// backward).
std::vector<at::Tensor> lang_lstm_fwd(at::Tensor ids, at::Tensor lengths, at::Tensor embed,
                                      at::Tensor kernel, at::Tensor bias) {
  LB_CHECK(ids); LB_CHECK(lengths); LB_CHECK(embed); LB_CHECK(kernel); LB_CHECK(bias);
  LB_F32(embed); LB_F32(kernel); LB_F32(bias);
  TORCH_CHECK(ids.scalar_type() == at::kLong && lengths.scalar_type() == at::kLong,
              "ids / lengths must be int64");
  TORCH_CHECK(ids.dim() == 2 && lengths.numel() == ids.size(0), "ids [N, L], lengths [N]");
  TORCH_CHECK(embed.dim() == 2 && embed.size(1) == 20, "embedding width 20");
  TORCH_CHECK(kernel.size(0) == 84 && kernel.size(1) == 256 && bias.numel() == 256,
              "language LSTM kernel [84, 256]");
  const int N = ids.size(0), L = ids.size(1);
  const c10::DeviceGuard guard(ids.device());
  auto o = embed.options();
  auto out = at::empty({N, 64}, o);
  auto acts = at::empty({L, N, 256}, o);
  auto cs = at::empty({L, N, 64}, o);
  auto xh = at::empty({L, N, 84}, o);
  if (N > 0 && L > 0)
    sa::lang_lstm_fwd_launch(ids.data_ptr<int64_t>(), lengths.data_ptr<int64_t>(),
                             embed.data_ptr<float>(), kernel.data_ptr<float>(),
                             bias.data_ptr<float>(), N, L, embed.size(0), out.data_ptr<float>(),
                             acts.data_ptr<float>(), cs.data_ptr<float>(),
                             xh.data_ptr<float>(), stream());
  else
    out.zero_();
  return {out, acts, cs, xh};
}

// -> {dgates [L, N, 256], dx [L, N, 20]}; with ids [N, L] and egrad [V, 20]
// the valid words' dx rows are added into egrad instead (dx comes back empty)
std::vector<at::Tensor> lang_lstm_bwd(at::Tensor lengths, at::Tensor kernel, at::Tensor dout,
                                      at::Tensor acts, at::Tensor cs,
                                      c10::optional<at::Tensor> ids,
                                      c10::optional<at::Tensor> egrad) {
  LB_CHECK(lengths); LB_CHECK(kernel); LB_CHECK(dout); LB_CHECK(acts); LB_CHECK(cs);
  LB_F32(dout); LB_F32(acts); LB_F32(cs); LB_F32(kernel);
  const int L = acts.size(0), N = acts.size(1);
  TORCH_CHECK(dout.numel() == static_cast<int64_t>(N) * 64, "dout [N, 64]");
  TORCH_CHECK(lengths.scalar_type() == at::kLong && lengths.numel() == N, "lengths [N] int64");
  const bool fused = egrad.has_value() && egrad->defined();
  int V = 0;
  if (fused) {
    TORCH_CHECK(ids.has_value() && ids->defined(), "egrad needs ids");
    LB_CHECK(*ids); LB_CHECK(*egrad); LB_F32(*egrad);
    TORCH_CHECK(ids->scalar_type() == at::kLong && ids->dim() == 2 && ids->size(0) == N &&
                    ids->size(1) == L, "ids [N, L] int64");
    TORCH_CHECK(egrad->dim() == 2 && egrad->size(1) == 20 && egrad->size(0) > 0,
                "egrad [V, 20]");
    V = egrad->size(0);
  }
  const c10::DeviceGuard guard(acts.device());
  auto dg = at::empty({L, N, 256}, acts.options());
  auto dx = fused ? at::empty({0}, acts.options()) : at::empty({L, N, 20}, acts.options());
  if (N > 0 && L > 0)
    sa::lang_lstm_bwd_launch(lengths.data_ptr<int64_t>(), kernel.data_ptr<float>(),
                             dout.data_ptr<float>(), acts.data_ptr<float>(),
                             cs.data_ptr<float>(), N, L, dg.data_ptr<float>(),
                             fused ? nullptr : dx.data_ptr<float>(),
                             fused ? ids->data_ptr<int64_t>() : nullptr, V,
                             fused ? egrad->data_ptr<float>() : nullptr, stream());
  return {dg, dx};
}

}  // namespace

void register_learner_ops(pybind11::module& m) {
  m.def("learner_head_fwd", &learner_head_fwd, pybind11::arg("core"), pybind11::arg("wp"),
        pybind11::arg("bp"), pybind11::arg("wb"), pybind11::arg("bb"),
        pybind11::arg("behaviour"), pybind11::arg("actions"), pybind11::arg("rewards"),
        pybind11::arg("done"), pybind11::arg("ticket"), pybind11::arg("discounting"),
        pybind11::arg("clip_mode"), pybind11::arg("clip_rho"), pybind11::arg("clip_pg_rho"),
        pybind11::arg("baseline_cost"), pybind11::arg("entropy_cost"),
        pybind11::arg("task") = pybind11::none(), pybind11::arg("mu") = pybind11::none(),
        pybind11::arg("nu") = pybind11::none(), pybind11::arg("want_vs") = false);
  m.def("learner_head_bwd", &learner_head_bwd, pybind11::arg("gscale"), pybind11::arg("core"),
        pybind11::arg("dlogits"), pybind11::arg("dvalues"), pybind11::arg("wp"),
        pybind11::arg("wb"), pybind11::arg("gwp"), pybind11::arg("gbp"), pybind11::arg("gwb"),
        pybind11::arg("gbb"), pybind11::arg("task") = pybind11::none());
  m.def("core_aug_fwd", &core_aug_fwd);
  m.def("lang_lstm_fwd", &lang_lstm_fwd);
  m.def("lang_lstm_bwd", &lang_lstm_bwd, pybind11::arg("lengths"), pybind11::arg("kernel"),
        pybind11::arg("dout"), pybind11::arg("acts"), pybind11::arg("cs"),
        pybind11::arg("ids") = pybind11::none(), pybind11::arg("egrad") = pybind11::none());
  m.def("gemm_f32", &gemm_f32, pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("ta"),
        pybind11::arg("tb"), pybind11::arg("C"), pybind11::arg("bias") = pybind11::none(),
        pybind11::arg("mask") = pybind11::none(), pybind11::arg("relu") = false,
        pybind11::arg("accumulate") = false, pybind11::arg("colsum") = pybind11::none(),
        pybind11::arg("aug_reward") = pybind11::none(),
        pybind11::arg("aug_action") = pybind11::none());
  m.def("gemm_bf16", &gemm_bf16, pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("ta"),
        pybind11::arg("tb"), pybind11::arg("C"), pybind11::arg("bias") = pybind11::none(),
        pybind11::arg("mask") = pybind11::none(), pybind11::arg("relu") = false,
        pybind11::arg("accumulate") = false, pybind11::arg("colsum") = pybind11::none(),
        pybind11::arg("aug_reward") = pybind11::none(),
        pybind11::arg("aug_action") = pybind11::none());
  m.def("colsum_f32_", &colsum_f32_);
  m.def("relu_bwd_colsum_", &relu_bwd_colsum_, pybind11::arg("dy"),
        pybind11::arg("y"), pybind11::arg("out") = pybind11::none());
  m.def("relu_mask_bf16_", &relu_mask_bf16_);
  m.def("board_epilogue", &board_epilogue, pybind11::arg("fields"), pybind11::arg("offs"),
        pybind11::arg("out"), pybind11::arg("M"), pybind11::arg("slot_bytes"),
        pybind11::arg("mask"), pybind11::arg("c2"), pybind11::arg("h2"), pybind11::arg("c"),
        pybind11::arg("h"), pybind11::arg("out_addr") = 0);
  m.def("actor_head_sample", &actor_head_sample, pybind11::arg("h"),
        pybind11::arg("wp"), pybind11::arg("bp"), pybind11::arg("wb"),
        pybind11::arg("bb"), pybind11::arg("seed"), pybind11::arg("offset"),
        pybind11::arg("offset_dev") = pybind11::none());
}
