"""Fused torso-FC -> core input -> LSTM-256 core (HIP backend learner path):
bf16-operand (_CoreLSTM, below) and exact-fp32 (_CoreLSTMF32) variants.

Reference: experiment.py:185-198 (Linear(256)+ReLU on the flattened conv
features; concat [torso, clip(reward, -1, 1), one_hot(last_action),
instruction]) and :228-235 (LSTMBlockCell(256) unrolled with done-reset).

Forward (one autograd node: 2 GEMM launches + the recurrence):
  h_aug  = [relu(feats W_fc + b_fc),           ONE bf16 MFMA GEMM (gemm_bf16:
            clip(r), one_hot(a), instr|0]      bias + ReLU + the core-input
                                               columns in its epilogue; the
                                               64 language-LSTM columns are
                                               copied in on instruction
                                               levels, else they are zero and
                                               their W_x rows drop out)
  xw     = h_aug W_x[:K] + b_lstm               gemm_bf16, fp32 out
  hs, cs = LSTM recurrence                      lstm.hip / lstm_gang.hip
Backward:
  dG (fp32 + bf16)                              LSTM bwd steps
  dh     = (dG W_x[:256]^T) * (h > 0)           gemm_bf16 (mask epilogue)
  dfeats = dh W_fc^T                            gemm_bf16
  dW_h  += hpm^T dG                             gemm_f32 (exact fp32)
  dW_x[:K] += h_aug^T dG ; db_lstm += colsum dG gemm_bf16 (split-K) + colsum
  dW_fc += feats^T dh ; db_fc += 1^T dh         ONE gemm_bf16 (ones row)
Weight gradients accumulate straight into the learner's flat fp32 gradient
buffer inside grad_sink.direct_grads(), and inside
grad_sink.overlap_weight_grads() the four weight-gradient products run on a
side stream concurrently with the conv-torso backward; the pad rows of W_x[:K] past the
one-hot (the first instruction rows) meet all-zero h_aug columns, so they
receive exactly 0.  Every GEMM is a hand-written MFMA kernel (no vendor
GEMM library on either path); the glue kernels are in
csrc/kernels/learner_io.hip.
"""

import contextlib

import torch

from . import grad_sink
from ._ext import ext

_nullctx = contextlib.nullcontext

CORE = 256


def aug_width(num_actions):
  """Columns of [h, clip(r), one_hot(a)] padded to a multiple of 16."""
  return (CORE + 1 + num_actions + 15) // 16 * 16


class _CoreLSTM(torch.autograd.Function):

  @staticmethod
  def forward(ctx, feats, w_fc, b_fc, kernel, bias, rewards, actions, c0, h0,
              done_u8, num_actions, instr_enc, allow_gang=True, cache=None):
    # the final cell state is rarely used: its gradient arrives as None
    # instead of a zero-filled tensor (the backward handles both)
    ctx.set_materialize_grads(False)
    C = ext()
    T, B = done_u8.shape
    N = T * B
    f_in = CORE + 1 + num_actions + 64
    c_instr = CORE + 1 + num_actions
    assert kernel.shape[0] == f_in + CORE
    bf = torch.bfloat16
    # cache: an inference agent's bf16 weight copies and packed W_h,
    # refreshed once per weight publish instead of on every step
    # (Agent.inference_cache)
    w16 = None if cache is None else cache.get('w16')
    w16_fc = w_fc.to(bf) if w16 is None else w16[0]
    if instr_enc is None:
      # the instruction columns are all zero: their W_x rows drop out
      K = ld = aug_width(num_actions)
    else:
      # the 64 language-LSTM columns join the core input (experiment.py:
      # 191-198); K padded to 16 with zero columns (the matching kernel rows
      # - W_h's first rows - meet zeros: no effect)
      K = ld = (f_in + 15) // 16 * 16
    # h_aug = [relu(feats W_fc + b_fc), clip(r), one_hot(a), 0...] in bf16:
    # ONE hand-written bf16 MFMA GEMM (bias + ReLU + the core-input columns
    # in its epilogue)
    h_aug = torch.empty(N, ld, dtype=bf, device=feats.device)
    C.gemm_bf16(feats, w16_fc, False, False, h_aug, bias=b_fc, relu=True,
                aug_reward=rewards, aug_action=actions)
    if instr_enc is not None:
      h_aug[:, c_instr:f_in].copy_(instr_enc)
    wx16 = kernel[:K].to(bf) if w16 is None else w16[1][:K]
    xw = torch.empty(N, 4 * CORE, dtype=torch.float32, device=feats.device)
    C.gemm_bf16(h_aug, wx16, False, False, xw, bias=bias)
    # bf16 path: the gang may run - unless the caller runs the conv torso
    # concurrently (the time-chunked pipeline): the gang's 8 workgroups must
    # co-reside, which persistent conv grids next to it cannot guarantee
    mode = C.lstm_mode(CORE, B, T, not allow_gang)
    hs, cs, acts, hpm, wt = C.lstm_fwd(xw.view(T, B, 4 * CORE), done_u8, c0, h0,
                                       kernel[f_in:], mode,
                                       _packed_w4(cache, mode))
    ctx.mode = mode
    ctx.save_for_backward(feats, w_fc, b_fc, kernel, bias, w16_fc, wx16, h_aug,
                          wt, acts, cs, c0, hpm, done_u8)
    ctx.f_in = f_in
    ctx.K = K
    ctx.c_instr = c_instr
    ctx.has_instr = instr_enc is not None
    return hs, cs[-1]

  @staticmethod
  def backward(ctx, dhs, dc_last):
    C = ext()
    (feats, w_fc, b_fc, kernel, bias, w16_fc, wx16, h_aug, wt, acts, cs, c0,
     hpm, done_u8) = ctx.saved_tensors
    f_in, K = ctx.f_in, ctx.K
    T, B, G = acts.shape
    N = T * B
    if dhs is None:
      dhs = torch.zeros(T, B, CORE, dtype=acts.dtype, device=acts.device)
    if dc_last is not None:
      dc_last = dc_last.contiguous()
    dg, dc0, dg16 = C.lstm_bwd(dhs.contiguous(), done_u8, wt, acts, cs, c0,
                               dc_last, True, ctx.mode)
    (gwfc, gbfc, gk, gb), direct = grad_sink.sinks([w_fc, b_fc, kernel, bias])
    dg2 = dg.view(N, G)
    dg16_2 = dg16.view(N, G)
    dev = dg.device
    bf = torch.bfloat16
    # critical path: dfeats feeds the conv-torso backward
    dh = torch.empty(N, CORE, dtype=bf, device=dev)
    C.gemm_bf16(dg16_2, wx16[:CORE], False, True, dh,
                mask=h_aug[:, :CORE])                               # (h > 0)
    dfeats = torch.empty_like(feats)
    C.gemm_bf16(dh, w16_fc, False, True, dfeats)
    # weight gradients only: on a side stream next to the torso backward
    # when they accumulate into the learner's sinks (grad_sink overlap)
    side = grad_sink.side_stream(dev) if all(direct) else None
    if side is not None:
      side.wait_stream(torch.cuda.current_stream(dev))
      for t in (hpm, dg, dg16, h_aug, feats, dh):
        t.record_stream(side)
    with torch.cuda.stream(side) if side is not None else _nullctx():
      C.gemm_f32(hpm.view(N, CORE), dg2, True, False, gk[f_in:],
                 accumulate=True)                                   # W_h (fp32)
      C.gemm_bf16(h_aug[:, :K], dg16_2, True, False, gk[:K],
                  accumulate=True)                                  # W_x rows
      C.colsum_f32_(dg2, gb)                                        # b_lstm
      C.gemm_bf16(feats, dh, True, False, gwfc, accumulate=True,
                  colsum=gbfc)                                      # W_fc, b_fc
    dh0 = None
    if ctx.needs_input_grad[8]:
      # (a chunk boundary of the pipelined unroll): exact-fp32 MFMA GEMM
      keep0 = (done_u8[0] == 0).to(torch.float32).unsqueeze(-1)
      dh0 = torch.empty(B, CORE, dtype=torch.float32, device=dg.device)
      C.gemm_f32(dg[0], kernel[f_in:], False, True, dh0)
      dh0.mul_(keep0)
    if not ctx.needs_input_grad[7]:
      dc0 = None
    d_instr = None
    if ctx.has_instr and ctx.needs_input_grad[11]:
      # into the language LSTM: dG W_x[instruction rows]^T
      d_instr = torch.empty(N, 64, dtype=torch.float32, device=dev)
      C.gemm_bf16(dg16_2, wx16[ctx.c_instr:f_in], False, True, d_instr)
    g_wfc, g_bfc, g_k, g_b = grad_sink.returned((gwfc, gbfc, gk, gb), direct)
    return (dfeats, g_wfc, g_bfc, g_k, g_b, None, None, dc0, dh0, None, None,
            d_instr, None, None)


class _CoreLSTMF32(torch.autograd.Function):
  """Reference-precision (fp32) variant: every product is the exact-fp32
  MFMA GEMM of kernels/gemm_f32.hip with its fused epilogue, the recurrence
  the exact fp32 LSTM kernels (never the bf16 gang).

  Forward (3 launches + the recurrence):
    h_aug = [relu(feats W_fc + b_fc), clip(r), one_hot(a), 0...]   ONE GEMM
            (bias + ReLU + the core-input columns in its epilogue)
    xw    = h_aug W_x[:K] + b_lstm                                  GEMM
  Backward:
    dh     = (dG W_x[:256]^T) * (h > 0)                             GEMM + mask
    dfeats = (dh W_fc^T) * (feats > 0)                              GEMM + mask
    dW_h  += hpm^T dG                                               GEMM (split-K)
    dW_x  += h_aug^T dG ; db_lstm += 1^T dG                         ONE GEMM (ones row)
    dW_fc += feats^T dh ; db_fc   += 1^T dh                         ONE GEMM (ones row)
  Weight-gradient reductions are split-K partial slabs summed in a fixed
  order (deterministic).
  """

  @staticmethod
  def forward(ctx, feats, w_fc, b_fc, kernel, bias, rewards, actions, c0, h0,
              done_u8, num_actions, instr_enc, allow_gang=True, cache=None):
    # the final cell state is rarely used: its gradient arrives as None
    # instead of a zero-filled tensor (the backward handles both)
    ctx.set_materialize_grads(False)
    C = ext()
    T, B = done_u8.shape
    N = T * B
    f_in = CORE + 1 + num_actions + 64
    c_instr = CORE + 1 + num_actions
    assert kernel.shape[0] == f_in + CORE
    if instr_enc is None:
      K = ld = aug_width(num_actions)
    else:
      # instruction columns join; K padded to 16 with zero columns (the
      # matching kernel rows - W_h's first rows - meet zeros: no effect)
      K = ld = (f_in + 15) // 16 * 16
    h_aug = torch.empty(N, ld, dtype=torch.float32, device=feats.device)
    C.gemm_f32(feats, w_fc, False, False, h_aug, bias=b_fc, relu=True,
               aug_reward=rewards, aug_action=actions)
    if instr_enc is not None:
      h_aug[:, c_instr:f_in].copy_(instr_enc)
    xw = torch.empty(N, 4 * CORE, dtype=torch.float32, device=feats.device)
    C.gemm_f32(h_aug, kernel[:K], False, False, xw, bias=bias)
    mode = C.lstm_mode(CORE, B, T, True)  # exact: never the bf16 gang
    hs, cs, acts, hpm, wt = C.lstm_fwd(xw.view(T, B, 4 * CORE), done_u8, c0, h0,
                                       kernel[f_in:], mode,
                                       _packed_w4(cache, mode))
    ctx.mode = mode
    ctx.save_for_backward(feats, w_fc, b_fc, kernel, bias, h_aug, wt, acts, cs,
                          c0, hpm, done_u8)
    ctx.f_in, ctx.K, ctx.c_instr = f_in, K, c_instr
    ctx.has_instr = instr_enc is not None
    return hs, cs[-1]

  @staticmethod
  def backward(ctx, dhs, dc_last):
    C = ext()
    (feats, w_fc, b_fc, kernel, bias, h_aug, wt, acts, cs, c0, hpm,
     done_u8) = ctx.saved_tensors
    f_in, K = ctx.f_in, ctx.K
    T, B, G = acts.shape
    N = T * B
    if dhs is None:
      dhs = torch.zeros(T, B, CORE, dtype=acts.dtype, device=acts.device)
    if dc_last is not None:
      dc_last = dc_last.contiguous()
    dg, dc0, _ = C.lstm_bwd(dhs.contiguous(), done_u8, wt, acts, cs, c0,
                            dc_last, False, ctx.mode)
    (gwfc, gbfc, gk, gb), direct = grad_sink.sinks([w_fc, b_fc, kernel, bias])
    dg2 = dg.view(N, G)
    dev = dg.device
    # critical path first: dfeats feeds the conv-torso backward
    dh = torch.empty(N, CORE, dtype=torch.float32, device=dev)
    C.gemm_f32(dg2, kernel[:CORE], False, True, dh, mask=h_aug[:, :CORE])
    dfeats = torch.empty_like(feats)
    # feats is the ReLU'd torso output (core_lstm's contract): its ReLU
    # gradient mask (feats > 0) is applied in this GEMM's epilogue, so the
    # torso backward skips its own relu_mask pass over dfeats
    C.gemm_f32(dh, w_fc, False, True, dfeats, mask=feats)
    dfeats._sa_scratch = True  # the torso backward may mask it in place
    dfeats._sa_relu_masked = True
    C.gemm_f32(hpm.view(N, CORE), dg2, True, False, gk[f_in:],
               accumulate=True)                                     # W_h
    C.gemm_f32(h_aug[:, :K], dg2, True, False, gk[:K], accumulate=True,
               colsum=gb)                                           # W_x, b_lstm
    C.gemm_f32(feats, dh, True, False, gwfc, accumulate=True,
               colsum=gbfc)                                         # W_fc, b_fc
    dh0 = None
    if ctx.needs_input_grad[8]:
      # (a chunk boundary of the pipelined unroll): exact-fp32 MFMA GEMM
      keep0 = (done_u8[0] == 0).to(torch.float32).unsqueeze(-1)
      dh0 = torch.empty(B, CORE, dtype=torch.float32, device=dg.device)
      C.gemm_f32(dg[0], kernel[f_in:], False, True, dh0)
      dh0.mul_(keep0)
    if not ctx.needs_input_grad[7]:
      dc0 = None
    d_instr = None
    if ctx.has_instr and ctx.needs_input_grad[11]:
      d_instr = torch.empty(N, 64, dtype=torch.float32, device=dev)
      C.gemm_f32(dg2, kernel[ctx.c_instr:f_in], False, True, d_instr)
    g_wfc, g_bfc, g_k, g_b = grad_sink.returned((gwfc, gbfc, gk, gb), direct)
    return (dfeats, g_wfc, g_bfc, g_k, g_b, None, None, dc0, dh0, None, None,
            d_instr, None, None)


def _packed_w4(cache, mode):
  """The cached per-step packing of W_h (inference agents), or None."""
  if cache is None or cache.get('w4') is None or mode == 2:  # 2: the gang
    return None
  return cache['w4']


def _as_u8(done):
  """done as a contiguous uint8 tensor: a bool tensor is reinterpreted in
  place (same 1-byte elements), anything else converted."""
  done = done.contiguous()
  if done.dtype == torch.bool:
    return done.view(torch.uint8)
  return done.to(torch.uint8)


def core_lstm(feats, w_fc, b_fc, kernel, bias, rewards, actions, done, state,
              num_actions, instr_enc=None, allow_gang=True, cache=None):
  """feats [T*B, F] (ReLU'd torso output: bf16 -> the bf16-operand path,
  fp32 -> the exact-fp32 path), rewards [T*B] f32, actions [T*B] (last
  actions), done [T,B] bool, state (c, h) [B,256], instr_enc None or the
  language-LSTM output [T*B, 64] (gradients flow back into it), cache None
  or an inference agent's {'w16': bf16 (w_fc, kernel[:K_max]) or None,
  'w4': W_h packed by lstm_pack_fwd} (no gradients)
  -> (hs [T,B,256] f32, (c_T, h_T))."""
  c0, h0 = state
  fn = _CoreLSTMF32 if feats.dtype == torch.float32 else _CoreLSTM
  hs, c_last = fn.apply(
      feats.contiguous(), w_fc, b_fc, kernel, bias,
      rewards.reshape(-1).to(torch.float32).contiguous(),
      actions.reshape(-1).to(torch.int64).contiguous(),
      c0.float().contiguous(), h0.float().contiguous(),
      _as_u8(done), int(num_actions),
      None if instr_enc is None else instr_enc.float().contiguous(),
      bool(allow_gang), cache)
  return hs, (c_last, hs[-1])
