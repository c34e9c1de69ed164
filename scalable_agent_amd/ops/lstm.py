"""LSTM core unroll on the fused per-step HIP kernels (csrc/kernels/lstm.hip).

x W_x + b for all T steps is ONE GEMM (hipBLASLt via torch.matmul, autograd
handles dX/dW_x/db); the serial recurrence runs as T fused step kernels
(recurrent GEMV + gates + cell + done-reset) forward and T fused reverse step
kernels backward; dW_h = sum_t (keep_t h_{t-1})^T dG_t is one GEMM.

The recurrence is differentiable w.r.t. its initial state too (dc0 from the
backward kernels' carry, dh0 = keep_0 * dG_0 W_h^T), so an unroll can be split
into time chunks that chain their states - the pipelined learner unroll
(models/agent.py) runs chunk k's recurrence on a side stream while the conv
torso of chunk k+1 runs on the main stream.
"""

import torch

from ._ext import ext, check_cuda


class _LSTMRecurrence(torch.autograd.Function):

  @staticmethod
  def forward(ctx, xw, w_h, c0, h0, done_u8, exact):
    xw = xw.contiguous()
    w_h_c = w_h.contiguous()
    c0 = c0.contiguous()
    h0 = h0.contiguous()
    T, B, H4 = xw.shape
    # resolved once: forward and backward must agree on the packed weights
    mode = ext().lstm_mode(H4 // 4, B, T, bool(exact))
    hs, cs, acts, hpm, wt = ext().lstm_fwd(xw, done_u8, c0, h0, w_h_c, mode)
    ctx.save_for_backward(w_h_c, wt, acts, cs, c0, hpm, done_u8)
    ctx.mode = mode
    return hs, cs[-1]

  @staticmethod
  def backward(ctx, dhs, dc_last):
    w_h, wt, acts, cs, c0, hpm, done_u8 = ctx.saved_tensors
    T, B, H4 = acts.shape
    H = H4 // 4
    if dhs is None:
      dhs = torch.zeros(T, B, H, dtype=acts.dtype, device=acts.device)
    if dc_last is not None:
      dc_last = dc_last.contiguous()
    dg, dc0, _ = ext().lstm_bwd(dhs.contiguous(), done_u8, wt, acts, cs, c0,
                                dc_last, False, ctx.mode)
    # dW_h = sum_t (keep_t h_{t-1})^T dG_t; hpm is saved by the fwd kernel
    dw_h = hpm.reshape(T * B, H).t() @ dg.reshape(T * B, 4 * H)
    dh0 = None
    if ctx.needs_input_grad[3]:
      keep0 = (done_u8[0] == 0).to(dg.dtype).unsqueeze(-1)
      dh0 = (dg[0] @ w_h.t()) * keep0
    if not ctx.needs_input_grad[2]:
      dc0 = None
    return dg, dw_h, dc0, dh0, None, None


def lstm_unroll(x, done, state, kernel, bias, w_x=None, w_h=None, exact=False):
  """x [T,B,F] f32, done [T,B] bool, state (c,h) -> (h_all, (c_T, h_T)).

  w_x / w_h: optional pre-sliced views of `kernel` (rows [:F] and [F:]); a
  chunked unroll passes the same views to every chunk so the slice backward
  runs once instead of once per chunk.  exact: reference (fp32) precision -
  the bf16-operand gang recurrence is never used.
  """
  c0, h0 = state
  check_cuda(x, kernel)
  F_in = x.shape[-1]
  if w_x is None:
    w_x = kernel[:F_in]
  if w_h is None:
    w_h = kernel[F_in:]
  xw = torch.matmul(x.float(), w_x) + bias
  hs, c_last = _LSTMRecurrence.apply(xw, w_h, c0.float(), h0.float(),
                                     done.to(torch.uint8).contiguous(),
                                     bool(exact))
  return hs, (c_last, hs[-1])


def set_persistent(on):
  """Selects the whole-unroll persistent kernels (B <= 32, H == 256; the
  default) or the per-step kernels; returns the previous setting."""
  prev = bool(ext().lstm_get_persistent())
  ext().lstm_set_persistent(bool(on))
  return prev


def set_gang(on):
  """Selects the 8-workgroup bf16-MFMA whole-unroll kernels (lstm_gang.hip;
  B <= 32, H == 256); they take precedence over set_persistent.  Returns the
  previous setting."""
  prev = bool(ext().lstm_get_gang())
  ext().lstm_set_gang(bool(on))
  return prev


def persistent_error_word(device):
  """The device-resident sticky timeout word itself (int32[4], element 0)."""
  return ext().lstm_error_word(torch.empty(0, device=device))


def set_gang_fault(on):
  """Test hook: every gang sweep reports a timeout.  Returns the previous
  setting."""
  return bool(ext().lstm_gang_fault(1 if on else 0))


def persistent_error(device):
  """Sticky timeout word of the persistent kernels on `device` (0 = healthy;
  nonzero means a workgroup could not co-reside and the unroll was
  abandoned).  Reading it synchronises the device."""
  like = torch.empty(0, device=device)
  return int(ext().lstm_error_word(like)[0].item())
