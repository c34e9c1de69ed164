"""LSTM core unroll on the fused per-step HIP kernels (csrc/kernels/lstm.hip).

x W_x + b for all T steps is ONE GEMM (hipBLASLt via torch.matmul, autograd
handles dX/dW_x/db); the serial recurrence runs as T fused step kernels
(recurrent GEMV + gates + cell + done-reset) forward and T fused reverse step
kernels backward; dW_h = sum_t (keep_t h_{t-1})^T dG_t is one GEMM.
"""

import torch

from ._ext import ext, check_cuda


class _LSTMRecurrence(torch.autograd.Function):

  @staticmethod
  def forward(ctx, xw, w_h, c0, h0, done_u8):
    xw = xw.contiguous()
    w_h_c = w_h.contiguous()
    hs, cs, acts = ext().lstm_fwd(xw, done_u8, c0.contiguous(),
                                  h0.contiguous(), w_h_c)
    ctx.save_for_backward(w_h_c, acts, cs, c0, h0, hs, done_u8)
    return hs, cs[-1]

  @staticmethod
  def backward(ctx, dhs, dc_last):
    w_h, acts, cs, c0, h0, hs, done_u8 = ctx.saved_tensors
    if dhs is None:
      dhs = torch.zeros_like(hs)
    dg = ext().lstm_bwd(dhs.contiguous(), done_u8, w_h, acts, cs,
                        c0.contiguous())
    T, B, H = hs.shape
    keep = (done_u8 == 0).to(hs.dtype).unsqueeze(-1)
    h_prev = torch.cat([h0.unsqueeze(0), hs[:-1]], 0) * keep
    dw_h = h_prev.reshape(T * B, H).t() @ dg.reshape(T * B, 4 * H)
    return dg, dw_h, None, None, None


def lstm_unroll(x, done, state, kernel, bias):
  """x [T,B,F] f32, done [T,B] bool, state (c,h) -> (h_all, (c_T, h_T))."""
  c0, h0 = state
  check_cuda(x, kernel)
  F_in = x.shape[-1]
  xw = torch.matmul(x.float(), kernel[:F_in]) + bias
  hs, c_last = _LSTMRecurrence.apply(xw, kernel[F_in:], c0.float(), h0.float(),
                                     done.to(torch.uint8).contiguous())
  return hs, (c_last, hs[-1])
