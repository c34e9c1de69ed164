"""Instruction encoder on one fused HIP kernel per direction.

Reference: experiment.py:123-146 - hashed word ids -> Embed(1000, 20) ->
dynamic_rnn(LSTMBlockCell(64), sequence_length) -> the output at the last
valid word (zeros for an empty instruction), gate order i, c~, f, o, forget
bias +1.  csrc/kernels/lang_lstm.hip runs the whole word loop of 16 frames
per workgroup (embedding gather, the [x_t, h_{t-1}] x K product on fp32
MFMA, the cell update) forward and backward; the parameter gradients are
dK = xh^T dgates and db = 1^T dgates (one exact-fp32 GEMM with the ones-row
bias gradient, gemm_f32); the backward kernel adds the valid words' dx rows
into the embedding gradient itself.
"""

import torch

from . import grad_sink
from ._ext import ext


class _LanguageLSTM(torch.autograd.Function):

  @staticmethod
  def forward(ctx, ids, lengths, embed, kernel, bias):
    out, acts, cs, xh = ext().lang_lstm_fwd(ids, lengths, embed, kernel, bias)
    ctx.save_for_backward(ids, lengths, embed, kernel, bias, acts, cs, xh)
    return out

  @staticmethod
  def backward(ctx, dout):
    ids, lengths, embed, kernel, bias, acts, cs, xh = ctx.saved_tensors
    C = ext()
    (gemb, gk, gb), direct = grad_sink.sinks([embed, kernel, bias])
    det = torch.are_deterministic_algorithms_enabled()
    # embedding rows: the backward kernel adds each valid word's dx into its
    # row (atomics, like a scatter-add); deterministic mode takes dx back and
    # sums it with a one-hot product in a fixed order
    dg, dx = C.lang_lstm_bwd(lengths, kernel, dout.float().contiguous(), acts, cs,
                             ids=None if det else ids,
                             egrad=None if det else gemb)
    L, N, G = dg.shape
    xh2, dg2 = xh.view(L * N, xh.shape[2]), dg.view(L * N, G)
    # the A^T B form takes any K (= L * N)
    C.gemm_f32(xh2, dg2, True, False, gk, accumulate=True, colsum=gb)
    if det:
      # steps past an instruction's length carry dx = 0; out-of-range ids
      # read row 0 in the forward kernel, so their gradient goes to row 0
      flat = ids.t().reshape(-1)  # [L*N] in the kernel's (t, n) order
      flat = torch.where((flat >= 0) & (flat < embed.shape[0]), flat,
                         torch.zeros_like(flat))
      dx2 = dx.view(L * N, dx.shape[2])
      onehot = torch.nn.functional.one_hot(flat, embed.shape[0]).to(dx2.dtype)
      gemb.add_(onehot.t() @ dx2)
    return (None, None) + grad_sink.returned((gemb, gk, gb), direct)


def language_lstm(ids, lengths, embed, kernel, bias):
  """ids [N, L] int64 word ids, lengths [N] -> [N, 64] (fp32)."""
  return _LanguageLSTM.apply(ids.to(torch.int64).contiguous(),
                             lengths.to(torch.int64).contiguous(),
                             embed.contiguous(), kernel.contiguous(),
                             bias.contiguous())
