"""TF1/Sonnet-semantics building blocks (pure PyTorch reference).

Layouts follow the reference's TF conventions so that checkpoints map 1:1 onto
the reference variable names:
  * activations NHWC, conv kernels HWIO `[kh, kw, cin, cout]`   (snt.Conv2D)
  * linear kernels `[in, out]`                                (snt.Linear)
  * LSTM kernels `[in + hidden, 4 * hidden]`, gate order i, c~, f, o, forget
    bias +1.0, no peephole, no clip                          (LSTMBlockCell)

These functions are the numerical oracle for the HIP kernels in
`scalable_agent_amd.ops`.
"""

import math

import torch
import torch.nn.functional as F


def same_pads(n, k, s):
  """TF 'SAME' padding (before, after) for one spatial dim."""
  out = -(-n // s)
  total = max((out - 1) * s + k - n, 0)
  return total // 2, total - total // 2


def same_out(n, s):
  return -(-n // s)


def conv2d_same_nhwc(x, w, b=None, stride=1):
  """x: [N,H,W,Cin], w: [kh,kw,Cin,Cout] -> [N,Ho,Wo,Cout] (TF SAME)."""
  kh, kw = w.shape[0], w.shape[1]
  ph = same_pads(x.shape[1], kh, stride)
  pw = same_pads(x.shape[2], kw, stride)
  xc = x.permute(0, 3, 1, 2)
  xc = F.pad(xc, (pw[0], pw[1], ph[0], ph[1]))
  y = F.conv2d(xc, w.permute(3, 2, 0, 1), b, stride=stride)
  return y.permute(0, 2, 3, 1)


def maxpool_same_nhwc(x, k=3, s=2):
  """Max pool with TF SAME padding (padding never wins: filled with -inf)."""
  ph = same_pads(x.shape[1], k, s)
  pw = same_pads(x.shape[2], k, s)
  xc = x.permute(0, 3, 1, 2)
  xc = F.pad(xc, (pw[0], pw[1], ph[0], ph[1]), value=float('-inf'))
  y = F.max_pool2d(xc, k, s)
  return y.permute(0, 2, 3, 1)


def lstm_block_cell(x, c, h, kernel, bias, forget_bias=1.0):
  """TF LSTMBlockCell step. Returns (h_new, c_new)."""
  gates = torch.cat([x, h], dim=-1) @ kernel + bias
  i, ci, f, o = gates.chunk(4, dim=-1)
  i = torch.sigmoid(i)
  f = torch.sigmoid(f + forget_bias)
  ci = torch.tanh(ci)
  c_new = ci * i + c * f
  h_new = torch.tanh(c_new) * torch.sigmoid(o)
  return h_new, c_new


# ---------------------------------------------------------------- initialisers

def truncated_normal_(t, std, generator=None):
  """TF truncated_normal: resample outside 2 std."""
  with torch.no_grad():
    t.normal_(0, 1, generator=generator)
    while True:
      bad = t.abs() > 2
      if not bad.any():
        break
      t[bad] = torch.randn(int(bad.sum()), generator=generator,
                           dtype=t.dtype, device=t.device)
    t.mul_(std)
  return t


def sonnet_linear_init_(w, generator=None):
  """snt.Linear / snt.Conv2D default: truncated normal, std 1/sqrt(fan_in)."""
  fan_in = int(math.prod(w.shape[:-1]))
  return truncated_normal_(w, 1.0 / math.sqrt(fan_in), generator)


def glorot_uniform_(w, generator=None):
  """tf.get_variable default initializer (LSTMBlockCell kernel)."""
  fan_in = int(math.prod(w.shape[:-1]))
  fan_out = int(w.shape[-1])
  limit = math.sqrt(6.0 / (fan_in + fan_out))
  with torch.no_grad():
    w.uniform_(-limit, limit, generator=generator)
  return w


class _EmbeddingLookup(torch.autograd.Function):
  """table[ids] whose backward is a fixed-size scatter-add: graph-capture
  safe on the GPU (torch's embedding backward sorts and compacts the ids,
  sizing work from the data, which a replayed hipGraph cannot follow).
  Deterministic mode (torch.are_deterministic_algorithms_enabled()): the
  gradient is one_hot(ids)^T @ g, a GEMM with a fixed summation order."""

  @staticmethod
  def forward(ctx, ids, table):
    flat = ids.reshape(-1)
    ctx.save_for_backward(flat)
    ctx.V = table.shape[0]
    return table.index_select(0, flat).view(*ids.shape, table.shape[1])

  @staticmethod
  def backward(ctx, g):
    (flat,) = ctx.saved_tensors
    g2 = g.reshape(flat.numel(), -1).float()
    if torch.are_deterministic_algorithms_enabled():
      onehot = F.one_hot(flat, ctx.V).to(g2.dtype)
      grad = onehot.t() @ g2
    else:
      grad = torch.zeros(ctx.V, g2.shape[1], dtype=g2.dtype, device=g2.device)
      grad.index_add_(0, flat, g2)
    return None, grad


def embedding_lookup(ids, table):
  """tf.nn.embedding_lookup (reference experiment.py:131-133)."""
  return _EmbeddingLookup.apply(ids, table)
