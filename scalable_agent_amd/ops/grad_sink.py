"""Direct gradient accumulation into the learner's flat fp32 gradient buffer.

The learner keeps every parameter's `.grad` as a view into ONE flat fp32
buffer (optim.FlatParams).  Inside `direct_grads()` the fused HIP ops
accumulate their weight gradients straight into those views (GEMM epilogues
with beta=1, fp32 atomics in the kernels) and return None for the parameter,
which is exactly AccumulateGrad's `grad += g` without the extra add kernel,
the temporary, and (for sliced weights such as the LSTM kernel) the
zero-filled full-size slice-backward tensor.  Outside the context (tests,
torch.autograd.grad) the ops return ordinary gradient tensors.
"""

import contextlib

import torch

_DIRECT = False


@contextlib.contextmanager
def direct_grads(on=True):
  """Backward passes run inside accumulate parameter gradients in place.
  (A module flag, not thread-local: autograd runs GPU backward nodes on its
  own worker thread.)"""
  global _DIRECT
  prev = _DIRECT
  _DIRECT = bool(on)
  try:
    yield
  finally:
    _DIRECT = prev


def sink(p):
  """p.grad when it can take in-place fp32 accumulation, else None."""
  if not _DIRECT:
    return None
  g = p.grad
  if (g is not None and g.dtype == torch.float32 and g.is_contiguous() and
      g.shape == p.shape and g.device == p.device):
    return g
  return None


def sinks(params):
  """-> (per-param fp32 accumulation buffers, per-param 'is p.grad')."""
  views, direct = [], []
  fresh = [q for q in params if sink(q) is None]
  buf = None
  if fresh:
    buf = torch.zeros(sum(q.numel() for q in fresh), dtype=torch.float32,
                      device=params[0].device)
  o = 0
  for q in params:
    s = sink(q)
    if s is not None:
      views.append(s)
      direct.append(True)
    else:
      views.append(buf[o:o + q.numel()].view_as(q))
      o += q.numel()
      direct.append(False)
  return views, direct


def returned(views, direct):
  """Gradients to hand back to autograd: None where accumulated in place."""
  return tuple(None if d else g for g, d in zip(views, direct))


# ---- off-critical-path weight-gradient GEMMs -------------------------------
# Inside overlap_weight_grads(), ops may enqueue work that only produces
# parameter gradients (into direct sinks) on a side stream, forked from the
# current stream; the context joins every side stream back into the caller's
# current stream on exit, so the optimizer (and a graph capture's end) sees
# the finished gradients.  The fused core uses it to run dW_h / dW_x / dW_fc
# / db_lstm next to the conv-torso backward instead of in front of it.
_OVERLAP = False
_SIDE_STREAMS = {}
_PENDING = []


@contextlib.contextmanager
def overlap_weight_grads(on=True):
  global _OVERLAP
  prev = _OVERLAP
  _OVERLAP = bool(on)
  try:
    yield
  finally:
    _OVERLAP = prev
    join_side_streams()


def side_stream(device):
  """The side stream for gradient-only work, or None when not overlapping."""
  if not (_OVERLAP and _DIRECT) or device.type != 'cuda':
    return None
  s = _SIDE_STREAMS.get(device)
  if s is None:
    s = torch.cuda.Stream(device)
    _SIDE_STREAMS[device] = s
  if s not in _PENDING:
    _PENDING.append(s)
  return s


def join_side_streams():
  while _PENDING:
    s = _PENDING.pop()
    torch.cuda.current_stream(s.device).wait_stream(s)
