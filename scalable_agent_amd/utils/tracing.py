"""roctx ranges.  With SA_TRACE=1 every `trace(name)` block
becomes a roctx range (torch.cuda.nvtx maps to roctx on ROCm), visible with
`rocprofv3 --marker-trace` next to the kernel trace.  Off by default: zero
cost beyond one flag test."""

import contextlib
import os

_ENABLED = os.environ.get('SA_TRACE', '0') == '1'


def enabled():
  return _ENABLED


def set_enabled(on):
  global _ENABLED
  _ENABLED = bool(on)


@contextlib.contextmanager
def trace(name):
  if not _ENABLED:
    yield
    return
  import torch
  torch.cuda.nvtx.range_push(name)
  try:
    yield
  finally:
    torch.cuda.nvtx.range_pop()


def mark(name):
  if _ENABLED:
    import torch
    torch.cuda.nvtx.mark(name)
