"""Loader for the in-tree HIP extension (`scalable_agent_amd/_C.so`)."""

import importlib
import importlib.util as importlib_util
import os

_EXT = None
_ERR = None


def load():
  """Imports the compiled extension; raises with a clear message if absent."""
  global _EXT, _ERR
  if _EXT is not None:
    return _EXT
  try:
    import torch  # noqa: F401  (libtorch must be loaded first)
    alt = os.environ.get('SA_EXT_PATH')  # experiment builds (e.g. ablation)
    if alt:
      spec = importlib_util.spec_from_file_location('scalable_agent_amd._C', alt)
      _EXT = importlib_util.module_from_spec(spec)
      spec.loader.exec_module(_EXT)
    else:
      _EXT = importlib.import_module('scalable_agent_amd._C')
  except Exception as e:  # pragma: no cover - depends on build state
    _ERR = e
    raise RuntimeError(
        'HIP extension scalable_agent_amd._C is not built/loadable (%s). '
        'Build it with `python csrc/build.py` (hipcc, gfx950).' % e) from e
  return _EXT


def available():
  try:
    load()
    return True
  except RuntimeError:
    return False


def ext():
  return load()


def check_cuda(*tensors):
  for t in tensors:
    if t is not None and not t.is_cuda:
      raise ValueError('HIP op called with a non-GPU tensor')
