"""Loader for the host-only C++ runtime (`_native.so`: dynamic batcher,
shared-memory trajectory ring, image ops).

`load(sanitize='thread'|'address')` loads the sanitizer build produced by
`python csrc/build.py --only native --sanitize <kind>` (host code only; the
process must be started with the sanitizer runtime preloaded).
"""

import importlib
import importlib.machinery
import importlib.util
import os

_MOD = None
_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))


def load(sanitize=None):
  global _MOD
  if sanitize:
    path = os.path.join(_ROOT, 'build', 'san_' + sanitize, '_native.so')
    if not os.path.exists(path):
      raise RuntimeError('sanitizer build missing: run `python csrc/build.py '
                         '--only native --sanitize %s`' % sanitize)
    loader = importlib.machinery.ExtensionFileLoader('_native', path)
    spec = importlib.util.spec_from_file_location('_native', path,
                                                  loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod
  if _MOD is None:
    try:
      _MOD = importlib.import_module('scalable_agent_amd.runtime._native')
    except ImportError as e:
      raise RuntimeError('native runtime not built: run `python csrc/build.py '
                         '--only native` (%s)' % e) from e
  return _MOD


def __getattr__(name):  # module-level lazy attribute access
  return getattr(load(), name)
