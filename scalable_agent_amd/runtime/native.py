"""Loader for the host-only C++ runtime (`_native.so`: batcher, shm ring)."""

import importlib

_MOD = None


def load(sanitize=None):
  global _MOD
  if sanitize:
    return importlib.import_module('scalable_agent_amd.runtime._native_' +
                                   sanitize)
  if _MOD is None:
    try:
      _MOD = importlib.import_module('scalable_agent_amd.runtime._native')
    except ImportError as e:
      raise RuntimeError('native runtime not built: run `python csrc/build.py '
                         '--only native` (%s)' % e) from e
  return _MOD


def __getattr__(name):  # module-level lazy attribute access
  return getattr(load(), name)
