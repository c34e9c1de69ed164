"""Experiment knobs of the Python side (the native ones: csrc/kernels/knobs.h).

`measure_env(name, default)` returns the environment variable `name` only
when SA_MEASURE_KNOBS=1 is set too, else `default`: the switches of
measured-and-rejected variants (profiles/experiments.md) and of diagnostic
runs (SA_BENCH_SKIP_H2D drops work from the timed step) cannot change a
production run by accident.  `set_knobs()` lists every SA_* variable of the
environment; bench.py reports it as config.knobs.
"""

import os


def measure_env(name, default=None):
  if os.environ.get('SA_MEASURE_KNOBS') != '1':
    return default
  return os.environ.get(name, default)


def set_knobs(environ=None):
  """{name: value} of every SA_* variable set in the environment."""
  env = os.environ if environ is None else environ
  return {k: v for k, v in sorted(env.items()) if k.startswith('SA_')}
