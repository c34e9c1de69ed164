"""General utilities (reference utils/utils.py:13-200): the `rl` logger,
AttrDict, str2bool, numpy helpers, filesystem layout of experiments
(train_dir/<experiments_root>/<experiment>/{cfg.json,.summary,.model}),
memory introspection and process killing (always by exact pid)."""

import argparse
import logging
import operator
import os
import signal
import sys
from os.path import join

import numpy as np
import psutil

MAP_FIGURE_ID = 2       # reference utils/plot.py
HEATMAP_FIGURE_ID = 3


class _ColorFormatter(logging.Formatter):
  """ANSI-coloured levels on a TTY (the reference uses colorlog, which is not
  in this image); plain text otherwise."""

  _COLORS = {'DEBUG': '\033[36m', 'INFO': '\033[1;37m',
             'WARNING': '\033[33m', 'ERROR': '\033[1;31m',
             'CRITICAL': '\033[31;47m'}

  def __init__(self, color):
    super().__init__('[%(asctime)s][%(process)05d] %(message)s')
    self._color = color

  def format(self, record):
    msg = super().format(record)
    if self._color and record.levelname in self._COLORS:
      return self._COLORS[record.levelname] + msg + '\033[0m'
    return msg


log = logging.getLogger('rl')
if not log.handlers:
  _h = logging.StreamHandler()
  _h.setLevel(logging.DEBUG)
  _h.setFormatter(_ColorFormatter(hasattr(sys.stderr, 'isatty')
                                  and sys.stderr.isatty()))
  log.addHandler(_h)
  log.setLevel(logging.DEBUG)
  log.propagate = False


class AttrDict(dict):
  """dict with attribute access; missing attributes raise AttributeError so
  `hasattr`, copy and pickle behave."""

  def __getattr__(self, item):
    try:
      return self[item]
    except KeyError:
      raise AttributeError(item)

  def __setattr__(self, key, value):
    self[key] = value

  def __delattr__(self, item):
    try:
      del self[item]
    except KeyError:
      raise AttributeError(item)


def str2bool(v):
  if isinstance(v, bool):
    return v
  if isinstance(v, str) and v.lower() in ('true', 't', 'yes', 'y', '1'):
    return True
  if isinstance(v, str) and v.lower() in ('false', 'f', 'no', 'n', '0'):
    return False
  raise argparse.ArgumentTypeError('Boolean value expected')


def scale_to_range(np_array, min_, max_):
  lo, hi = np.min(np_array), np.max(np_array)
  unit = (np_array - lo) / (hi - lo)
  return unit * (max_ - min_) + min_


def op_with_idx(x, op):
  assert len(x) > 0
  best_idx, best_x = 0, x[0]
  for i, v in enumerate(x):
    if op(v, best_x):
      best_x, best_idx = v, i
  return best_x, best_idx


def min_with_idx(x):
  return op_with_idx(x, operator.lt)


def max_with_idx(x):
  return op_with_idx(x, operator.gt)


def numpy_all_the_way(list_of_arrays):
  """List of same-shape arrays -> one array with a new leading dimension."""
  return np.stack([np.asarray(a) for a in list_of_arrays])


def numpy_flatten(list_of_arrays):
  return np.concatenate(list_of_arrays, axis=0)


def ensure_contigious(x):
  return x if x.flags['C_CONTIGUOUS'] else np.ascontiguousarray(x)


def figure_to_numpy(figure):
  """Matplotlib figure -> HxWx4 RGBA uint8 array."""
  figure.canvas.draw()
  w, h = figure.canvas.get_width_height()
  argb = np.frombuffer(figure.canvas.tostring_argb(), dtype=np.uint8)
  return np.roll(argb.reshape(h, w, 4), 3, axis=2)


def memory_consumption_mb():
  return psutil.Process(os.getpid()).memory_info().rss / (1024 * 1024)


def kill(pid, sig=signal.SIGKILL):
  """Kills ONE exact pid and its descendants (never pattern-based)."""
  try:
    proc = psutil.Process(pid)
    children = proc.children(recursive=True)
  except psutil.NoSuchProcess:
    return
  for p in children + [proc]:
    try:
      p.send_signal(sig)
    except psutil.NoSuchProcess:
      pass


def kill_processes(processes):
  for p in processes:
    try:
      if p.is_running():
        p.kill()
    except psutil.NoSuchProcess:
      pass


def list_child_processes():
  return psutil.Process(os.getpid()).children(recursive=True)


def ensure_dir_exists(path):
  os.makedirs(path, exist_ok=True)
  return path


def remove_if_exists(file):
  if os.path.isfile(file):
    os.remove(file)


def project_root():
  """Root of the repository (train_dir and caches live under it)."""
  return os.path.dirname(os.path.dirname(os.path.dirname(
      os.path.abspath(__file__))))


def experiments_dir():
  root = os.environ.get('SA_TRAIN_DIR') or join(project_root(), 'train_dir')
  return ensure_dir_exists(root)


def experiment_dir(experiment=None, experiments_root=None, cfg=None):
  if cfg is not None:
    experiment = _cfg_get(cfg, 'experiment')
    experiments_root = _cfg_get(cfg, 'experiments_root')
  root = experiments_dir()
  if experiments_root is not None:
    root = join(root, experiments_root)
  return ensure_dir_exists(join(root, experiment))


def model_dir(experiment_dir_):
  return ensure_dir_exists(join(experiment_dir_, '.model'))


def summaries_dir(experiment_dir_):
  return ensure_dir_exists(join(experiment_dir_, '.summary'))


def cfg_file(cfg):
  return join(experiment_dir(cfg=cfg), 'cfg.json')


def _cfg_get(cfg, key, default=None):
  if isinstance(cfg, dict):
    return cfg.get(key, default)
  return getattr(cfg, key, default)
