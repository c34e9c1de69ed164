"""General utilities (reference utils/utils.py): logger, AttrDict, str2bool,
filesystem helpers, memory introspection, process killing."""

import argparse
import logging
import os
import signal

import psutil

log = logging.getLogger('rl')
if not log.handlers:
  _h = logging.StreamHandler()
  _h.setFormatter(logging.Formatter(
      '[%(asctime)s][%(process)05d] %(levelname)s %(message)s'))
  log.addHandler(_h)
  log.setLevel(logging.DEBUG)
  log.propagate = False


class AttrDict(dict):
  __getattr__ = dict.__getitem__

  def __setattr__(self, key, value):
    self[key] = value


def str2bool(v):
  if isinstance(v, bool):
    return v
  if isinstance(v, str) and v.lower() in ('true', 't', 'yes', 'y', '1'):
    return True
  if isinstance(v, str) and v.lower() in ('false', 'f', 'no', 'n', '0'):
    return False
  raise argparse.ArgumentTypeError('Boolean value expected')


def ensure_dir_exists(path):
  os.makedirs(path, exist_ok=True)
  return path


def remove_if_exists(file):
  if os.path.isfile(file):
    os.remove(file)


def project_root():
  return os.path.dirname(os.path.dirname(os.path.dirname(
      os.path.abspath(__file__))))


def experiments_dir(root=None):
  return ensure_dir_exists(os.path.join(root or project_root(), 'train_dir'))


def experiment_dir(experiment, root=None):
  return ensure_dir_exists(os.path.join(experiments_dir(root), experiment))


def cfg_file(experiment, root=None):
  return os.path.join(experiment_dir(experiment, root), 'cfg.json')


def memory_consumption_mb():
  return psutil.Process(os.getpid()).memory_info().rss / 1e6


def kill(pid, sig=signal.SIGKILL):
  """Kills ONE exact pid (never pattern-based)."""
  try:
    os.kill(pid, sig)
  except ProcessLookupError:
    pass


def list_child_processes():
  return psutil.Process(os.getpid()).children(recursive=True)


def kill_processes(processes):
  for p in processes:
    try:
      if p.is_running():
        p.kill()
    except psutil.NoSuchProcess:
      pass
