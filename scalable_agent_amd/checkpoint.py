"""Checkpoint / resume (reference: MonitoredTrainingSession, experiment.py:608-612).

Layout in `logdir` (TF-Saver-like):
  checkpoint                         text file naming the latest checkpoint
  checkpoint_<num_env_frames>.pt     {params (by TF variable name), RMSProp
                                      ms/mom, num_environment_frames, flags,
                                      rng state, format version}
Saved atomically (write to a temp file, fsync, rename), every
`save_checkpoint_secs` (600 by default), keeping the newest `keep` (5, the TF
Saver default).  Restore happens automatically on start; `--mode=test` reads
the same files.  Files are loaded with `torch.load(weights_only=True)`.

`--checkpoint_format=tf` writes the reference's own layout instead
(experiment.py:608-616): `model.ckpt-<frames>.{index,data-00000-of-00001}`
plus a TF `checkpoint` index (tf_checkpoint.export_tf_checkpoint), with the
RMSProp slots, the frame counter and PopArt statistics as extra variables.
`latest_checkpoint` / `restore` / `load_state` accept either layout, so
training resumes and `--mode=test` evaluates from whichever a logdir holds.
"""

import glob
import os
import re
import time

import torch

FORMAT_VERSION = 1
_RE = re.compile(r'checkpoint_(\d+)\.pt$')


def _list(logdir):
  out = []
  for p in glob.glob(os.path.join(logdir, 'checkpoint_*.pt')):
    m = _RE.search(p)
    if m:
      out.append((int(m.group(1)), p))
  return sorted(out)


def is_tf(path):
  """True for a TF checkpoint prefix (model.ckpt-N), False for a .pt file."""
  return path is not None and not path.endswith('.pt') and os.path.exists(
      path + '.index')


def latest_checkpoint(logdir):
  """Path of the latest checkpoint in logdir (a .pt file or a TF prefix), or
  None."""
  from . import tf_checkpoint
  idx = os.path.join(logdir, 'checkpoint')
  if os.path.exists(idx):
    text = open(idx).read()
    if 'model_checkpoint_path' in text:
      p = tf_checkpoint.latest_checkpoint(logdir)
      if p is not None and is_tf(p):
        return p
    else:
      p = os.path.join(logdir, text.strip())
      if os.path.exists(p):
        return p
  # no (usable) index: the newest of either layout
  cands = _list(logdir) + tf_checkpoint.list_tf_checkpoints(logdir)
  return max(cands)[1] if cands else None


def _to_cpu(x):
  if torch.is_tensor(x):
    return x.detach().to('cpu')
  if isinstance(x, dict):
    return {k: _to_cpu(v) for k, v in x.items()}
  return x


def save_tf(logdir, learner, keep=5):
  """The reference layout: model.ckpt-<frames> + `checkpoint`."""
  from . import tf_checkpoint
  os.makedirs(logdir, exist_ok=True)
  extra = {}
  if getattr(learner, 'popart', None) is not None:
    for k, v in learner.popart.state_dict().items():
      extra['popart/' + k] = v.detach().cpu().numpy()
  return tf_checkpoint.export_tf_checkpoint(logdir, learner, keep=keep,
                                            extra=extra)


def save(logdir, learner, flags=None, keep=5, extra=None, fmt='pt'):
  """Writes checkpoint_<frames>.pt atomically and prunes old ones (fmt='tf':
  save_tf)."""
  if fmt == 'tf':
    return save_tf(logdir, learner, keep)
  os.makedirs(logdir, exist_ok=True)
  frames = int(learner.frames.item())
  names = learner.agent.tf_variable_names()
  state = {
      'format_version': FORMAT_VERSION,
      'num_environment_frames': frames,
      'params': {names[n]: p.detach().cpu() for n, p in learner.flat.named},
      'rmsprop': {'ms': learner.opt.ms.detach().cpu(),
                  'mom': learner.opt.mom.detach().cpu()},
      'flags': {k: v for k, v in vars(flags).items()
                if isinstance(v, (int, float, str, bool))} if flags else {},
      'torch_rng': torch.get_rng_state(),
      'time': time.time(),
  }
  if getattr(learner, 'popart', None) is not None:
    state['popart'] = _to_cpu(learner.popart.state_dict())
  if extra:
    state['extra'] = _to_cpu(extra)
  name = 'checkpoint_%d.pt' % frames
  path = os.path.join(logdir, name)
  tmp = path + '.tmp'
  with open(tmp, 'wb') as f:
    torch.save(state, f)
    f.flush()
    os.fsync(f.fileno())
  os.replace(tmp, path)
  idx_tmp = os.path.join(logdir, 'checkpoint.tmp')
  with open(idx_tmp, 'w') as f:
    f.write(name + '\n')
  os.replace(idx_tmp, os.path.join(logdir, 'checkpoint'))
  for _, old in _list(logdir)[:-keep]:
    try:
      os.remove(old)
    except OSError:
      pass
  return path


def load_state(path):
  """-> {'params': {tf_name: tensor}, 'num_environment_frames', ...}."""
  if is_tf(path):
    from . import tf_checkpoint
    t = tf_checkpoint.read_checkpoint(path)
    params = {k: torch.from_numpy(v.copy()) for k, v in t.items()
              if not k.endswith(('/RMSProp', '/RMSProp_1')) and
              k != 'num_environment_frames' and not k.startswith('popart/')}
    state = {'params': params, 'format': 'tf',
             'num_environment_frames': int(t.get('num_environment_frames',
                                                 0))}
    pop = {k[len('popart/'):]: torch.from_numpy(v.copy())
           for k, v in t.items() if k.startswith('popart/')}
    if pop:
      state['popart'] = pop
    return state
  return torch.load(path, map_location='cpu', weights_only=True)


def restore_agent(agent, state):
  """Loads parameters (by TF variable name) into an Agent."""
  names = agent.tf_variable_names()
  params = state['params']
  with torch.no_grad():
    for n, p in agent.named_parameters():
      p.copy_(params[names[n]].to(p.device))
  if getattr(agent, '_inference_cache', None) is not None:
    # an inference agent's per-step weight forms; its inference runs on its
    # model's own stream, so the refresh is finished here
    agent.refresh_inference_cache()
    if agent.lstm_kernel.is_cuda:
      torch.cuda.current_stream(agent.lstm_kernel.device).synchronize()


def restore(logdir, learner):
  """Restores the latest checkpoint into a Learner; returns frames or None."""
  path = latest_checkpoint(logdir)
  if path is None:
    return None
  if is_tf(path):
    from . import tf_checkpoint
    frames = tf_checkpoint.import_tf_checkpoint(path, learner=learner)
    if getattr(learner, 'popart', None) is not None:
      pop = load_state(path).get('popart')
      if pop:
        learner.popart.load_state_dict(pop)
    return int(frames or 0)
  state = load_state(path)
  restore_agent(learner.agent, state)
  learner.opt.ms.copy_(state['rmsprop']['ms'].to(learner.opt.ms.device))
  learner.opt.mom.copy_(state['rmsprop']['mom'].to(learner.opt.mom.device))
  learner.frames.fill_(int(state['num_environment_frames']))
  if getattr(learner, 'popart', None) is not None and 'popart' in state:
    learner.popart.load_state_dict(state['popart'])
  if 'torch_rng' in state:
    torch.set_rng_state(state['torch_rng'])
  return int(state['num_environment_frames'])


class PeriodicSaver(object):
  """Saves every `secs` seconds (save_checkpoint_secs)."""

  def __init__(self, logdir, learner, flags, secs=600, keep=5):
    self.logdir, self.learner, self.flags = logdir, learner, flags
    self.secs, self.keep = secs, keep
    self.fmt = getattr(flags, 'checkpoint_format', 'pt') if flags else 'pt'
    self._last = time.time()

  def maybe_save(self, force=False):
    if force or time.time() - self._last >= self.secs:
      self._last = time.time()
      return save(self.logdir, self.learner, self.flags, self.keep,
                  fmt=self.fmt)
    return None
