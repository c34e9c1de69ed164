"""A stand-in `deepmind_lab` module (DeepMind Lab is not installed in the
image) implementing the slice of the Lab API that PyProcessDmLab uses, and
recording every call so tests can check the adapter's behaviour.

Episodes last `episodeLengthSteps` (config, default 5) calls to step(); the
reward of a step is num_steps * (1 + first action component != 0); frames
encode (reset seed, step) so tests can tell episodes apart."""

import numpy as np

CALLS = []
RUNFILES = []


def set_runfiles_path(path):
  RUNFILES.append(path)


class Lab(object):

  def __init__(self, level, observations, config=None, level_cache=None,
               renderer='software'):
    CALLS.append(('init', level, tuple(observations), dict(config or {}),
                  renderer))
    for v in (config or {}).values():
      assert isinstance(v, str), 'Lab configs are strings'
    self.level = level
    self._obs = list(observations)
    self._config = dict(config or {})
    self._w = int(self._config.get('width', 96))
    self._h = int(self._config.get('height', 72))
    self._len = int(self._config.get('episodeLengthSteps', 5))
    self._seed = None
    self._t = 0
    self._running = False
    self.steps = []
    self.resets = []
    self.closed = False

  def reset(self, seed=None):
    self.resets.append(seed)
    CALLS.append(('reset', seed))
    self._seed = seed
    self._t = 0
    self._running = True

  def is_running(self):
    return self._running

  def observations(self):
    assert self._running, 'observations() after the episode ended'
    frame = np.zeros((self._h, self._w, 3), np.uint8)
    frame[..., 0] = (self._seed or 0) % 251
    frame[..., 1] = self._t % 251
    out = {'RGB_INTERLEAVED': frame,
           'INSTR': 'go to the red ball' if self._t % 2 == 0 else 'pick it up'}
    return {k: out[k] for k in self._obs}

  def step(self, action, num_steps=1):
    assert self._running
    action = np.asarray(action)
    assert action.dtype == np.intc and action.shape == (7,), action
    self.steps.append((action.copy(), num_steps))
    CALLS.append(('step', tuple(int(a) for a in action), num_steps))
    self._t += 1
    if self._t >= self._len:
      self._running = False
    return float(num_steps * (1 + (action[0] != 0)))

  def close(self):
    self.closed = True
    CALLS.append(('close',))
