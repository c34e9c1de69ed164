"""Timing helpers: the reference's `Timing` context timers (utils/timing.py)
plus `StepTimer`, the always-on learner throughput meter."""

import time
from collections import deque

from .utils import AttrDict

EPS = 1e-8


class AvgTime(object):
  def __init__(self, num_values_to_avg):
    self.values = deque([], maxlen=num_values_to_avg)

  def __str__(self):
    return '%.4f' % (sum(self.values) / max(1, len(self.values)))


class TimingContext(object):
  def __init__(self, timer, key, additive=False, average=None):
    self._timer, self._key = timer, key
    self._additive, self._average = additive, average
    self._time_enter = None

  def __enter__(self):
    self._time_enter = time.time()

  def __exit__(self, type_, value, traceback):
    if self._key not in self._timer:
      self._timer[self._key] = (AvgTime(self._average)
                                if self._average is not None else 0)
    passed = max(time.time() - self._time_enter, EPS)
    if self._additive:
      self._timer[self._key] += passed
    elif self._average is not None:
      self._timer[self._key].values.append(passed)
    else:
      self._timer[self._key] = passed


class Timing(AttrDict):
  def timeit(self, key):
    return TimingContext(self, key)

  def add_time(self, key):
    return TimingContext(self, key, additive=True)

  def time_avg(self, key, average=10):
    return TimingContext(self, key, average=average)

  def __str__(self):
    parts = []
    for key, value in self.items():
      parts.append('%s: %s' % (key, ('%.4f' % value) if isinstance(value, float)
                               else str(value)))
    return ', '.join(parts)


class StepTimer(object):
  """Sliding-window frames/s, learner steps/s and queue-wait fraction."""

  def __init__(self, frames_per_step, window=50):
    self.frames_per_step = frames_per_step
    self._times = deque(maxlen=window)
    self._waits = deque(maxlen=window)
    self._pending_wait = 0.0
    self._times.append(time.time())

  def add_wait(self, secs):
    self._pending_wait += secs

  def step(self):
    self._times.append(time.time())
    self._waits.append(self._pending_wait)
    self._pending_wait = 0.0

  def steps_per_sec(self):
    if len(self._times) < 2:
      return 0.0
    return (len(self._times) - 1) / max(self._times[-1] - self._times[0], EPS)

  def frames_per_sec(self):
    return self.steps_per_sec() * self.frames_per_step

  def wait_fraction(self):
    if len(self._times) < 2:
      return 0.0
    return min(1.0, sum(self._waits) / max(self._times[-1] - self._times[0],
                                           EPS))
