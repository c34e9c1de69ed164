"""Piecewise-linear schedules (reference utils/decay.py: LinearDecay)."""

import math


class LinearDecay(object):
  """Linear interpolation between (step, value) milestones, optional stairs."""

  def __init__(self, milestones, staircase=None):
    if not milestones:
      raise Exception('Milestones list should not be empty!')
    self._schedule = sorted(milestones)
    self._staircase = staircase

  def at(self, step):
    if step <= self._schedule[0][0]:
      return self._schedule[0][1]
    if step >= self._schedule[-1][0]:
      return self._schedule[-1][1]
    m = 0
    while self._schedule[m][0] < step:
      m += 1
    x0, y0 = self._schedule[m - 1]
    x1, y1 = self._schedule[m]
    value = y0 + (y1 - y0) * (step - x0) / (x1 - x0)
    if self._staircase is None:
      return value
    stairs = math.floor(value / self._staircase)
    return max(stairs * self._staircase, self._schedule[0][1])
