"""Discretized continuous action space (reference
algorithms/spaces/discretized.py:4-14): a Discrete(n) whose index i maps to
min + i * (max - min) / (n - 1)."""

from ..envs.gym_compat import Discrete


class Discretized(Discrete):

  def __init__(self, n, min_action, max_action):
    super().__init__(n)
    self.min_action = min_action
    self.max_action = max_action

  def to_continuous(self, discrete_action):
    step = (self.max_action - self.min_action) / (self.n - 1)
    return self.min_action + discrete_action * step

  def __repr__(self):
    return 'Discretized(%d, %g, %g)' % (self.n, self.min_action,
                                         self.max_action)
