"""Landmark-based exploration bonus (reference envs/doom/wrappers/
exploration.py): +0.1 intrinsic reward (info['intrinsic_reward']) for
reaching a pose farther than 75 units (distance + angle/2) from all of the
last 200 landmarks."""

import collections
import math

import numpy as np

from ...gym_compat import Wrapper


class ExplorationWrapper(Wrapper):

  def __init__(self, env):
    super().__init__(env)
    self.landmarks = collections.deque([], maxlen=200)
    self.landmark_threshold = 75.0

  def _calc_intrinsic_reward(self, info):
    pos = info.get('pos', None)
    if pos is None:
      return 0.0
    x, y, a = pos['agent_x'], pos['agent_y'], pos['agent_a']
    for (x0, y0, a0) in self.landmarks:
      da = abs(a - a0)
      d = math.hypot(x - x0, y - y0) + min(da, 360.0 - da) / 2
      if d < self.landmark_threshold:
        reward = 0.0
        break
    else:
      self.landmarks.appendleft((x, y, a))
      reward = 0.1
    while len(self.landmarks) >= self.landmarks.maxlen:
      del self.landmarks[np.random.randint(0, len(self.landmarks))]
    return reward

  def reset(self, **kwargs):
    self.landmarks = collections.deque([], maxlen=200)
    return self.env.reset()

  def step(self, action):
    obs, reward, done, info = self.env.step(action)
    info['intrinsic_reward'] = info.get('intrinsic_reward', 0.0) + \
        self._calc_intrinsic_reward(info)
    return obs, reward, done, info
