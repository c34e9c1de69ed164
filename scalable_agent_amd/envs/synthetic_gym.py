"""Synthetic gym env (no simulator): random frames from a fixed pool,
geometric episode lengths, Discrete(9) actions.  Used for tests and for
measuring the vectorised-env machinery (MultiEnv) without a game engine.
Names: synthetic_<H>x<W> (default 72x96)."""

import re

import numpy as np

from . import gym_compat as gym


class SyntheticGymEnv(gym.Env):

  def __init__(self, height=72, width=96, num_actions=9, episode_length=100,
               frameskip=4, pool=16):
    self.observation_space = gym.spaces.Box(0, 255, (height, width, 3),
                                            dtype=np.uint8)
    self.action_space = gym.spaces.Discrete(num_actions)
    self._episode_length = episode_length
    self._frameskip = frameskip
    self._pool_n = pool
    self._rng = np.random.RandomState(0)
    self._pool = None
    self._t = 0

  def seed(self, seed=None):
    self._rng = np.random.RandomState(0 if seed is None else seed)
    self._pool = None
    return [seed]

  def _frame(self):
    if self._pool is None:
      self._pool = self._rng.randint(
          0, 256, (self._pool_n,) + self.observation_space.shape,
          dtype=np.uint8)
    return self._pool[self._rng.randint(self._pool_n)]

  def reset(self):
    self._t = 0
    return self._frame()

  def step(self, action):
    assert self.action_space.contains(action), action
    self._t += 1
    reward = float(self._rng.rand() < 0.05)
    done = self._t >= self._episode_length or self._rng.rand() < 0.005
    return self._frame(), reward, done, {'num_frames': self._frameskip}


def make_synthetic_gym_env(env_name, cfg=None, **kwargs):
  del kwargs
  m = re.match(r'synthetic_(\d+)x(\d+)', env_name)
  h, w = (int(m.group(1)), int(m.group(2))) if m else (72, 96)
  skip = getattr(cfg, 'env_frameskip', None) if cfg is not None else None
  return SyntheticGymEnv(h, w, frameskip=skip or 4)
