"""DeepMind Lab as a gym env (reference envs/dmlab/dmlab_utils.py):
84x84 RGB from the no-reticle player camera, 5 actions (idle, forward,
backward, look left/right), action repeat, seeded resets, and a level cache
that keeps compiled .pk3 maps under <repo>/.dmlab_cache.
`deepmind_lab` is imported lazily (not installed in this image)."""

import os
import shutil
import time
from os.path import join

import numpy as np

from .. import gym_compat as gym
from ..env_wrappers import PixelFormatChwWrapper, RecordingWrapper
from ...utils.utils import ensure_dir_exists, project_root

ACTION_SET = (
    (0, 0, 0, 0, 0, 0, 0),    # Idle
    (0, 0, 0, 1, 0, 0, 0),    # Forward
    (0, 0, 0, -1, 0, 0, 0),   # Backward
    (-20, 0, 0, 0, 0, 0, 0),  # Look Left
    (20, 0, 0, 0, 0, 0, 0),   # Look Right
)


class LevelCache(object):

  def __init__(self, cache_dir):
    self._cache_dir = cache_dir

  def fetch(self, key, pk3_path):
    path = join(self._cache_dir, key)
    if os.path.isfile(path):
      shutil.copyfile(path, pk3_path)
      return True
    return False

  def write(self, key, pk3_path):
    ensure_dir_exists(self._cache_dir)
    path = join(self._cache_dir, key)
    if not os.path.isfile(path):
      shutil.copyfile(pk3_path, path)


level_cache = LevelCache(join(project_root(), '.dmlab_cache'))


class DmlabGymEnv(gym.Env):

  def __init__(self, level, action_repeat, extra_cfg=None):
    import deepmind_lab  # pylint: disable=import-outside-toplevel
    self._width = self._height = 84
    self._main_observation = 'DEBUG.CAMERA_INTERLEAVED.PLAYER_VIEW_NO_RETICLE'
    self._action_repeat = action_repeat
    config = {'width': self._width, 'height': self._height}
    config.update(extra_cfg or {})
    self._dmlab = deepmind_lab.Lab(
        level, [self._main_observation, 'DEBUG.POS.TRANS'],
        config={k: str(v) for k, v in config.items()}, renderer='hardware',
        level_cache=level_cache)
    self._action_set = ACTION_SET
    self._action_list = np.array(ACTION_SET, dtype=np.intc)
    self._last_observation = None
    self._render_scale, self._render_fps = 5, 30
    self._last_frame = time.time()
    self.action_space = gym.spaces.Discrete(len(ACTION_SET))
    self.observation_space = gym.spaces.Box(
        0, 255, (self._height, self._width, 3), dtype=np.uint8)
    self._random_state = None
    self.seed()

  def seed(self, seed=None):
    initial = gym.seeding.hash_seed(seed) % 2 ** 32
    self._random_state = np.random.RandomState(seed=initial)
    return [initial]

  def reset(self):
    self._dmlab.reset(seed=self._random_state.randint(0, 2 ** 31 - 1))
    self._last_observation = self._dmlab.observations()[
        self._main_observation]
    return self._last_observation

  def step(self, action):
    reward = self._dmlab.step(self._action_list[action],
                              num_steps=self._action_repeat)
    done = not self._dmlab.is_running()
    if not done:
      self._last_observation = self._dmlab.observations()[
          self._main_observation]
    return self._last_observation, reward, done, {
        'num_frames': self._action_repeat}

  def render(self, mode='human'):
    if self._last_observation is None and self._dmlab.is_running():
      self._last_observation = self._dmlab.observations()[
          self._main_observation]
    if mode == 'rgb_array':
      return self._last_observation
    if mode != 'human':
      raise Exception('Rendering mode %s not supported' % mode)
    from ..doom.doom_render import show_image  # pylint: disable=import-outside-toplevel
    big = np.kron(self._last_observation,
                  np.ones((self._render_scale, self._render_scale, 1),
                          np.uint8))
    show_image('dmlab', big)
    wait = 1.0 / self._render_fps - (time.time() - self._last_frame)
    if wait > 0:
      time.sleep(wait)
    self._last_frame = time.time()
    return big

  def close(self):
    self._dmlab.close()


class DmLabSpec(object):

  def __init__(self, name, level, extra_cfg=None):
    self.name = name
    self.level = level
    self.extra_cfg = extra_cfg or {}


DMLAB_ENVS = [
    DmLabSpec('dmlab_sparse', 'contributed/dmlab30/explore_goal_locations_large'),
    DmLabSpec('dmlab_very_sparse',
              'contributed/dmlab30/explore_goal_locations_large',
              extra_cfg={'minGoalDistance': '10'}),
    DmLabSpec('dmlab_sparse_doors',
              'contributed/dmlab30/explore_obstructed_goals_large'),
    DmLabSpec('dmlab_nonmatch',
              'contributed/dmlab30/rooms_select_nonmatching_object'),
    DmLabSpec('dmlab_watermaze', 'contributed/dmlab30/rooms_watermaze'),
]


def dmlab_env_by_name(name):
  for spec in DMLAB_ENVS:
    if spec.name == name:
      return spec
  raise Exception('Unknown DMLab env')


def _cfg(cfg, key, default=None):
  if isinstance(cfg, dict):
    return cfg.get(key, default)
  return getattr(cfg, key, default)


def make_dmlab_env_impl(spec, cfg, **kwargs):
  del kwargs
  skip = _cfg(cfg, 'env_frameskip') or 4
  env = DmlabGymEnv(spec.level, skip, spec.extra_cfg)
  if _cfg(cfg, 'record_to') is not None:
    env = RecordingWrapper(env, _cfg(cfg, 'record_to'), 0)
  if _cfg(cfg, 'pixel_format', 'CHW') == 'CHW':
    env = PixelFormatChwWrapper(env)
  return env


def make_dmlab_env(env_name, cfg=None, **kwargs):
  return make_dmlab_env_impl(dmlab_env_by_name(env_name), cfg=cfg, **kwargs)
