"""Gym env wrappers (reference envs/env_wrappers.py:20-497).

Same wrapper set and semantics (old 4-tuple step API); frame resizing and
grayscale conversion run in the native image ops (`runtime._native
.resize_u8 / rgb_to_gray`, csrc/envpool/image_ops.cc) instead of OpenCV,
and episode frames are recorded with the built-in PNG encoder.
"""

import datetime
import json
import os
from collections import deque
from os.path import join

import numpy as np

from . import gym_compat as gym
from .gym_compat import spaces
from ..algo.algo_utils import num_env_steps
from ..utils.png import write_png
from ..utils.utils import ensure_dir_exists, log, numpy_all_the_way

INTER_NEAREST, INTER_AREA, INTER_LINEAR = 0, 1, 2


def resize(img, w, h, interpolation=INTER_NEAREST):
  from ..runtime import native
  return native.resize_u8(img, h, w, interpolation)


def rgb_to_gray(img):
  from ..runtime import native
  return native.rgb_to_gray(img)


def reset_with_info(env):
  """reset() plus the info of the first frame when the env provides it."""
  obs = env.reset()
  info = {}
  if hasattr(env.unwrapped, 'get_info_all'):
    info = env.unwrapped.get_info_all()
  return obs, info


def unwrap_env(wrapped_env):
  return wrapped_env.unwrapped


def is_goal_based_env(env):
  if not isinstance(env.observation_space, spaces.Dict):
    return False
  return all(k in env.observation_space.spaces for k in ('obs', 'goal'))


def main_observation_space(env):
  if hasattr(env.observation_space, 'spaces'):
    return env.observation_space.spaces['obs']
  return env.observation_space


def has_image_observations(observation_space):
  """Heuristic: rank >= 2 observations are images."""
  return len(observation_space.shape) >= 2


class StackFramesWrapper(gym.Wrapper):
  """Stacks the last N observations (vectors, or 2D single-channel images
  along a new channel axis, HWC or CHW)."""

  def __init__(self, env, stack_past_frames, channel_config='HWC'):
    super().__init__(env)
    shape = env.observation_space.shape
    if len(shape) not in (1, 2):
      raise Exception('Stack frames works with vector observations and 2D '
                      'single channel images')
    self._stack_past = stack_past_frames
    self._frames = None
    self._image_obs = has_image_observations(env.observation_space)
    self.channel_config = channel_config
    if self._image_obs:
      if channel_config == 'CHW':
        new_shape = (stack_past_frames,) + tuple(shape)
      elif channel_config == 'HWC':
        new_shape = tuple(shape) + (stack_past_frames,)
      else:
        raise Exception('Unknown channel config %s' % channel_config)
    else:
      new_shape = (shape[0] * stack_past_frames,) + tuple(shape[1:])
    self.observation_space = spaces.Box(
        env.observation_space.low.flat[0], env.observation_space.high.flat[0],
        shape=new_shape, dtype=env.observation_space.dtype)

  def _render_stacked_frames(self):
    if not self._image_obs:
      return np.array(self._frames).flatten()
    img = numpy_all_the_way(self._frames)
    if self.channel_config == 'CHW':
      return img
    return np.transpose(img, (1, 2, 0))

  def reset(self):
    observation = self.env.reset()
    self._frames = deque([observation] * self._stack_past)
    return self._render_stacked_frames()

  def step(self, action):
    obs, reward, done, info = self.env.step(action)
    self._frames.popleft()
    self._frames.append(obs)
    return self._render_stacked_frames(), reward, done, info


class SkipFramesWrapper(gym.Wrapper):
  """Action repeat: the same action for up to N frames (stops at done)."""

  def __init__(self, env, skip_frames=4):
    super().__init__(env)
    self._skip_frames = skip_frames

  def reset(self):
    return self.env.reset()

  def step(self, action):
    total_reward, num_frames = 0, 0
    obs, done, info = None, False, None
    for _ in range(self._skip_frames):
      obs, reward, done, info = self.env.step(action)
      num_frames += 1
      total_reward += reward
      if done:
        break
    info['num_frames'] = num_frames
    return obs, total_reward, done, info


class SkipAndStackFramesWrapper(StackFramesWrapper):
  """Action repeat where every intermediate frame enters the stack."""

  def __init__(self, env, skip_frames=4, stack_frames=4, channel_config='HWC'):
    super().__init__(env, stack_past_frames=stack_frames,
                     channel_config=channel_config)
    self._skip_frames = skip_frames

  def step(self, action):
    total_reward, num_frames = 0, 0
    done, info = False, {}
    for _ in range(self._skip_frames):
      obs, reward, done, info = self.env.step(action)
      num_frames += 1
      total_reward += reward
      self._frames.popleft()
      self._frames.append(obs)
      if done:
        break
    info['num_frames'] = num_frames
    return self._render_stacked_frames(), total_reward, done, info


class NormalizeWrapper(gym.Wrapper):
  """Maps a low-dimensional Box observation to [-1, 1]."""

  def __init__(self, env):
    super().__init__(env)
    if len(env.observation_space.shape) != 1:
      raise Exception('NormalizeWrapper only works with lowdimensional envs')
    self.wrapped_env = env
    self._normalize_to = 1.0
    self._mean = (env.observation_space.high + env.observation_space.low) * .5
    self._max = env.observation_space.high
    self.observation_space = spaces.Box(
        -self._normalize_to, self._normalize_to,
        shape=env.observation_space.shape, dtype=np.float32)

  def _normalize(self, obs):
    obs = obs - self._mean
    obs *= self._normalize_to / (self._max - self._mean)
    return obs

  def reset(self):
    return self._normalize(self.env.reset())

  def step(self, action):
    obs, reward, done, info = self.env.step(action)
    return self._normalize(obs), reward, done, info

  @property
  def range(self):
    return [-self._normalize_to, self._normalize_to]


class ResizeWrapper(gym.Wrapper):
  """Resizes frames to (w, h), optionally to grayscale (+ channel dim)."""

  def __init__(self, env, w, h, grayscale=True, add_channel_dim=False,
               area_interpolation=False):
    super().__init__(env)
    self.w, self.h = w, h
    self.grayscale = grayscale
    self.add_channel_dim = add_channel_dim
    self.interpolation = INTER_AREA if area_interpolation else INTER_NEAREST
    if isinstance(env.observation_space, spaces.Dict):
      self.observation_space = spaces.Dict({
          k: self._calc_new_obs_space(s)
          for k, s in env.observation_space.spaces.items()})
    else:
      self.observation_space = self._calc_new_obs_space(env.observation_space)

  def _calc_new_obs_space(self, old_space):
    low, high = old_space.low.flat[0], old_space.high.flat[0]
    if self.grayscale:
      shape = [self.h, self.w, 1] if self.add_channel_dim else [self.h, self.w]
    else:
      shape = [self.h, self.w, old_space.shape[-1]]
    return spaces.Box(low, high, shape=shape, dtype=old_space.dtype)

  def _convert_obs(self, obs):
    if obs is None:
      return obs
    obs = resize(obs, self.w, self.h, self.interpolation)
    if self.grayscale and obs.ndim == 3:
      obs = rgb_to_gray(obs)
    return obs[:, :, None] if self.add_channel_dim else obs

  def _observation(self, obs):
    if isinstance(obs, dict):
      return {k: self._convert_obs(v) for k, v in obs.items()}
    return self._convert_obs(obs)

  def reset(self):
    return self._observation(self.env.reset())

  def step(self, action):
    obs, reward, done, info = self.env.step(action)
    return self._observation(obs), reward, done, info


class VerticalCropWrapper(gym.ObservationWrapper):
  """Keeps the central `crop_h` rows."""

  def __init__(self, env, crop_h):
    super().__init__(env)
    self.crop_h = crop_h
    old = env.observation_space
    h, w, c = old.shape
    self.observation_space = spaces.Box(old.low.flat[0], old.high.flat[0],
                                        shape=[crop_h, w, c], dtype=old.dtype)

  def observation(self, observation):
    h = observation.shape[0]
    top = (h - self.crop_h) // 2
    return observation[top:top + self.crop_h, :, :]


class RewardScalingWrapper(gym.RewardWrapper):

  def __init__(self, env, scaling_factor):
    super().__init__(env)
    self._scaling = scaling_factor
    lo, hi = env.reward_range
    self.reward_range = (lo * scaling_factor, hi * scaling_factor)

  def reward(self, reward):
    return reward * self._scaling


class TimeLimitWrapper(gym.Wrapper):
  """Ends the episode after `limit` (+- random variation) env frames."""

  terminated_by_timer = 'terminated_by_timer'

  def __init__(self, env, limit, random_variation_steps=0):
    super().__init__(env)
    self._limit = limit
    self._variation_steps = random_variation_steps
    self._num_steps = 0
    self._terminate_in = self._random_limit()

  def _random_limit(self):
    return np.random.randint(-self._variation_steps,
                             self._variation_steps + 1) + self._limit

  def reset(self):
    self._num_steps = 0
    self._terminate_in = self._random_limit()
    return self.env.reset()

  def step(self, action):
    obs, reward, done, info = self.env.step(action)
    if obs is None:
      return obs, reward, done, info
    self._num_steps += num_env_steps([info])
    if not done and self._num_steps >= self._terminate_in:
      done = True
      info[self.terminated_by_timer] = True
    return obs, reward, done, info


class RemainingTimeWrapper(gym.ObservationWrapper):
  """Adds {'timer': fraction of the time limit used} (needs TimeLimit)."""

  def __init__(self, env):
    super().__init__(env)
    self.observation_space = spaces.Dict({
        'timer': spaces.Box(0.0, 1.0, shape=[1], dtype=np.float32),
        'obs': env.observation_space,
    })
    inner = env
    while not isinstance(inner, TimeLimitWrapper):
      inner = getattr(inner, 'env', None)
      if not isinstance(inner, gym.Wrapper):
        raise Exception('RemainingTimeWrapper is supposed to wrap '
                        'TimeLimitWrapper')
    self.time_limit_wrapper = inner

  def observation(self, observation):
    tl = self.time_limit_wrapper
    return {'timer': tl._num_steps / tl._terminate_in, 'obs': observation}


class PixelFormatChwWrapper(gym.ObservationWrapper):
  """HWC -> CHW image observations (also inside a Dict under 'obs')."""

  def __init__(self, env):
    super().__init__(env)
    if isinstance(env.observation_space, spaces.Dict):
      img_space = env.observation_space['obs']
      self.dict_obs_space = True
    else:
      img_space = env.observation_space
      self.dict_obs_space = False
    if not has_image_observations(img_space):
      raise Exception('Pixel format wrapper only works with image-based envs')
    shape = img_space.shape
    if len(shape) <= 2:
      raise Exception('Env obs do not have channel dimension?')
    if shape[0] <= 4:
      raise Exception('Env obs already in CHW format?')
    h, w, c = shape
    dtype = img_space.dtype if img_space.dtype is not None else np.float32
    new_space = spaces.Box(img_space.low.flat[0], img_space.high.flat[0],
                           shape=[c, h, w], dtype=dtype)
    if self.dict_obs_space:
      d = dict(env.observation_space.spaces)
      d['obs'] = new_space
      self.observation_space = spaces.Dict(d)
    else:
      self.observation_space = new_space
    self.action_space = env.action_space

  @staticmethod
  def _transpose(obs):
    return np.transpose(obs, (2, 0, 1))

  def observation(self, observation):
    if observation is None:
      return observation
    if self.dict_obs_space:
      observation = dict(observation)
      observation['obs'] = self._transpose(observation['obs'])
      return observation
    return self._transpose(observation)


class ClipRewardWrapper(gym.RewardWrapper):
  """Clips rewards to [-0.1, 5]."""

  def reward(self, reward):
    return max(-0.1, min(5.0, reward))


class RecordingWrapper(gym.Wrapper):
  """Records every episode as PNG frames + actions.json into
  <record_to>/<timestamp>/ep_XXX_p<player>_r<reward>/."""

  def __init__(self, env, record_to, player_id=0):
    super().__init__(env)
    stamp = datetime.datetime.now().strftime('%Y_%m_%d--%H_%M_%S')
    self._record_to = join(record_to, stamp)
    self._episode_recording_dir = None
    self._record_id = 0
    self._frame_id = 0
    self._player_id = player_id
    self._recorded_episode_reward = 0
    self._recorded_episode_shaping_reward = 0
    self._recorded_actions = []

  def _finish_episode(self):
    with open(join(self._episode_recording_dir, 'actions.json'), 'w') as f:
      json.dump(self._recorded_actions, f)
    reward = (self._recorded_episode_reward +
              self._recorded_episode_shaping_reward)
    new_dir = self._episode_recording_dir + '_r%.2f' % reward
    os.rename(self._episode_recording_dir, new_dir)
    log.info('Finished recording %s (rew %.3f, shaping %.3f)', new_dir, reward,
             self._recorded_episode_shaping_reward)
    self._episode_recording_dir = None

  def reset(self):
    if self._episode_recording_dir is not None and self._record_id > 0:
      self._finish_episode()
    name = 'ep_%03d_p%s' % (self._record_id, self._player_id)
    self._episode_recording_dir = ensure_dir_exists(join(self._record_to,
                                                         name))
    self._record_id += 1
    self._frame_id = 0
    self._recorded_episode_reward = 0
    self._recorded_episode_shaping_reward = 0
    self._recorded_actions = []
    return self.env.reset()

  def _record(self, img):
    img = img['obs'] if isinstance(img, dict) else img
    if img is None:
      return
    if img.ndim == 3 and img.shape[0] <= 4 and img.shape[-1] > 4:
      img = np.transpose(img, (1, 2, 0))
    write_png(join(self._episode_recording_dir, '%05d.png' % self._frame_id),
              img)
    self._frame_id += 1

  def step(self, action):
    obs, reward, done, info = self.env.step(action)
    if isinstance(action, np.ndarray):
      self._recorded_actions.append(action.tolist())
    elif isinstance(action, np.integer):
      self._recorded_actions.append(int(action))
    elif isinstance(action, tuple):
      self._recorded_actions.append([int(a) if isinstance(a, np.integer)
                                     else a for a in action])
    else:
      self._recorded_actions.append(action)
    self._record(obs)
    self._recorded_episode_reward += reward
    if hasattr(self.env.unwrapped, '_total_shaping_reward'):
      self._recorded_episode_shaping_reward = \
          self.env.unwrapped._total_shaping_reward
    return obs, reward, done, info

  def close(self):
    if self._episode_recording_dir is not None and self._frame_id > 0:
      self._finish_episode()
    return self.env.close()
