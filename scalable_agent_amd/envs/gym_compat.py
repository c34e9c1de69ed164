"""Minimal gym-API core: spaces, Env and the Wrapper family.

The reference's env stack (envs/env_wrappers.py, envs/doom/*, algorithms/*)
is written against OpenAI gym (old 4-tuple `step` API).  gym is not part of
this image, so when it is importable its classes are re-exported (so
isinstance checks interoperate with third-party envs); otherwise the small
self-contained implementation below provides the same surface:

  spaces.Discrete / Box / Tuple / Dict / MultiDiscrete (sample, contains,
  seed, shape, dtype), Env (reset/step/render/close/seed, unwrapped),
  Wrapper (attribute forwarding), ObservationWrapper, RewardWrapper,
  ActionWrapper, error.Error and utils.seeding.{np_random, hash_seed}.
"""

import hashlib

import numpy as np

try:  # pragma: no cover - gym is not installed in this image
  import gym as _gym
  HAVE_GYM = True
except ImportError:
  _gym = None
  HAVE_GYM = False


# ----------------------------------------------------------------------------
# seeding (gym.utils.seeding semantics: hash_seed -> 8-byte sha512 prefix)

class seeding(object):  # pylint: disable=invalid-name

  @staticmethod
  def hash_seed(seed=None, max_bytes=8):
    if seed is None:
      seed = int.from_bytes(np.random.bytes(max_bytes), 'little')
    digest = hashlib.sha512(str(seed).encode('utf8')).digest()
    return int.from_bytes(digest[:max_bytes], 'little')

  @staticmethod
  def np_random(seed=None):
    if seed is not None and not (isinstance(seed, (int, np.integer))
                                 and seed >= 0):
      raise ValueError('Seed must be a non-negative integer or omitted, '
                       'not %r' % (seed,))
    seed = seeding.hash_seed(seed, max_bytes=4) if seed is None else seed
    rng = np.random.RandomState()
    rng.seed(int(seed) % (2 ** 32))
    return rng, seed


class Error(Exception):
  pass


class error(object):  # pylint: disable=invalid-name
  Error = Error


# ----------------------------------------------------------------------------
# spaces

class Space(object):

  def __init__(self, shape=None, dtype=None):
    self.shape = None if shape is None else tuple(shape)
    self.dtype = None if dtype is None else np.dtype(dtype)
    self.np_random = None
    self.seed()

  def seed(self, seed=None):
    self.np_random, seed = seeding.np_random(seed)
    return [seed]

  def sample(self):
    raise NotImplementedError

  def contains(self, x):
    raise NotImplementedError

  def __contains__(self, x):
    return self.contains(x)


class Discrete(Space):

  def __init__(self, n):
    assert n >= 0
    self.n = int(n)
    super().__init__((), np.int64)

  def sample(self):
    return int(self.np_random.randint(self.n))

  def contains(self, x):
    if isinstance(x, (int, np.integer)):
      v = int(x)
    elif isinstance(x, np.ndarray) and x.shape == () and \
        x.dtype.kind in 'iu':
      v = int(x)
    else:
      return False
    return 0 <= v < self.n

  def __repr__(self):
    return 'Discrete(%d)' % self.n

  def __eq__(self, other):
    return isinstance(other, Discrete) and other.n == self.n

  __hash__ = Space.__hash__


class Box(Space):

  def __init__(self, low, high, shape=None, dtype=np.float32):
    dtype = np.dtype(dtype)
    if shape is None:
      low = np.asarray(low)
      shape = low.shape
    shape = tuple(int(s) for s in shape)
    self.low = np.broadcast_to(np.asarray(low, dtype=dtype), shape).copy()
    self.high = np.broadcast_to(np.asarray(high, dtype=dtype), shape).copy()
    super().__init__(shape, dtype)

  def sample(self):
    if self.dtype.kind in 'iu':
      return self.np_random.randint(
          self.low.astype(np.int64), self.high.astype(np.int64) + 1,
          size=self.shape).astype(self.dtype)
    lo = np.where(np.isfinite(self.low), self.low, -1e6)
    hi = np.where(np.isfinite(self.high), self.high, 1e6)
    return self.np_random.uniform(lo, hi, size=self.shape).astype(self.dtype)

  def contains(self, x):
    x = np.asarray(x)
    return (x.shape == self.shape and bool(np.all(x >= self.low))
            and bool(np.all(x <= self.high)))

  def __repr__(self):
    return 'Box(%s, %s)' % (self.shape, self.dtype)

  def __eq__(self, other):
    return (isinstance(other, Box) and other.shape == self.shape
            and np.allclose(other.low, self.low)
            and np.allclose(other.high, self.high))

  __hash__ = Space.__hash__


class MultiDiscrete(Space):

  def __init__(self, nvec):
    self.nvec = np.asarray(nvec, dtype=np.int64)
    super().__init__(self.nvec.shape, np.int64)

  def sample(self):
    return (self.np_random.random_sample(self.nvec.shape)
            * self.nvec).astype(np.int64)

  def contains(self, x):
    x = np.asarray(x)
    return x.shape == self.shape and bool(np.all((x >= 0) & (x < self.nvec)))


class Tuple(Space):

  def __init__(self, spaces):
    self.spaces = tuple(spaces)
    super().__init__(None, None)

  def seed(self, seed=None):
    seeds = super().seed(seed)
    for s in getattr(self, 'spaces', ()):
      seeds += s.seed(None if seed is None else seed + len(seeds))
    return seeds

  def sample(self):
    return tuple(s.sample() for s in self.spaces)

  def contains(self, x):
    if isinstance(x, (list, np.ndarray)):
      x = tuple(x)
    return (isinstance(x, tuple) and len(x) == len(self.spaces)
            and all(s.contains(v) for s, v in zip(self.spaces, x)))

  def __getitem__(self, i):
    return self.spaces[i]

  def __len__(self):
    return len(self.spaces)

  def __repr__(self):
    return 'Tuple(%s)' % ', '.join(repr(s) for s in self.spaces)


class Dict(Space):

  def __init__(self, spaces=None, **kwargs):
    spaces = dict(spaces or {}, **kwargs)
    self.spaces = dict(spaces)
    super().__init__(None, None)

  def sample(self):
    return {k: s.sample() for k, s in self.spaces.items()}

  def contains(self, x):
    return (isinstance(x, dict) and set(x) == set(self.spaces)
            and all(self.spaces[k].contains(v) for k, v in x.items()))

  def __getitem__(self, key):
    return self.spaces[key]

  def __setitem__(self, key, value):
    self.spaces[key] = value

  def __repr__(self):
    return 'Dict(%s)' % ', '.join('%s: %r' % kv for kv in self.spaces.items())


class spaces(object):  # pylint: disable=invalid-name
  Space = Space
  Discrete = Discrete
  Box = Box
  MultiDiscrete = MultiDiscrete
  Tuple = Tuple
  Dict = Dict


# ----------------------------------------------------------------------------
# Env / wrappers

class Env(object):
  metadata = {'render.modes': []}
  reward_range = (-float('inf'), float('inf'))
  spec = None
  action_space = None
  observation_space = None

  def step(self, action):
    raise NotImplementedError

  def reset(self):
    raise NotImplementedError

  def render(self, mode='human'):
    raise NotImplementedError

  def close(self):
    pass

  def seed(self, seed=None):
    return []

  @property
  def unwrapped(self):
    return self

  def __enter__(self):
    return self

  def __exit__(self, *args):
    self.close()
    return False


class Wrapper(Env):

  def __init__(self, env):
    self.env = env
    self._action_space = None
    self._observation_space = None
    self._reward_range = None
    self._metadata = None

  def __getattr__(self, name):
    if name.startswith('_'):
      raise AttributeError(
          "attempted to get missing private attribute '%s'" % name)
    return getattr(self.env, name)

  @property
  def action_space(self):
    return self.env.action_space if self._action_space is None \
        else self._action_space

  @action_space.setter
  def action_space(self, space):
    self._action_space = space

  @property
  def observation_space(self):
    return self.env.observation_space if self._observation_space is None \
        else self._observation_space

  @observation_space.setter
  def observation_space(self, space):
    self._observation_space = space

  @property
  def reward_range(self):
    return self.env.reward_range if self._reward_range is None \
        else self._reward_range

  @reward_range.setter
  def reward_range(self, value):
    self._reward_range = value

  @property
  def metadata(self):
    return self.env.metadata if self._metadata is None else self._metadata

  @metadata.setter
  def metadata(self, value):
    self._metadata = value

  def step(self, action):
    return self.env.step(action)

  def reset(self, **kwargs):
    return self.env.reset(**kwargs)

  def render(self, mode='human', **kwargs):
    return self.env.render(mode, **kwargs)

  def close(self):
    return self.env.close()

  def seed(self, seed=None):
    return self.env.seed(seed)

  @property
  def unwrapped(self):
    return self.env.unwrapped

  def __repr__(self):
    return '<%s%r>' % (type(self).__name__, self.env)


class ObservationWrapper(Wrapper):

  def reset(self, **kwargs):
    return self.observation(self.env.reset(**kwargs))

  def step(self, action):
    obs, reward, done, info = self.env.step(action)
    return self.observation(obs), reward, done, info

  def observation(self, observation):
    raise NotImplementedError


class RewardWrapper(Wrapper):

  def step(self, action):
    obs, reward, done, info = self.env.step(action)
    return obs, self.reward(reward), done, info

  def reward(self, reward):
    raise NotImplementedError


class ActionWrapper(Wrapper):

  def step(self, action):
    return self.env.step(self.action(action))

  def action(self, action):
    raise NotImplementedError


if HAVE_GYM:  # pragma: no cover
  spaces = _gym.spaces  # noqa: F811
  Space, Discrete, Box = _gym.Space, _gym.spaces.Discrete, _gym.spaces.Box
  Tuple, Dict = _gym.spaces.Tuple, _gym.spaces.Dict
  MultiDiscrete = _gym.spaces.MultiDiscrete
  Env, Wrapper = _gym.Env, _gym.Wrapper
  ObservationWrapper = _gym.ObservationWrapper
  RewardWrapper, ActionWrapper = _gym.RewardWrapper, _gym.ActionWrapper
  error = _gym.error  # noqa: F811
  Error = _gym.error.Error

