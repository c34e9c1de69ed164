"""Environment protocol, DeepMind Lab adapter and step bookkeeping.

Reference: environments.py:33-233.
  * `DEFAULT_ACTION_SET` (9 DMLab actions x 7-dim, :53-63);
  * `PyProcessDmLab` (:66-140): `deepmind_lab.Lab` with RGB_INTERLEAVED +
    INSTR observations, `step(action, num_steps=repeats)`, auto-reset on done,
    seeded resets, `benchmark_mode` replacing the action by a random one;
    DeepMind Lab is not installed in this image, so construction raises a
    clear ImportError (the synthetic env is the runnable stand-in);
  * `LocalLevelCache` (:33-50);
  * `FlowEnvironment` (:143-233): initial output (reward 0, info (0,0),
    done=True), per-step episode_return / episode_step accumulation that is
    emitted with the step and reset in the carried state on done.  In eager
    Python there is no graph to serialise, so the reference's `flow` counter
    becomes a plain step counter.
"""

import os
import shutil

import numpy as np

from .structs import StepOutput, StepOutputInfo

DEFAULT_ACTION_SET = (
    (0, 0, 0, 1, 0, 0, 0),    # Forward
    (0, 0, 0, -1, 0, 0, 0),   # Backward
    (0, 0, -1, 0, 0, 0, 0),   # Strafe Left
    (0, 0, 1, 0, 0, 0, 0),    # Strafe Right
    (-20, 0, 0, 0, 0, 0, 0),  # Look Left
    (20, 0, 0, 0, 0, 0, 0),   # Look Right
    (-20, 0, 0, 1, 0, 0, 0),  # Look Left + Forward
    (20, 0, 0, 1, 0, 0, 0),   # Look Right + Forward
    (0, 0, 0, 0, 1, 0, 0),    # Fire.
)


class LocalLevelCache(object):
  """Local level cache (DMLab level_cache protocol)."""

  def __init__(self, cache_dir='/tmp/level_cache'):
    self._cache_dir = cache_dir
    os.makedirs(cache_dir, exist_ok=True)

  def fetch(self, key, pk3_path):
    path = os.path.join(self._cache_dir, key)
    if os.path.exists(path):
      shutil.copyfile(path, pk3_path)
      return True
    return False

  def write(self, key, pk3_path):
    path = os.path.join(self._cache_dir, key)
    if not os.path.exists(path):
      shutil.copyfile(pk3_path, path)


class PyProcessDmLab(object):
  """DeepMind Lab wrapper (run inside an EnvProcess / PyProcess)."""

  def __init__(self, level, config, num_action_repeats, seed,
               runfiles_path=None, level_cache=None):
    try:
      import deepmind_lab  # pylint: disable=g-import-not-at-top
    except ImportError as e:
      raise ImportError(
          'deepmind_lab is not installed; use --env=synthetic (or install '
          'DeepMind Lab) to run level %r' % level) from e
    self._num_action_repeats = num_action_repeats
    self._random_state = np.random.RandomState(seed=seed)
    if runfiles_path:
      deepmind_lab.set_runfiles_path(runfiles_path)
    config = {k: str(v) for k, v in config.items()}
    self._observation_spec = ['RGB_INTERLEAVED', 'INSTR']
    renderer = config.get('renderer', 'software')
    self.benchmark_mode = int(config.get('benchmark_mode', '0'))
    self._env = deepmind_lab.Lab(level=level,
                                 observations=self._observation_spec,
                                 config=config, level_cache=level_cache,
                                 renderer=renderer)

  def _reset(self):
    self._env.reset(seed=self._random_state.randint(0, 2 ** 31 - 1))

  def _observation(self):
    d = self._env.observations()
    return [d[k] for k in self._observation_spec]

  def initial(self):
    self._reset()
    return self._observation()

  def step(self, action):
    if self.benchmark_mode:
      # throughput measurement: ignore the policy, act randomly
      a = self._random_state.randint(0, len(DEFAULT_ACTION_SET))
      action = np.array(DEFAULT_ACTION_SET[a], dtype=np.intc)
    reward = self._env.step(np.asarray(action, dtype=np.intc),
                            num_steps=self._num_action_repeats)
    done = np.array(not self._env.is_running())
    if done:
      self._reset()
    observation = self._observation()
    return np.array(reward, dtype=np.float32), done, observation

  def close(self):
    self._env.close()


class FlowEnvironment(object):
  """Adds the reference's step bookkeeping on top of a raw env.

  `env` exposes `initial() -> observation` and `step(action) -> (reward, done,
  observation)`, where a done step's observation is the first of the next
  episode (environments.py:159-169).
  """

  def __init__(self, env):
    self._env = env

  def initial(self):
    initial_info = StepOutputInfo(np.float32(0.), np.int32(0))
    observation = self._env.initial()
    output = StepOutput(np.float32(0.), initial_info, np.bool_(True),
                        observation)
    return output, initial_info

  def step(self, action, state):
    reward, done, observation = self._env.step(action)
    new_info = StepOutputInfo(np.float32(state.episode_return + reward),
                              np.int32(state.episode_step + 1))
    new_state = (StepOutputInfo(np.float32(0.), np.int32(0)) if done
                 else new_info)
    output = StepOutput(np.float32(reward), new_info, np.bool_(done),
                        observation)
    return output, new_state

  def close(self):
    if hasattr(self._env, 'close'):
      self._env.close()
