"""Vectorised gym environments on worker processes or threads (reference
algorithms/utils/multi_env.py:42-386).

`MultiEnv(num_envs, num_workers, make_env_func, stats_episodes)` splits the
envs evenly over workers; every call fans one message out to all workers and
gathers the per-env results in env order.  Messages:

  INIT             build the worker's envs (make_env_func(AttrDict(
                   worker_index, vector_index))), seed(i), reset
  RESET / INFO     reset() / unwrapped.get_info_all() for every env
  STEP_REAL        step; envs that finish are reset in place and return the
                   new episode's first observation (and its info)
  STEP_REAL_RESET  same, with a per-env forced-reset flag
  STEP_IMAGINED    `predict`: deep copies of the real envs step through
                   candidate action lists (discarded on the next real step)
  TERMINATE        close everything

Multi-agent envs (num_agents > 1) are done when all agents are done.
Episode reward/length statistics are tracked per env on the caller side.
"""

import copy
import enum
import multiprocessing
import queue
import threading

import numpy as np

from .algo_utils import list_to_string
from ..utils.utils import AttrDict, log

_CTX = multiprocessing.get_context('fork')


class MsgType(enum.Enum):
  INIT, TERMINATE, RESET, STEP_REAL, STEP_REAL_RESET, STEP_IMAGINED, INFO = \
      range(7)


def safe_get(q, timeout=1e6, msg='Queue timeout'):
  """Blocking get that wakes periodically (keeps KeyboardInterrupt live)."""
  while True:
    try:
      return q.get(timeout=timeout)
    except queue.Empty:
      log.info('Queue timed out (%s), timeout %.3f', msg, timeout)


def empty_queue(q):
  while True:
    try:
      q.get(timeout=0.1)
    except queue.Empty:
      break


class _MultiEnvWorker(object):

  def __init__(self, env_indices, make_env_func, use_multiprocessing):
    self.env_indices = env_indices
    self.make_env_func = make_env_func
    self.is_multiagent = False
    if use_multiprocessing:
      self.task_queue, self.result_queue = _CTX.Queue(), _CTX.Queue()
      self.process = _CTX.Process(target=self.start, daemon=True)
    else:
      self.task_queue, self.result_queue = queue.Queue(), queue.Queue()
      self.process = threading.Thread(target=self.start, daemon=True)
    self.process.start()

  def _init(self, envs):
    log.info('Initializing envs %s...', list_to_string(self.env_indices))
    worker_index = self.env_indices[0] // len(self.env_indices)
    for i in self.env_indices:
      env = self.make_env_func(AttrDict(worker_index=worker_index,
                                        vector_index=i - self.env_indices[0]))
      env.seed(i)
      env.reset()
      if getattr(env, 'num_agents', 1) > 1:
        self.is_multiagent = True
      envs.append(env)

  @staticmethod
  def _get_info(env):
    if hasattr(env, 'unwrapped') and hasattr(env.unwrapped, 'get_info_all'):
      return env.unwrapped.get_info_all()
    return {}

  def _episode_done(self, done):
    return all(done) if self.is_multiagent else bool(done)

  def start(self):
    real_envs, imagined_envs = [], None
    while True:
      data, msg = safe_get(self.task_queue)
      if msg == MsgType.INIT:
        try:
          self._init(real_envs)
          self.result_queue.put(('ok', None))
        except Exception as e:  # pylint: disable=broad-except
          self.result_queue.put(('error', repr(e)))
        continue
      if msg == MsgType.TERMINATE:
        for e in real_envs + (imagined_envs or []):
          e.close()
        self.result_queue.put(('ok', None))
        break
      try:
        results = self._handle(msg, data, real_envs, imagined_envs)
        if msg == MsgType.STEP_IMAGINED:
          results, imagined_envs = results
        elif msg != MsgType.INFO:
          for e in imagined_envs or []:
            e.close()
          imagined_envs = None
        self.result_queue.put(('ok', results))
      except Exception as e:  # pylint: disable=broad-except
        self.result_queue.put(('error', repr(e)))

  def _handle(self, msg, data, real_envs, imagined_envs):
    if msg == MsgType.RESET:
      return [env.reset() for env in real_envs]
    if msg == MsgType.INFO:
      return [self._get_info(env) for env in real_envs]
    if msg == MsgType.STEP_IMAGINED:
      if imagined_envs is None:
        assert len(data) == len(real_envs)
        imagined_envs = [copy.deepcopy(real_envs[i])
                         for i in range(len(data)) for _ in data[i]]
      actions = np.asarray(data).reshape(-1)
      flat = [env.step(a) for env, a in zip(imagined_envs, actions)]
      per_env = len(flat) // len(real_envs)
      return [flat[i * per_env:(i + 1) * per_env]
              for i in range(len(real_envs))], imagined_envs
    actions, resets = data, [False] * len(real_envs)
    if msg == MsgType.STEP_REAL_RESET:
      actions, resets = zip(*data)
    assert len(actions) == len(real_envs)
    results = []
    for i, (env, a) in enumerate(zip(real_envs, actions)):
      obs, rew, done, info = env.step(a)
      # Multi-agent envs reset themselves once every agent is done.
      if (self._episode_done(done) and not self.is_multiagent) or resets[i]:
        obs = env.reset()
        if not self.is_multiagent:
          info = self._get_info(env)
      results.append((obs, rew, done, info))
    return results


class MultiEnv(object):
  """Runs gym envs in parallel with (roughly) the single-env interface."""

  def __init__(self, num_envs, num_workers, make_env_func, stats_episodes,
               use_multiprocessing=True):
    if num_workers > num_envs or num_envs % num_workers != 0:
      raise Exception('num_envs should be a multiple of num_workers')
    env = make_env_func(None)
    self.action_space = env.action_space
    self.observation_space = env.observation_space
    env.close()
    self.num_envs = num_envs
    self.num_workers = num_workers
    splits = np.split(np.arange(num_envs), num_workers)
    self.workers = [_MultiEnvWorker(s.tolist(), make_env_func,
                                    use_multiprocessing) for s in splits]
    for w in self.workers:
      w.task_queue.put((None, MsgType.INIT))
    for w in self.workers:
      status, payload = safe_get(w.result_queue, 60.0, 'env init')
      if status != 'ok':
        self.close()
        raise RuntimeError('env worker failed to initialize: %s' % payload)
    log.info('Envs initialized!')
    n = self._num_actors()
    self.curr_episode_reward = [0] * n
    self.episode_rewards = [[] for _ in range(n)]
    self.curr_episode_duration = [0] * n
    self.episode_lengths = [[] for _ in range(n)]
    self.stats_episodes = stats_episodes

  def _num_actors(self):
    return self.num_envs

  def _preprocess_data(self, data):
    if data is None:
      data = [None] * self.num_envs
    assert len(data) == self.num_envs
    per = self.num_envs // self.num_workers
    return [list(data[i * per:(i + 1) * per]) for i in range(self.num_workers)]

  def _process_results(self, task_type, timeout):
    results = []
    for w in self.workers:
      status, payload = safe_get(
          w.result_queue, timeout,
          'Takes a surprisingly long time to process task %s, retry...' %
          task_type)
      if status != 'ok':
        raise RuntimeError('env worker error in %s: %s' % (task_type, payload))
      results.extend(payload)
    return results

  def await_tasks(self, data, task_type, timeout=None):
    data = self._preprocess_data(data)
    for w, task in zip(self.workers, data):
      w.task_queue.put((task, task_type))
    if timeout is None:
      timeout = max(1.0, self._num_actors() // self.num_workers * 0.02)
    return self._process_results(task_type, timeout)

  def info(self):
    return self.await_tasks(None, MsgType.INFO)

  def reset(self):
    return self.await_tasks(None, MsgType.RESET)

  def step(self, actions, reset=None):
    """Vectors of (obs, rewards, dones, infos); call reset() first."""
    if reset is None:
      results = self.await_tasks(actions, MsgType.STEP_REAL)
    else:
      results = self.await_tasks(list(zip(actions, reset)),
                                 MsgType.STEP_REAL_RESET)
    observations, rewards, dones, infos = zip(*results)
    self._update_stats(rewards, dones, infos)
    return observations, rewards, dones, infos

  def predict(self, imagined_action_lists):
    """Steps copies of every env through candidate actions (no side effects
    on the real envs); returns per-candidate (obs, rewards, dones)."""
    assert len(imagined_action_lists) == self.num_envs
    per_worker = self._preprocess_data(imagined_action_lists)
    for w, lists in zip(self.workers, per_worker):
      w.task_queue.put((lists, MsgType.STEP_IMAGINED))
    observations, rewards, dones = [], [], []
    for w in self.workers:
      status, payload = safe_get(w.result_queue, 10.0, 'predict')
      if status != 'ok':
        raise RuntimeError('env worker error in predict: %s' % payload)
      for per_env in payload:
        o, r, d, _ = zip(*per_env)
        observations.append(o)
        rewards.append(r)
        dones.append(d)
    return observations, rewards, dones

  def close(self):
    log.info('Stopping multi env wrapper...')
    for w in self.workers:
      w.task_queue.put((None, MsgType.TERMINATE))
    for w in self.workers:
      try:
        w.result_queue.get(timeout=10)
      except queue.Empty:
        pass
      w.process.join(timeout=10)

  def _update_stats(self, rewards, dones, infos):
    for i in range(self._num_actors()):
      self.curr_episode_reward[i] += rewards[i]
      step_len = 1
      if infos[i] is not None and 'num_frames' in infos[i]:
        step_len = infos[i]['num_frames']
      self.curr_episode_duration[i] += step_len
      if dones[i]:
        self._update_episode_stats(self.episode_rewards[i],
                                   self.curr_episode_reward[i])
        self.curr_episode_reward[i] = 0
        self._update_episode_stats(self.episode_lengths[i],
                                   self.curr_episode_duration[i])
        self.curr_episode_duration[i] = 0

  def _update_episode_stats(self, episode_stats, value):
    target = 2 * (1 + self.stats_episodes // self._num_actors())
    episode_stats.append(value)
    if len(episode_stats) > target * 2:
      del episode_stats[:target]

  def _calc_episode_stats(self, episode_data, n):
    n_per_actor = 1 + n // self._num_actors()
    total, count = 0, 0
    for i in range(self._num_actors()):
      last = episode_data[i][-n_per_actor:]
      total += np.sum(last)
      count += len(last)
    if count < max(n, self._num_actors()):
      return np.nan
    return total / count

  def calc_avg_rewards(self, n):
    return self._calc_episode_stats(self.episode_rewards, n)

  def calc_avg_episode_lengths(self, n):
    return self._calc_episode_stats(self.episode_lengths, n)

  def stats_num_episodes(self):
    return sum(len(r) for r in self.episode_rewards)

