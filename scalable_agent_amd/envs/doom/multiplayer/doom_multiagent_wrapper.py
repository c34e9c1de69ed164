"""Several Doom players as one multi-agent env (reference
envs/doom/multiplayer/doom_multiagent_wrapper.py:37-389).

  * `MultiAgentEnvWorker` owns one player's game instance on a thread (or a
    process) and serves INIT / RESET / STEP / STEP_UPDATE / INFO / SET_ATTR /
    TERMINATE tasks;
  * `MultiAgentEnv` fans every call out to all players: ViZDoom multiplayer
    must advance all instances in lockstep, so frame skipping is done here
    (skip-1 STEP tasks without state, then one STEP_UPDATE), and the match is
    reset when every agent is done; initialisation retries with fresh ports;
  * `MultiAgentEnvAggregator` vectorises several multi-agent envs on top of
    `MultiEnv`, flattening agents so every agent looks like one env;
  * UDP ports: DEFAULT_UDP_PORT + 100 * worker_index + vector_index, bumped by
    1000 until free.
"""

import enum
import multiprocessing
import queue
import threading
import time

from ...gym_compat import Env
from ....algo.multi_env import MsgType, MultiEnv
from ....utils.utils import kill, log
from . import doom_multiagent as dma

_CTX = multiprocessing.get_context('fork')


def safe_get(q, timeout=1e6, msg='Queue timeout'):
  while True:
    try:
      return q.get(timeout=timeout)
    except queue.Empty:
      log.warning(msg)


def udp_port_num(env_config):
  if env_config is None:
    return dma.DEFAULT_UDP_PORT
  return (dma.DEFAULT_UDP_PORT + 100 * env_config.worker_index +
          env_config.vector_index)


class _WorkerError(RuntimeError):
  pass


class TaskType(enum.Enum):
  INIT, TERMINATE, RESET, STEP, STEP_UPDATE, INFO, SET_ATTR = range(7)


def init_multiplayer_env(make_env_func, player_id, env_config, init_info=None):
  env = make_env_func(player_id=player_id)
  u = env.unwrapped
  if env_config is not None and 'worker_index' in env_config:
    u.worker_index = env_config.worker_index
  if env_config is not None and 'vector_index' in env_config:
    u.vector_index = env_config.vector_index
  if init_info is None:
    port = dma.find_available_port(udp_port_num(env_config), increment=1000)
    log.debug('Using port %d', port)
    init_info = dict(port=port)
  u.init_info = init_info
  env.seed(u.worker_index * 1000 + u.vector_index * 10 + player_id)
  return env


class MultiAgentEnvWorker(object):

  def __init__(self, player_id, make_env_func, env_config,
               use_multiprocessing=False):
    self.player_id = player_id
    self.make_env_func = make_env_func
    self.env_config = env_config
    if use_multiprocessing:
      self.task_queue, self.result_queue = _CTX.Queue(), _CTX.Queue()
      self.process = _CTX.Process(target=self.start, daemon=True)
    else:
      self.task_queue, self.result_queue = queue.Queue(), queue.Queue()
      self.process = threading.Thread(target=self.start, daemon=True)
    self.process.start()

  def _init(self, init_info):
    log.info('Initializing env for player %d, init_info: %r...',
             self.player_id, init_info)
    env = init_multiplayer_env(self.make_env_func, self.player_id,
                               self.env_config, init_info)
    env.reset()
    return env

  @staticmethod
  def _get_info(env):
    u = env.unwrapped
    return u.get_info_all() if hasattr(u, 'get_info_all') else {}

  def _set_env_attr(self, env, player_id, attr_chain, value):
    """attr_chain like 'unwrapped.foo.bar'."""
    assert player_id == self.player_id
    names = attr_chain.split('.')
    obj = env
    try:
      for n in names[:-1]:
        obj = getattr(obj, n)
    except AttributeError:
      log.error('Env does not have an attribute %s', attr_chain)
    setattr(obj, names[-1], value)

  def start(self):
    env = None
    while True:
      data, task = safe_get(self.task_queue)
      if task == TaskType.INIT:
        try:
          env = self._init(data)
          self.result_queue.put(None)
        except Exception as e:  # pylint: disable=broad-except
          log.warning('player %d init failed: %r', self.player_id, e)
          self.result_queue.put(e)
        continue
      if task == TaskType.TERMINATE:
        if env is not None:
          env.close()
        break
      results = None
      try:
        if task == TaskType.RESET:
          results = env.reset()
        elif task == TaskType.INFO:
          results = self._get_info(env)
        elif task in (TaskType.STEP, TaskType.STEP_UPDATE):
          env.unwrapped.update_state = task == TaskType.STEP_UPDATE
          results = env.step(data)
        elif task == TaskType.SET_ATTR:
          self._set_env_attr(env, *data)
        else:
          raise Exception('Unknown task type %s' % task)
      except Exception as e:  # pylint: disable=broad-except
        # Ship the failure to the caller instead of dying silently (the
        # caller would otherwise wait on this player forever).
        results = _WorkerError('player %d %s failed: %r' % (
            self.player_id, task, e))
      self.result_queue.put(results)


class MultiAgentEnv(Env):

  def __init__(self, num_agents, make_env_func, env_config, skip_frames):
    self.num_agents = num_agents
    log.debug('Multi agent env, num agents: %d', num_agents)
    self.skip_frames = skip_frames
    env = make_env_func(player_id=-1)  # only to query the spaces
    self.action_space = env.action_space
    self.observation_space = env.observation_space
    self.default_reward_shaping = None
    rs = getattr(env.unwrapped, '_reward_shaping_wrapper', None)
    if rs is not None:
      self.default_reward_shaping = rs.reward_shaping_scheme
    env.close()
    self.make_env_func = make_env_func
    self.env_config = env_config
    self.workers = None
    self.enable_rendering = False
    self.last_obs = None
    self.initialized = False

  def await_tasks(self, data, task_type, timeout=None):
    """-> tuple of per-agent lists, e.g. ([obs0, obs1..], [rew0, ..], ..)."""
    if data is None:
      data = [None] * self.num_agents
    assert len(data) == self.num_agents
    for i, w in enumerate(self.workers):
      w.task_queue.put((data[i], task_type))
    result_lists = None
    for w in self.workers:
      r = safe_get(w.result_queue, 0.2 if timeout is None else timeout,
                   'Takes a surprisingly long time to process task %s, '
                   'retry...' % task_type)
      if isinstance(r, _WorkerError):
        raise r
      if not isinstance(r, (tuple, list)):
        r = [r]
      if result_lists is None:
        result_lists = tuple([] for _ in r)
      for j, v in enumerate(r):
        result_lists[j].append(v)
    return result_lists

  def _ensure_initialized(self):
    if self.initialized:
      return
    attempts = 25
    for attempt in range(attempts):
      self.workers = [MultiAgentEnvWorker(i, self.make_env_func,
                                          self.env_config)
                      for i in range(self.num_agents)]
      try:
        port = dma.find_available_port(udp_port_num(self.env_config), 1000)
        init_info = dict(port=port)
        for w in self.workers:
          w.task_queue.put((init_info, TaskType.INIT))
          time.sleep(0.01)
        for w in self.workers:
          r = w.result_queue.get(timeout=5)
          if isinstance(r, Exception):
            raise r
      except Exception as exc:  # pylint: disable=broad-except
        for w in self.workers:
          if isinstance(w.process, threading.Thread):
            raise RuntimeError('Critical error: worker stuck on '
                               'initialization. Abort!') from exc
          kill(w.process.pid)
        self.workers = None
        log.warning('Could not initialize env, try again! Error: %r', exc)
        time.sleep(1)
      else:
        break
    else:
      raise RuntimeError('Critical error: worker stuck on initialization, '
                         'num attempts exceeded. Abort!')
    log.debug('%d agent workers initialized! (%d attempts)',
              len(self.workers), attempt + 1)
    self.initialized = True

  def info(self):
    self._ensure_initialized()
    return self.await_tasks(None, TaskType.INFO)[0]

  def reset(self):
    self._ensure_initialized()
    return self.await_tasks(None, TaskType.RESET, timeout=2.0)[0]

  def step(self, actions):
    self._ensure_initialized()
    for _ in range(self.skip_frames - 1):
      self.await_tasks(actions, TaskType.STEP)
    obs, rew, dones, infos = self.await_tasks(actions, TaskType.STEP_UPDATE)
    for info in infos:
      info['num_frames'] = self.skip_frames
    if all(dones):
      obs = self.await_tasks(None, TaskType.RESET, timeout=2.0)[0]
    if self.enable_rendering:
      self.last_obs = obs
    return obs, rew, dones, infos

  def render(self, *args, **kwargs):
    self.enable_rendering = True
    if self.last_obs is None:
      return None
    from ..doom_render import concat_grid, show_image  # pylint: disable=import-outside-toplevel
    grid = concat_grid([o['obs'] if isinstance(o, dict) else o
                        for o in self.last_obs])
    show_image('vizdoom', grid)
    return grid

  def close(self):
    if self.workers is not None:
      for w in self.workers:
        w.task_queue.put((None, TaskType.TERMINATE))
      for w in self.workers:
        w.process.join(timeout=10)

  def seed(self, seed=None):
    """Players are seeded individually on init."""
    return []

  def set_env_attr(self, agent_idx, attr_chain, value):
    w = self.workers[agent_idx]
    w.task_queue.put(((agent_idx, attr_chain, value), TaskType.SET_ATTR))
    assert safe_get(w.result_queue, timeout=0.1) is None


class MultiAgentEnvAggregator(MultiEnv):
  """Vectorised multi-agent envs where every agent shares one policy: agent
  j of env i is actor i * num_agents + j."""

  def __init__(self, num_envs, num_workers, make_env_func, stats_episodes,
               use_multiprocessing=True):
    tmp = make_env_func(None)
    if not hasattr(tmp, 'num_agents'):
      raise Exception('Expected multi-agent environment')
    self.num_agents = tmp.num_agents
    tmp.close()
    dma.DEFAULT_UDP_PORT = dma.find_available_port(dma.DEFAULT_UDP_PORT)
    log.debug('Default UDP port changed to %r', dma.DEFAULT_UDP_PORT)
    super().__init__(num_envs, num_workers, make_env_func, stats_episodes,
                     use_multiprocessing)

  def _num_actors(self):
    return self.num_envs * self.num_agents

  def _preprocess_data(self, data):
    if data is None:
      data = [None] * self.num_agents * self.num_envs
    assert len(data) == self.num_agents * self.num_envs
    per_env = [list(data[i * self.num_agents:(i + 1) * self.num_agents])
               for i in range(self.num_envs)]
    per = self.num_envs // self.num_workers
    return [per_env[w * per:(w + 1) * per] for w in range(self.num_workers)]

  def reset(self):
    per_env = self.await_tasks(None, MsgType.RESET)
    return [o for env_obs in per_env for o in env_obs]

  def step(self, actions, reset=None):
    if reset is None:
      results = self.await_tasks(actions, MsgType.STEP_REAL)
    else:
      results = self.await_tasks(list(zip(actions, reset)),
                                 MsgType.STEP_REAL_RESET)
    obs, rew, dones, infos = [], [], [], []
    for o, r, d, i in results:
      obs.extend(o)
      rew.extend(r)
      dones.extend(d)
      infos.extend(i)
    self._update_stats(rew, dones, infos)
    return obs, rew, dones, infos

