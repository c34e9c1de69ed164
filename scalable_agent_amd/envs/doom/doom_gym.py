"""Gym environment around a ViZDoom `DoomGame` (reference
envs/doom/doom_gym.py:52-562).

Behaviour kept from the reference:
  * game lifecycle: lazy `initialize()` on first reset, seeded from the env's
    RNG, PLAYER (or ASYNC_PLAYER) mode, hidden window in 'algo' mode;
  * action conversion (`_convert_actions`): every sub-space of a Tuple action
    space maps to buttons - Discrete(n) -> (n-1)-wide one-hot with 0 = no-op,
    Discretized -> one continuous delta, Box -> value x 7.5;
  * game variables are named through the scenario's variable list;
  * on episode end the observation is a black screen and info repeats the
    last frame's variables; DEATHCOUNT/HITCOUNT/DAMAGECOUNT are made
    per-episode (ViZDoom does not reset them on new_episode);
  * optional positional-coverage histogram, demo recording, human play and
    demo replay.

Backend: real `vizdoom` when importable, else (or with SA_DOOM_BACKEND=sim)
the in-tree `SimDoomGame` test double - see sim_game.py.
"""

import copy
import os
import time

import numpy as np

from .. import gym_compat as gym
from ...algo.spaces import Discretized
from ...utils.utils import log
from . import scenarios as scn

DELTA_ACTIONS_SCALING = 7.5


def doom_backend(backend=None):
  """-> module-like object exposing DoomGame, ScreenResolution, Mode,
  AutomapMode for the selected backend ('vizdoom' or 'sim')."""
  backend = backend or os.environ.get('SA_DOOM_BACKEND', 'auto')
  if backend in ('auto', 'vizdoom'):
    try:
      import vizdoom  # pylint: disable=import-outside-toplevel
      return vizdoom
    except ImportError:
      if backend == 'vizdoom':
        raise
  if backend in ('auto', 'sim'):
    if backend == 'auto':
      raise ImportError(
          'ViZDoom is not installed. Install vizdoom to run Doom '
          'environments, or set SA_DOOM_BACKEND=sim to use the in-tree '
          'simulator (a test double for the framework plumbing).')
    from . import sim_game  # pylint: disable=import-outside-toplevel

    class _Sim(object):
      DoomGame = sim_game.SimDoomGame
      ScreenResolution = sim_game.ScreenResolution
      Mode = sim_game.Mode
      AutomapMode = sim_game.AutomapMode
    return _Sim
  raise ValueError('unknown Doom backend %r' % backend)


def key_to_action_default(key):
  """Keyboard -> button index for the full 14-button layout (human play)."""
  from pynput.keyboard import Key  # pylint: disable=import-outside-toplevel
  table = {Key.up: 0, Key.down: 1, Key.alt: 6, Key.ctrl: 11, Key.shift: 12,
           Key.space: 13, Key.right: 'turn_right', Key.left: 'turn_left'}
  return table.get(key, None)


class VizdoomEnv(gym.Env):

  def __init__(self, action_space, config_file, coord_limits=None,
               max_histogram_length=200, show_automap=False, skip_frames=1,
               async_mode=False, record_to=None, backend=None):
    self.initialized = False
    self.game = None
    self.state = None
    self.curr_seed = 0
    self.rng = None
    self.skip_frames = skip_frames
    self.async_mode = async_mode
    self.show_automap = show_automap
    self.coord_limits = coord_limits
    self._backend = doom_backend(backend)

    self.screen_w, self.screen_h, self.channels = 640, 480, 3
    self.screen_resolution = self._backend.ScreenResolution.RES_640X480
    self.calc_observation_space()
    self.black_screen = None

    self.action_space = action_space
    self.composite_action_space = hasattr(action_space, 'spaces')
    self.delta_actions_scaling_factor = DELTA_ACTIONS_SCALING

    if os.path.isfile(config_file):
      self.config_path = config_file
      with open(config_file) as f:
        variables = scn.parse_cfg(f.read()).get('available_game_variables',
                                                [])
    else:
      scenario = scn.scenario_by_cfg(config_file)
      self.config_path = scenario.write_cfg()
      variables = scenario.game_variables
    self.variable_indices = {v: i for i, v in enumerate(variables)}

    self.viewer = None
    self.record_to = record_to
    self.is_multiplayer = False

    self.max_histogram_length = max_histogram_length
    self.current_histogram = self.previous_histogram = None
    if coord_limits:
      x = coord_limits[2] - coord_limits[0]
      y = coord_limits[3] - coord_limits[1]
      if x > y:
        lx, ly = max_histogram_length, int(y / x * max_histogram_length)
      else:
        lx, ly = int(x / y * max_histogram_length), max_histogram_length
      self.current_histogram = np.zeros((lx, ly), np.int32)
      self.previous_histogram = np.zeros_like(self.current_histogram)

    self._terminate = False
    self._current_actions = []
    self._actions_flattened = None
    self._prev_info = None
    self._last_episode_info = None
    self._num_episodes = 0
    self.mode = 'algo'
    self.seed()

  # -- setup -----------------------------------------------------------------
  def seed(self, seed=None):
    self.curr_seed = gym.seeding.hash_seed(seed, max_bytes=4)
    self.rng, _ = gym.seeding.np_random(seed=self.curr_seed)
    return [self.curr_seed, self.rng]

  def calc_observation_space(self):
    self.observation_space = gym.spaces.Box(
        0, 255, (self.screen_h, self.screen_w, self.channels), dtype=np.uint8)

  def _set_game_mode(self, mode):
    modes = self._backend.Mode
    if mode != 'replay' and self.async_mode:
      log.info('Starting in async mode! Use this only for testing, otherwise '
               'PLAYER mode is much faster')
      self.game.set_mode(modes.ASYNC_PLAYER)
    else:
      self.game.set_mode(modes.PLAYER)

  def _create_doom_game(self, mode):
    self.game = self._backend.DoomGame()
    self.game.load_config(self.config_path)
    self.game.set_screen_resolution(self.screen_resolution)
    self.game.set_seed(self.rng.randint(0, 2 ** 32 - 1))
    if mode == 'algo':
      self.game.set_window_visible(False)
    elif mode in ('human', 'replay'):
      self.game.add_game_args('+freelook 1')
      self.game.set_window_visible(True)
    else:
      raise Exception('Unsupported mode')
    self._set_game_mode(mode)

  def initialize(self):
    self._create_doom_game(self.mode)
    if self.show_automap:
      g = self.game
      g.set_automap_buffer_enabled(True)
      g.set_automap_mode(self._backend.AutomapMode.OBJECTS)
      g.set_automap_rotate(False)
      g.set_automap_render_textures(False)
      bg = 'ffffff'
      for arg in ('+viz_am_center 1', '+am_backcolor ' + bg,
                  '+am_tswallcolor dddddd', '+am_yourcolor ' + bg,
                  '+am_cheat 0', '+am_thingcolor 0000ff',
                  '+am_thingcolor_item 00ff00'):
        g.add_game_args(arg)
    self.game.init()
    self.initialized = True

  def _ensure_initialized(self):
    if not self.initialized:
      self.initialize()

  def _black_screen(self):
    if self.black_screen is None or \
        self.black_screen.shape != self.observation_space.shape:
      self.black_screen = np.zeros(self.observation_space.shape, np.uint8)
    return self.black_screen

  def _game_variables_dict(self, state):
    gv = state.game_variables
    return {name: gv[i] for name, i in self.variable_indices.items()}

  def demo_path(self, episode_idx):
    return os.path.normpath(os.path.join(self.record_to,
                                         'ep_%03d_rec.lmp' % episode_idx))

  # -- gym API ---------------------------------------------------------------
  def reset(self):
    self._ensure_initialized()
    if self.record_to is not None and not self.is_multiplayer:
      os.makedirs(self.record_to, exist_ok=True)
      path = self.demo_path(self._num_episodes)
      log.warning('Recording episode demo to %s', path)
      self.game.new_episode(path)
    else:
      self.game.new_episode()
    self.state = self.game.get_state()
    img = None if self.state is None else self.state.screen_buffer
    if img is None:
      log.error('Game returned None screen buffer! This is not supposed to '
                'happen!')
      img = np.transpose(self._black_screen(), (2, 0, 1))
    if self.current_histogram is not None:
      self.current_histogram, self.previous_histogram = \
          self.previous_histogram, self.current_histogram
      self.current_histogram.fill(0)
    self._actions_flattened = None
    self._last_episode_info = copy.deepcopy(self._prev_info)
    self._prev_info = None
    self._num_episodes += 1
    return np.transpose(img, (1, 2, 0))

  def _convert_actions(self, actions):
    """Gym action -> flat ViZDoom button vector (see module docstring)."""
    if self.composite_action_space:
      spaces = self.action_space.spaces
    else:
      spaces, actions = (self.action_space,), (actions,)
    flat = []
    for space, action in zip(spaces, actions):
      if isinstance(space, gym.spaces.Box):
        flat.extend(list(np.asarray(action) *
                         self.delta_actions_scaling_factor))
      elif isinstance(space, Discretized):
        flat.append(space.to_continuous(action))
      elif isinstance(space, gym.spaces.Discrete):
        one_hot = [0] * (space.n - 1)
        if action > 0:
          one_hot[int(action) - 1] = 1
        flat.extend(one_hot)
      else:
        raise NotImplementedError('Action subspace type %s is not supported!'
                                  % type(space))
    return flat

  def _vizdoom_variables_bug_workaround(self, info, done):
    if done and 'DAMAGECOUNT' in info:
      log.info('DAMAGECOUNT value on done: %r', info.get('DAMAGECOUNT'))
    if self._last_episode_info is not None:
      for v in ('DEATHCOUNT', 'HITCOUNT', 'DAMAGECOUNT'):
        if v in info:
          info[v] -= self._last_episode_info.get(v, 0)

  def step(self, actions):
    info = {'num_frames': self.skip_frames}
    if self._actions_flattened is not None:
      flat, self._actions_flattened = self._actions_flattened, None
    else:
      flat = self._convert_actions(actions)
    reward = self.game.make_action(flat, self.skip_frames)
    state = self.game.get_state()
    done = self.game.is_episode_finished()
    if not done:
      observation = np.transpose(state.screen_buffer, (1, 2, 0))
      info.update(self.get_info(self._game_variables_dict(state)))
      self._update_histogram(info)
      self._prev_info = copy.deepcopy(info)
    else:
      observation = self._black_screen()
      info.update(self._prev_info or {})
    self._vizdoom_variables_bug_workaround(info, done)
    return observation, reward, done, info

  def render(self, mode='human'):
    state = self.game.get_state() if self.game is not None else None
    if state is None:
      return None
    img = np.transpose(state.screen_buffer, (1, 2, 0))
    if mode == 'rgb_array':
      return img
    from .doom_render import show_image  # pylint: disable=import-outside-toplevel
    show_image('vizdoom', img)
    return img

  def close(self):
    if self.game is not None:
      try:
        self.game.close()
      except Exception:  # pylint: disable=broad-except
        pass
    self.initialized = False

  def get_info(self, variables=None):
    if variables is None:
      variables = self._game_variables_dict(self.game.get_state())
    info = {'pos': self.get_positions(variables)}
    info.update(variables)
    return info

  def get_info_all(self, variables=None):
    state = self.game.get_state() if variables is None else None
    if variables is None and state is None:
      return dict(self._prev_info or {})
    if variables is None:
      variables = self._game_variables_dict(state)
    info = self.get_info(variables)
    if self.previous_histogram is not None:
      info['previous_histogram'] = self.previous_histogram
    return info

  def get_positions(self, variables):
    return self._get_positions(variables)

  @staticmethod
  def _get_positions(variables):
    if all(k in variables for k in ('POSITION_X', 'POSITION_Y', 'ANGLE')):
      return {'agent_x': variables['POSITION_X'],
              'agent_y': variables['POSITION_Y'],
              'agent_a': variables['ANGLE']}
    return {'agent_x': np.nan, 'agent_y': np.nan, 'agent_a': np.nan}

  def get_automap_buffer(self):
    if self.game.is_episode_finished():
      return None
    m = self.game.get_state().automap_buffer
    return None if m is None else np.transpose(m, (1, 2, 0))

  def _update_histogram(self, info, eps=1e-8):
    if self.current_histogram is None:
      return
    cl = self.coord_limits
    dx = (info['pos']['agent_x'] - cl[0]) / (cl[2] - cl[0])
    dy = (info['pos']['agent_y'] - cl[1]) / (cl[3] - cl[1])
    ix = int((dx - eps) * self.current_histogram.shape[0])
    iy = int((dy - eps) * self.current_histogram.shape[1])
    self.current_histogram[ix, iy] += 1

  # -- human play / replay -----------------------------------------------------
  def _key_to_action(self, key):
    if hasattr(self.action_space, 'key_to_action'):
      return self.action_space.key_to_action(key)
    return key_to_action_default(key)

  def _keyboard_on_press(self, key):
    from pynput.keyboard import Key  # pylint: disable=import-outside-toplevel
    if key == Key.esc:
      self._terminate = True
      return False
    action = self._key_to_action(key)
    if action is not None and action not in self._current_actions:
      self._current_actions.append(action)
    return True

  def _keyboard_on_release(self, key):
    action = self._key_to_action(key)
    if action is not None and action in self._current_actions:
      self._current_actions.remove(action)

  @staticmethod
  def play_human_mode(env, skip_frames=1, num_episodes=3, num_actions=None):
    """Keyboard play (needs pynput and a display)."""
    import threading  # pylint: disable=import-outside-toplevel
    from pynput.keyboard import Listener  # pylint: disable=import-outside-toplevel
    doom = env.unwrapped
    doom.skip_frames = 1

    def listen():
      with Listener(on_press=doom._keyboard_on_press,
                    on_release=doom._keyboard_on_release) as listener:
        listener.join()

    thread = threading.Thread(target=listen, daemon=True)
    thread.start()
    num_actions = 14 if num_actions is None else num_actions
    for _ in range(num_episodes):
      doom.mode = 'human'
      env.reset()
      last = time.time()
      while not doom.game.is_episode_finished() and not doom._terminate:
        actions = [0] * num_actions
        for a in doom._current_actions:
          if isinstance(a, int):
            actions[a] = 1
          elif a == 'turn_left':
            actions[-1] = -doom.delta_actions_scaling_factor
          elif a == 'turn_right':
            actions[-1] = doom.delta_actions_scaling_factor
        for _ in range(skip_frames):
          doom._actions_flattened = actions
          env.step(actions)
          wait = 1.0 / 35.0 - (time.time() - last)
          if wait > 0:
            time.sleep(wait)
          last = time.time()
    thread.join(timeout=1.0)

  @staticmethod
  def replay(env, rec_path):
    doom = env.unwrapped
    doom.mode = 'replay'
    doom._ensure_initialized()
    doom.game.replay_episode(rec_path)
    total, start = 0.0, time.time()
    while not doom.game.is_episode_finished():
      doom.game.advance_action()
      total += doom.game.get_last_reward()
      log.info('Episode reward: %.3f, time so far: %.1f s', total,
               time.time() - start)
    log.info('Finishing replay')
    doom.close()
