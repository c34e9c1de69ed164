"""Multiplayer ViZDoom instance (reference envs/doom/multiplayer/
doom_multiagent.py:25-220).

Player 0 hosts a deathmatch on a UDP port (`-host N -port P -deathmatch`
with forced respawn, no autoaim/crouch/jump/freelook/exit, respawn delay,
4-minute time limit); the other players `-join 127.0.0.1:P`.  The host adds
bots on every reset: named bots, or - when an adaptive difficulty is set -
random bots whose difficulty is drawn around the mean (rounded to tens,
clamped to [10, 100]).  With several agents and skip_frames == 1 the wrapper
drives frames with set_action/advance_action and only materialises the
state on `update_state` steps.
"""

import copy
import os

import numpy as np

from ..doom_gym import VizdoomEnv
from ....utils.network import is_udp_port_available
from ....utils.utils import log

DEFAULT_UDP_PORT = int(os.environ.get('DOOM_DEFAULT_UDP_PORT', 40300))


def find_available_port(start_port, increment=1000):
  port = start_port
  while port < 65535 and not is_udp_port_available(port):
    port += increment
  log.debug('Port %r is available', port)
  return port


class VizdoomEnvMultiplayer(VizdoomEnv):

  BOT_NAMES = ['Blazkowicz', 'PerfectBlue', 'PerfectRed', 'PerfectGreen',
               'PerfectPurple', 'PerfectYellow', 'PerfectWhite',
               'PerfectLtGreen']

  def __init__(self, action_space, config_file, player_id, num_agents,
               max_num_players, num_bots, skip_frames, async_mode=False,
               respawn_delay=0, record_to=None, backend=None):
    super().__init__(action_space, config_file, skip_frames=skip_frames,
                     async_mode=async_mode, record_to=record_to,
                     backend=backend)
    self.worker_index = 0
    self.vector_index = 0
    self.player_id = player_id
    self.num_agents = num_agents
    self.max_num_players = max_num_players
    self.num_bots = num_bots
    self.timestep = 0
    self.update_state = True
    self.bot_names = list(self.BOT_NAMES)
    self.bot_difficulty_mean = self.bot_difficulty_std = None
    self.hardest_bot, self.easiest_bot = 100, 10
    self.respawn_delay = respawn_delay
    self.is_multiplayer = True
    self.init_info = None

  def _is_server(self):
    return self.player_id == 0

  def _ensure_initialized(self):
    if self.initialized:
      return
    self._create_doom_game(self.mode)
    port = DEFAULT_UDP_PORT if self.init_info is None else \
        self.init_info.get('port', DEFAULT_UDP_PORT)
    if self._is_server():
      log.info('Using port %d on host...', port)
      if not is_udp_port_available(port):
        raise Exception('Port %r unavailable' % port)
      self.game.add_game_args(' '.join([
          '-host %d' % self.max_num_players, '-port %d' % port,
          '-deathmatch', '+timelimit 4.0', '+sv_forcerespawn 1',
          '+sv_noautoaim 1', '+sv_respawnprotect 1', '+sv_spawnfarthest 1',
          '+sv_nocrouch 1', '+sv_nojump 1', '+sv_nofreelook 1',
          '+sv_noexit 1', '+viz_respawn_delay %d' % self.respawn_delay,
          '+viz_connect_timeout 4']))
      self.game.add_game_args('+name AI%d_host +colorset 0' % self.player_id)
    else:
      self.game.add_game_args('-join 127.0.0.1:%d +viz_connect_timeout 4 '
                              % port)
      self.game.add_game_args('+name AI%d +colorset 0' % self.player_id)
    self.game.init()
    log.info('Initialized w:%d v:%d player:%d', self.worker_index,
             self.vector_index, self.player_id)
    self.initialized = True

  def _random_bot(self, difficulty, used_bots):
    while True:
      name = 'BOT_%d_%d' % (difficulty, self.rng.randint(0, self.num_bots))
      if name not in used_bots:
        used_bots.append(name)
        return name

  def reset(self):
    obs = super().reset()
    if self._is_server() and self.num_bots > 0:
      self.game.send_game_command('removebots')
      names = copy.deepcopy(self.bot_names)
      self.rng.shuffle(names)
      used = []
      for i in range(self.num_bots):
        if self.bot_difficulty_mean is None:
          suffix = ' ' + names[i] if i < len(names) else ''
          self.game.send_game_command('addbot' + suffix)
        else:
          diff = self.rng.normal(self.bot_difficulty_mean,
                                 self.bot_difficulty_std)
          diff = int(round(diff, -1))
          diff = min(self.hardest_bot, max(self.easiest_bot, diff))
          self.game.send_game_command('addbot ' + self._random_bot(diff,
                                                                   used))
    self.timestep = 0
    self.update_state = True
    return obs

  def step(self, actions):
    if self.skip_frames > 1 or self.num_agents == 1:
      return super().step(actions)
    self._ensure_initialized()
    info = {}
    self.game.set_action(self._convert_actions(actions))
    self.game.advance_action(1, self.update_state)
    self.timestep += 1
    if not self.update_state:
      return None, None, None, None
    state = self.game.get_state()
    reward = self.game.get_last_reward()
    done = self.game.is_episode_finished()
    if not done:
      obs = np.transpose(state.screen_buffer, (1, 2, 0))
      info.update(self.get_info(self._game_variables_dict(state)))
    else:
      obs = np.zeros(self.observation_space.shape, np.uint8)
    self._vizdoom_variables_bug_workaround(info, done)
    return obs, reward, done, info
