"""Adaptive bot difficulty (reference envs/doom/wrappers/bot_difficulty.py):
+10 after winning a match outright, -10 after finishing last or second to
last, clamped to [0, 150]; disabled when starting at the maximum."""

from ...gym_compat import Wrapper
from ....utils.utils import log


class BotDifficultyWrapper(Wrapper):

  def __init__(self, env, initial_difficulty=None):
    super().__init__(env)
    self._min_difficulty, self._max_difficulty = 0, 150
    self._difficulty_step = 10
    self._curr_difficulty = 20 if initial_difficulty is None \
        else initial_difficulty
    self._difficulty_std = 10
    log.info('Starting with bot difficulty %d', self._curr_difficulty)
    self._adaptive_curriculum = initial_difficulty != self._max_difficulty
    if not self._adaptive_curriculum:
      log.debug('Starting at max difficulty, disable adaptive skill '
                'curriculum')

  def _analyze_standings(self, info):
    if 'FINAL_PLACE' not in info:
      return
    place = info['FINAL_PLACE']
    if place <= 1 and info.get('LEADER_GAP', 0.0) < 0:
      self._curr_difficulty = min(self._curr_difficulty +
                                  self._difficulty_step, self._max_difficulty)
    elif place >= int(info.get('PLAYER_COUNT', 1)) - 1:
      self._curr_difficulty = max(self._curr_difficulty -
                                  self._difficulty_step, self._min_difficulty)

  def reset(self, **kwargs):
    u = self.env.unwrapped
    if hasattr(u, 'bot_difficulty_mean'):
      u.bot_difficulty_mean = self._curr_difficulty
      u.bot_difficulty_std = self._difficulty_std
    return self.env.reset()

  def step(self, action):
    obs, reward, done, info = self.env.step(action)
    if obs is None:
      return obs, reward, done, info
    if done and self._adaptive_curriculum:
      self._analyze_standings(info)
    info['BOT_DIFFICULTY'] = self._curr_difficulty
    return obs, reward, done, info
