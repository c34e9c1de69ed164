"""Match standings in info (reference envs/doom/wrappers/
multiplayer_stats.py): KDR, FINAL_PLACE (1 = leader) and LEADER_GAP (frags
behind the leader; <= 0 gap to 2nd place when leading), refreshed every 20
steps and at the episode end."""

import numpy as np

from ...gym_compat import Wrapper


class MultiplayerStatsWrapper(Wrapper):

  def __init__(self, env):
    super().__init__(env)
    self.timestep = 0
    self.prev_extra_info = {}

  def _parse_info(self, info, done):
    if (self.timestep % 20 == 0 or done) and 'FRAGCOUNT' in info:
      extra = {'KDR': float(info.get('FRAGCOUNT', 0.0) /
                            (info.get('DEATHCOUNT', 0.0) + 1))}
      me = int(info.get('PLAYER_NUM', info.get('PLAYER_NUMBER', 1)))
      count = max(int(info.get('PLAYER_COUNT', 1)), me)
      frags = [int(info.get('PLAYER%d_FRAGCOUNT' % p, -100000))
               for p in range(1, count + 1)]
      order = list(np.argsort(frags, kind='stable'))
      place = count - order.index(me - 1)
      extra['FINAL_PLACE'] = place
      if place > 1:
        extra['LEADER_GAP'] = max(frags) - frags[me - 1]
      elif count > 1:
        top = sorted(frags, reverse=True)
        extra['LEADER_GAP'] = top[1] - top[0]
        assert extra['LEADER_GAP'] <= 0
      else:
        extra['LEADER_GAP'] = 0
      self.prev_extra_info = extra
    else:
      extra = self.prev_extra_info
    info.update(extra)
    return info

  def reset(self, **kwargs):
    self.timestep = 0
    self.prev_extra_info = {}
    return self.env.reset()

  def step(self, action):
    obs, reward, done, info = self.env.step(action)
    if obs is None:
      return obs, reward, done, info
    info = self._parse_info(info, done)
    self.timestep += 1
    return obs, reward, done, info
