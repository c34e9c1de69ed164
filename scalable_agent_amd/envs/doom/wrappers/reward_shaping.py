"""Game-variable reward shaping for Doom (reference
envs/doom/wrappers/reward_shaping.py).

A scheme maps variable deltas to rewards: `delta[VAR] = (reward per unit
increase, reward per unit decrease)`, plus a per-weapon bonus for keeping a
selected weapon with ammo unholstered for 5 consecutive steps.  Deltas of
DAMAGECOUNT/HITCOUNT are capped; no shaping on the respawn step or at the
episode end.  At the end the wrapper sets info['true_reward'] (env reward sum
or a scheme-specific function of the final info).

Fix vs the reference: the selected-weapon bonus is looked up for the weapon
actually selected (the reference reads a module-level loop variable,
reward_shaping.py:148).
"""

import collections
import copy
import operator

from ...gym_compat import Wrapper
from ....algo.algo_utils import EPS
from ....utils.utils import log

NUM_WEAPONS = 8

WEAPON_PREFERENCE = {2: 1, 3: 5, 4: 5, 5: 5, 6: 10, 7: 10}  # pistol..bfg

WEAPON_DELTA_REWARDS = {}
SELECTED_WEAPON_REWARDS = {}
for _w in range(NUM_WEAPONS):
  _pref = WEAPON_PREFERENCE.get(_w, 1)
  WEAPON_DELTA_REWARDS['WEAPON%d' % _w] = (+0.02 * _pref, -0.01 * _pref)
  WEAPON_DELTA_REWARDS['AMMO%d' % _w] = (+0.0002 * _pref, -0.0001 * _pref)
  SELECTED_WEAPON_REWARDS['SELECTED%d' % _w] = 0.0002 * _pref

REWARD_SHAPING_DEATHMATCH_V0 = dict(
    delta=dict(FRAGCOUNT=(+1, -1.5), DEATHCOUNT=(-0.75, +0.75),
               HITCOUNT=(+0.01, -0.01), DAMAGECOUNT=(+0.003, -0.003),
               HEALTH=(+0.005, -0.003), ARMOR=(+0.005, -0.001),
               **WEAPON_DELTA_REWARDS),
    selected_weapon=SELECTED_WEAPON_REWARDS)

# "zero-sum" scheme for self-play
REWARD_SHAPING_DEATHMATCH_V1 = copy.deepcopy(REWARD_SHAPING_DEATHMATCH_V0)
REWARD_SHAPING_DEATHMATCH_V1['delta'].update(dict(
    FRAGCOUNT=(+1, -0.001), DEATHCOUNT=(-1, +1), HITCOUNT=(0, 0),
    DAMAGECOUNT=(+0.01, -0.01), HEALTH=(+0.01, -0.01)))

# battle: also reward ammo pickups so the agent does not run dry
REWARD_SHAPING_BATTLE = copy.deepcopy(REWARD_SHAPING_DEATHMATCH_V0)
REWARD_SHAPING_BATTLE['delta'].update(dict(AMMO2=(+0.02, -0.001)))


def true_reward_final_position(info):
  if info['LEADER_GAP'] == 0:
    return 0.0     # ties are not wins
  if info['FINAL_PLACE'] > 1:
    return 0.0
  assert info['FINAL_PLACE'] == 1
  return 1.0


def true_reward_frags(info):
  return info['FRAGCOUNT']


class DoomRewardShapingWrapper(Wrapper):

  def __init__(self, env, reward_shaping_scheme=None, true_reward_func=None):
    super().__init__(env)
    self.reward_shaping_scheme = reward_shaping_scheme
    self.true_reward_func = true_reward_func
    self.reward_delta_limits = dict(DAMAGECOUNT=200, HITCOUNT=5)
    self.prev_vars = {}
    self.prev_dead = True
    self.orig_env_reward = self.total_shaping_reward = 0.0
    self.selected_weapon = collections.deque([], maxlen=5)
    self.reward_structure = {}
    self.verbose = False
    self.print_once = False
    self.env.unwrapped._reward_shaping_wrapper = self

  def _delta_rewards(self, info):
    reward, deltas = 0.0, []
    for var, (up, down) in self.reward_shaping_scheme['delta'].items():
      if var not in self.prev_vars:
        continue
      delta = info.get(var, 0.0) - self.prev_vars[var]
      if var in self.reward_delta_limits:
        delta = min(delta, self.reward_delta_limits[var])
      if abs(delta) > EPS:
        r = delta * up if delta > EPS else -delta * down
        reward += r
        deltas.append((var, r, delta))
        self.reward_structure[var] = self.reward_structure.get(var, 0.0) + r
    return reward, deltas

  def _selected_weapon_rewards(self, selected_weapon, selected_weapon_ammo,
                               deltas):
    unholstered = len(self.selected_weapon) > 4 and all(
        sw == selected_weapon for sw in self.selected_weapon)
    reward = 0.0
    if selected_weapon_ammo > 0 and unholstered:
      reward = self.reward_shaping_scheme['selected_weapon'].get(
          'SELECTED%d' % selected_weapon, 0.0)
      key = 'weapon%d' % selected_weapon
      deltas.append((key, reward))
      self.reward_structure[key] = self.reward_structure.get(key, 0.0) + reward
    return reward

  def _parse_info(self, info, done):
    if self.reward_shaping_scheme is None:
      return 0.0
    selected_weapon = int(max(0, info.get('SELECTED_WEAPON', 0.0)))
    ammo = float(max(0.0, info.get('SELECTED_WEAPON_AMMO', 0.0)))
    self.selected_weapon.append(selected_weapon)
    just_respawned = self.prev_dead and not info.get('DEAD', 0.0)
    shaping = 0.0
    if not done and not just_respawned:
      shaping, deltas = self._delta_rewards(info)
      shaping += self._selected_weapon_rewards(selected_weapon, ammo, deltas)
      if abs(shaping) > 2.5 and not self.print_once:
        log.info('Large shaping reward %.3f for %r', shaping, deltas)
        self.print_once = True
    if done and 'FRAGCOUNT' in self.reward_structure:
      items = sorted(self.reward_structure.items(),
                     key=operator.itemgetter(1))
      log.info('Sum rewards: %.3f, reward structure: %r',
               sum(r for _, r in items), {k: '%.3f' % r for k, r in items})
    return shaping

  def reset(self):
    obs = self.env.reset()
    self.prev_vars = {}
    self.prev_dead = True
    self.reward_structure = {}
    self.selected_weapon.clear()
    self.orig_env_reward = self.total_shaping_reward = 0.0
    self.print_once = False
    return obs

  def step(self, action):
    obs, rew, done, info = self.env.step(action)
    if obs is None:
      return obs, rew, done, info
    self.orig_env_reward += rew
    shaping = self._parse_info(info, done)
    rew += shaping
    self.total_shaping_reward += shaping
    if self.verbose:
      log.info('Original env reward before shaping: %.3f',
               self.orig_env_reward)
      log.info('Total shaping reward is %.3f for %d (done %d)',
               self.total_shaping_reward,
               getattr(self.env.unwrapped, 'player_id', 1), done)
    if self.reward_shaping_scheme is not None:
      for var in self.reward_shaping_scheme['delta']:
        self.prev_vars[var] = info.get(var, 0.0)
    self.prev_dead = bool(info.get('DEAD', 0.0))
    if done:
      info['true_reward'] = (self.orig_env_reward
                             if self.true_reward_func is None
                             else self.true_reward_func(info))
    return obs, rew, done, info

  def close(self):
    self.env.unwrapped._reward_shaping_wrapper = None
    return self.env.close()
