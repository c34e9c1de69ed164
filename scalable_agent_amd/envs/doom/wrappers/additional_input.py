"""Measurement-vector input for Doom (reference
envs/doom/wrappers/additional_input.py): observation becomes
{'obs': frame, 'measurements': float32[7 + 2*NUM_WEAPONS]} with the DFP-style
scaled selected weapon/ammo, health, armor, kills, attack-ready, player
count, per-weapon ownership and ammo."""

import numpy as np

from ...gym_compat import Box, Dict, Wrapper
from .reward_shaping import NUM_WEAPONS


class DoomAdditionalInput(Wrapper):

  def __init__(self, env):
    super().__init__(env)
    self.num_weapons = NUM_WEAPONS
    low = [0.0, 0.0, -1.0, -1.0, -50.0, 0.0, 0.0] + [0.0] * (2 * NUM_WEAPONS)
    high = [20.0, 50.0, 50.0, 50.0, 50.0, 1.0, 10.0] + \
        [5.0] * NUM_WEAPONS + [50.0] * NUM_WEAPONS
    self.observation_space = Dict({
        'obs': env.observation_space,
        'measurements': Box(low=np.array(low, np.float32),
                            high=np.array(high, np.float32),
                            dtype=np.float32)})
    self.measurements_vec = np.zeros([len(low)], np.float32)

  def _parse_info(self, obs, info):
    m = self.measurements_vec
    weapon = round(max(0, info.get('SELECTED_WEAPON', 0.0)))
    ammo = min(max(0.0, info.get('SELECTED_WEAPON_AMMO', 0.0)) / 15.0, 5.0)
    info['HEALTH'] = max(0.0, info.get('HEALTH', 0.0))
    vals = [float(weapon), float(ammo), info['HEALTH'] / 30.0,
            info.get('ARMOR', 0.0) / 30.0, info.get('USER2', 0.0) / 10.0,
            info.get('ATTACK_READY', 0.0), info.get('PLAYER_COUNT', 1) / 5.0]
    vals += [max(0.0, info.get('WEAPON%d' % w, 0.0))
             for w in range(self.num_weapons)]
    vals += [min(max(0.0, info.get('AMMO%d' % w, 0.0)) / 15.0, 5.0)
             for w in range(self.num_weapons)]
    m[:] = vals
    return {'obs': obs, 'measurements': m}

  def reset(self):
    obs = self.env.reset()
    return self._parse_info(obs, self.env.unwrapped.get_info())

  def step(self, action):
    obs, rew, done, info = self.env.step(action)
    if obs is None:
      return obs, rew, done, info
    return self._parse_info(obs, info), rew, done, info
