"""+1 reward whenever health increases (gathering scenarios; reference
envs/doom/wrappers/scenario_wrappers/gathering_reward_shaping.py)."""

from ....gym_compat import Wrapper


class DoomGatheringRewardShaping(Wrapper):

  def __init__(self, env):
    super().__init__(env)
    self._prev_health = None

  def _reward_shaping(self, info, done):
    if info is None or done:
      return 0.0
    health = info.get('HEALTH', 0.0)
    reward = 1.0 if (self._prev_health is not None and
                     health - self._prev_health > 0.0) else 0.0
    self._prev_health = health
    return reward

  def reset(self):
    self._prev_health = None
    return self.env.reset()

  def step(self, action):
    obs, reward, done, info = self.env.step(action)
    return obs, reward + self._reward_shaping(info, done), done, info
