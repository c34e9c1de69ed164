"""Single-agent env seen as a 1-agent multi-agent env (reference
algorithms/utils/multi_agent.py): lists of length 1, auto-reset on done."""

from ..envs.gym_compat import Wrapper


class MultiAgentWrapper(Wrapper):

  def __init__(self, env):
    super().__init__(env)
    self.num_agents = 1

  def reset(self, **kwargs):
    return [self.env.reset(**kwargs)]

  def step(self, action):
    obs, rew, done, info = self.env.step(action[0])
    if done:
      obs = self.env.reset()
    return [obs], [rew], [done], [info]
