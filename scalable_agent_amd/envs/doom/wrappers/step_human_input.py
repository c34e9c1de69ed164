"""Human-input stepping (reference envs/doom/wrappers/step_human_input.py):
ignores the agent action and advances the game with keyboard input."""

import numpy as np

from ...gym_compat import Wrapper


class StepHumanInput(Wrapper):

  def reset(self):
    self.unwrapped.mode = 'human'
    self.unwrapped._ensure_initialized()
    return self.env.reset()

  def step(self, action):
    del action
    doom = self.unwrapped
    doom.mode = 'human'
    doom._ensure_initialized()
    doom.game.advance_action()
    state = doom.game.get_state()
    done = doom.game.is_episode_finished()
    reward = doom.game.get_last_reward()
    if not done:
      obs = np.transpose(state.screen_buffer, (1, 2, 0))
    else:
      obs = np.zeros(self.observation_space.shape, np.uint8)
    return obs, reward, done, {'dummy': 0}
