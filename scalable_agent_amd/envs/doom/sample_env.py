"""Runs one doom_battle episode with random actions (reference
envs/doom/sample_env.py)."""

import sys

from ..arguments import default_cfg
from ..create_env import create_env
from ...utils.utils import log


def main(env_name='doom_battle', render=True):
  env = create_env(env_name, cfg=default_cfg(env=env_name))
  env.reset()
  done, steps, total = False, 0, 0.0
  while not done:
    if render:
      env.render()
    _, rew, done, _ = env.step(env.action_space.sample())
    steps += 1
    total += rew
  log.info('Done! %d steps, reward %.3f', steps, total)
  env.close()
  return 0


if __name__ == '__main__':
  sys.exit(main())
