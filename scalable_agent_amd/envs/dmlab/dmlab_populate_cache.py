"""Pre-builds DMLab level .pk3 files into the level cache by resetting many
watermaze envs in parallel (reference envs/dmlab/dmlab_populate_cache.py)."""

import sys

from ...algo.multi_env import MultiEnv
from ...utils.utils import log
from .dmlab_utils import DmlabGymEnv


def main(num_envs=64, num_workers=16, max_resets=None):
  def make_env(env_config):
    del env_config
    return DmlabGymEnv('contributed/dmlab30/rooms_watermaze', 4)

  multi_env = MultiEnv(num_envs, num_workers, make_env, stats_episodes=100)
  resets = 0
  try:
    while max_resets is None or resets < max_resets:
      multi_env.reset()
      resets += 1
      log.info('Generated %d environments...', resets * num_envs)
  except (Exception, KeyboardInterrupt, SystemExit):  # pylint: disable=broad-except
    log.exception('Interrupt...')
  finally:
    log.info('Closing env...')
    multi_env.close()
  return 0


if __name__ == '__main__':
  sys.exit(main())
