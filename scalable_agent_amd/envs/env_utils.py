"""Vectorised env construction (reference envs/env_utils.py): multi-agent
envs go through MultiAgentEnvAggregator, others through MultiEnv."""

from ..algo.multi_env import MultiEnv
from ..utils.utils import log


def create_multi_env(num_envs, num_workers, make_env_func, stats_episodes,
                     use_multiprocessing=True):
  tmp = make_env_func(None)
  agents = getattr(tmp, 'num_agents', 1)
  tmp.close()
  if agents > 1:
    from .doom.multiplayer.doom_multiagent_wrapper import \
        MultiAgentEnvAggregator  # pylint: disable=import-outside-toplevel
    assert num_envs % agents == 0
    log.debug('Num envs %d agents %d', num_envs, agents)
    return MultiAgentEnvAggregator(num_envs // agents, num_workers,
                                   make_env_func, stats_episodes,
                                   use_multiprocessing)
  return MultiEnv(num_envs, num_workers, make_env_func, stats_episodes,
                  use_multiprocessing)
