"""Wire structures exchanged between envs, actors and the learner.

Mirrors the namedtuples of the reference:
  * `ActorOutput`, `AgentOutput`            experiment.py:98-102
  * `StepOutput`, `StepOutputInfo`          environments.py:143-146
  * `VTraceReturns`, `VTraceFromLogitsReturns`  vtrace.py:37-42

Every time-indexed field of an unroll has T+1 entries; element 0 overlaps the
last element of the previous unroll (experiment.py:305-321).
"""

import collections

ActorOutput = collections.namedtuple(
    'ActorOutput', 'level_name agent_state env_outputs agent_outputs')
AgentOutput = collections.namedtuple('AgentOutput',
                                     'action policy_logits baseline')
StepOutputInfo = collections.namedtuple('StepOutputInfo',
                                        'episode_return episode_step')
StepOutput = collections.namedtuple('StepOutput',
                                    'reward info done observation')
VTraceFromLogitsReturns = collections.namedtuple(
    'VTraceFromLogitsReturns',
    ['vs', 'pg_advantages', 'log_rhos', 'behaviour_action_log_probs',
     'target_action_log_probs'])
VTraceReturns = collections.namedtuple('VTraceReturns', 'vs pg_advantages')
