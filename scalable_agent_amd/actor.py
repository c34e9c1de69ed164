"""Actors: env interaction loop producing T+1-step unrolls.

Reference: build_actor (experiment.py:240-321).  The actor keeps persistent
state across unrolls - last env output, env state, agent (LSTM) state and last
agent output - and every unroll:
  * records the agent state at the START of the unroll (experiment.py:286, 307);
  * runs `unroll_length` steps: agent(last action, env output, state) -> new
    action (batched on the GPU through the dynamic batcher), env.step(action);
  * emits T+1 time-indexed entries whose element 0 repeats the previous
    unroll's last element (experiment.py:305-321).
Output arrays are numpy, time-major, without the batch dimension.
"""

import logging
import time

import numpy as np

from .models.instruction import tokenize
from .py_process import EnvRestartedError
from .utils.tracing import trace
from .structs import ActorOutput, AgentOutput, StepOutput, StepOutputInfo

INSTR_LEN = 16  # max words kept per instruction (batcher rows need one shape)


def encode_instruction(instr):
  if instr is None or (isinstance(instr, (str, bytes)) and len(instr) == 0):
    return np.zeros(INSTR_LEN, np.int64), np.int64(0)
  ids, lengths = tokenize([instr], max_len=INSTR_LEN)
  n = min(int(lengths[0]), INSTR_LEN)
  out = np.zeros(INSTR_LEN, np.int64)
  out[:n] = ids[0, :n]
  return out, np.int64(n)


class Actor(object):
  """One actor = one env + persistent recurrent state."""

  def __init__(self, env, infer_fn, level_name, action_set, unroll_length,
               num_actions, core_size=256, use_instruction=True, stall_ms=0):
    """env: FlowEnvironment; infer_fn(last_action, reward, done, frame,
    instr_ids, instr_len, c, h) on batch-1 numpy arrays -> (action, logits,
    baseline, c, h)."""
    self._env = env
    self._infer = infer_fn
    self.level_name = level_name
    self._action_set = action_set
    self._T = unroll_length
    self._A = num_actions
    self._core = core_size
    self._use_instr = use_instruction
    self._env_output = None
    self._stall_s = stall_ms / 1000.0  # fault injection: slow actor
    self.env_restarts = 0

  def _reset(self):
    env_output, env_state = self._env.initial()
    self._env_output, self._env_state = env_output, env_state
    self._agent_state = (np.zeros(self._core, np.float32),
                         np.zeros(self._core, np.float32))
    self._agent_output = AgentOutput(np.int64(0),
                                     np.zeros(self._A, np.float32),
                                     np.float32(0.))

  def _step_agent(self):
    eo = self._env_output
    frame, instr = eo.observation
    ids, n = encode_instruction(instr if self._use_instr else None)
    c, h = self._agent_state
    with trace('actor_inference'):
      out = self._infer(
          np.asarray([self._agent_output.action], np.int64),
          np.asarray([eo.reward], np.float32),
          np.asarray([eo.done], np.bool_),
          np.asarray(frame, np.uint8)[None],
          ids[None], np.asarray([n], np.int64), c[None], h[None])
    action, logits, baseline, c2, h2 = out
    self._agent_state = (np.asarray(c2[0], np.float32),
                         np.asarray(h2[0], np.float32))
    self._agent_output = AgentOutput(np.int64(action[0]),
                                     np.asarray(logits[0], np.float32),
                                     np.float32(baseline[0]))

  def unroll(self):
    """Runs one unroll; returns an ActorOutput of numpy arrays [T+1, ...].

    If the env worker dies or hangs mid-unroll (EnvRestartedError), the
    partial unroll is dropped and a fresh episode starts."""
    while True:
      try:
        return self._unroll()
      except EnvRestartedError as e:
        self.env_restarts += 1
        logging.getLogger('scalable_agent_amd').warning(
            'actor %s: %s; dropping the in-flight unroll', self.level_name, e)
        self._env_output = None

  def _unroll(self):
    if self._stall_s:
      time.sleep(self._stall_s)
    if self._env_output is None:
      self._reset()
    T1 = self._T + 1
    first_state = (self._agent_state[0].copy(), self._agent_state[1].copy())
    frame0 = np.asarray(self._env_output.observation[0])
    frames = np.empty((T1,) + frame0.shape, np.uint8)
    reward = np.empty(T1, np.float32)
    done = np.empty(T1, np.bool_)
    ep_ret = np.empty(T1, np.float32)
    ep_step = np.empty(T1, np.int32)
    instr_ids = np.zeros((T1, INSTR_LEN), np.int64)
    instr_len = np.zeros(T1, np.int64)
    action = np.empty(T1, np.int64)
    logits = np.empty((T1, self._A), np.float32)
    baseline = np.empty(T1, np.float32)

    def record(t):
      eo, ao = self._env_output, self._agent_output
      frames[t] = eo.observation[0]
      reward[t] = eo.reward
      done[t] = eo.done
      ep_ret[t] = eo.info.episode_return
      ep_step[t] = eo.info.episode_step
      if self._use_instr:
        instr_ids[t], instr_len[t] = encode_instruction(eo.observation[1])
      action[t] = ao.action
      logits[t] = ao.policy_logits
      baseline[t] = ao.baseline

    record(0)
    for t in range(1, T1):
      self._step_agent()
      raw_action = self._action_set[int(self._agent_output.action)]
      self._env_output, self._env_state = self._env.step(raw_action,
                                                         self._env_state)
      record(t)
    return ActorOutput(
        level_name=self.level_name, agent_state=first_state,
        env_outputs=StepOutput(reward, StepOutputInfo(ep_ret, ep_step), done,
                               (frames, (instr_ids, instr_len))),
        agent_outputs=AgentOutput(action, logits, baseline))


  # ---------------------------------------------------- trajectory queue
  def unroll_into(self, tq, level_index, stop=None):
    """Runs one unroll straight into a claimed column of a
    runtime.traj_queue.TrajectoryQueue slab: every step's fields land in
    their time-major [t, column] position (no per-unroll arrays, no stacking
    or transposing on the learner side).  Returns False when the queue is
    closed / `stop` is set before a column was claimed.  An env restart
    mid-unroll rewrites the same column from a fresh episode."""
    while True:
      s, col, v = tq.claim(timeout_ms=200)
      if s >= 0:
        break
      if s == -2 or (stop is not None and stop.is_set()):
        return False
    while True:
      try:
        self._unroll_to(v, col, level_index)
        break
      except EnvRestartedError as e:
        self.env_restarts += 1
        logging.getLogger('scalable_agent_amd').warning(
            'actor %s: %s; dropping the in-flight unroll (its column is '
            'rewritten from a fresh episode)', self.level_name, e)
        self._env_output = None
    tq.commit(s)
    return True

  def _unroll_to(self, v, col, level_index):
    if self._stall_s:
      time.sleep(self._stall_s)
    if self._env_output is None:
      self._reset()
    v['level'][col] = level_index
    v['c'][col] = self._agent_state[0]
    v['h'][col] = self._agent_state[1]
    frame, reward, done = v['frame'], v['reward'], v['done']
    ep_ret, ep_step = v['episode_return'], v['episode_step']
    action, logits, baseline = v['action'], v['policy_logits'], v['baseline']
    use_instr = self._use_instr and 'instr_ids' in v

    def record(t):
      eo, ao = self._env_output, self._agent_output
      frame[t, col] = eo.observation[0]
      reward[t, col] = eo.reward
      done[t, col] = eo.done
      ep_ret[t, col] = eo.info.episode_return
      ep_step[t, col] = eo.info.episode_step
      if use_instr:
        v['instr_ids'][t, col], v['instr_len'][t, col] = encode_instruction(
            eo.observation[1])
      action[t, col] = ao.action
      logits[t, col] = ao.policy_logits
      baseline[t, col] = ao.baseline

    record(0)
    for t in range(1, self._T + 1):
      self._step_agent()
      raw_action = self._action_set[int(self._agent_output.action)]
      self._env_output, self._env_state = self._env.step(raw_action,
                                                         self._env_state)
      record(t)


def stack_unrolls(unrolls, use_instruction=False, pin=False):
  """B unrolls -> one time-major batch (torch tensors [T+1, B, ...])."""
  import torch  # local: actors may run without torch on the hot path
  def st(xs, axis=1):
    return torch.from_numpy(np.ascontiguousarray(np.stack(xs, axis)))
  eo = [u.env_outputs for u in unrolls]
  ao = [u.agent_outputs for u in unrolls]
  frames = st([e.observation[0] for e in eo])
  instr = None
  if use_instruction:
    instr = (st([e.observation[1][0] for e in eo]),
             st([e.observation[1][1] for e in eo]))
  out = ActorOutput(
      level_name=[u.level_name for u in unrolls],
      agent_state=(st([u.agent_state[0] for u in unrolls], 0),
                   st([u.agent_state[1] for u in unrolls], 0)),
      env_outputs=StepOutput(st([e.reward for e in eo]),
                             StepOutputInfo(st([e.info.episode_return
                                                for e in eo]),
                                            st([e.info.episode_step
                                                for e in eo])),
                             st([e.done for e in eo]), (frames, instr)),
      agent_outputs=AgentOutput(st([a.action for a in ao]),
                                st([a.policy_logits for a in ao]),
                                st([a.baseline for a in ao])))
  if pin:
    from .learner import _map_tensors
    out = _map_tensors(out, lambda t: t.pin_memory())
  return out
