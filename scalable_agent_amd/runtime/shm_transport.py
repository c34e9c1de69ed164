"""Distributed (multi-process) actors on one node over shared memory.

Replaces the reference's distributed mode (experiment.py:497-512, 669-672;
TF gRPC ClusterSpec with a learner-side FIFOQueue and parameter pulls):

  * unrolls travel through the native `ShmRing` (csrc/envpool/shm_ring.cc):
    every actor process claims a slot, writes its T+1-step ActorOutput in
    place (fixed byte layout, `UnrollLayout`) and commits it; the learner
    claims committed slots in commit order;
  * weights travel through a seqlock-protected shared-memory snapshot
    (`WeightStore`): the learner publishes its flat fp32 parameter buffer
    after each update, actors re-read it when the version changes.

Segment names are derived from the logdir, so `--job_name=learner --task=0`
and `--job_name=actor --task=i` started with the same flags rendezvous
without any network service.
"""

import hashlib
import logging
import struct
import time

import numpy as np

from . import native
from ..structs import ActorOutput, AgentOutput, StepOutput, StepOutputInfo

log = logging.getLogger('scalable_agent_amd')
INSTR_LEN = 16


def segment_names(logdir):
  h = hashlib.sha1(logdir.encode()).hexdigest()[:12]
  return '/sa_ring_' + h, '/sa_w_' + h


class UnrollLayout(object):
  """Fixed byte layout of one ActorOutput inside a ring slot."""

  def __init__(self, T1, frame_shape, num_actions, core_size=256):
    spec = [('level', np.int32, ()), ('c', np.float32, (core_size,)),
            ('h', np.float32, (core_size,)), ('reward', np.float32, (T1,)),
            ('done', np.bool_, (T1,)), ('ep_ret', np.float32, (T1,)),
            ('ep_step', np.int32, (T1,)),
            ('frames', np.uint8, (T1,) + tuple(frame_shape)),
            ('instr_ids', np.int64, (T1, INSTR_LEN)),
            ('instr_len', np.int64, (T1,)), ('action', np.int64, (T1,)),
            ('logits', np.float32, (T1, num_actions)),
            ('baseline', np.float32, (T1,))]
    self.fields = []
    off = 0
    for name, dt, shape in spec:
      n = int(np.prod(shape)) * np.dtype(dt).itemsize
      off = (off + 63) // 64 * 64
      self.fields.append((name, dt, shape, off, n))
      off += n
    self.nbytes = off

  def views(self, buf):
    return {name: np.frombuffer(buf, dtype=dt, count=int(np.prod(shape)),
                                offset=off).reshape(shape)
            for name, dt, shape, off, _ in self.fields}

  def encode(self, out, level_index, buf):
    v = self.views(buf)
    eo, ao = out.env_outputs, out.agent_outputs
    v['level'][...] = level_index
    v['c'][...] = out.agent_state[0]
    v['h'][...] = out.agent_state[1]
    v['reward'][...] = eo.reward
    v['done'][...] = eo.done
    v['ep_ret'][...] = eo.info.episode_return
    v['ep_step'][...] = eo.info.episode_step
    v['frames'][...] = eo.observation[0]
    v['instr_ids'][...] = eo.observation[1][0]
    v['instr_len'][...] = eo.observation[1][1]
    v['action'][...] = ao.action
    v['logits'][...] = ao.policy_logits
    v['baseline'][...] = ao.baseline

  def decode(self, buf, level_names):
    v = {k: a.copy() for k, a in self.views(buf).items()}
    return ActorOutput(
        level_name=level_names[int(v['level'])],
        agent_state=(v['c'], v['h']),
        env_outputs=StepOutput(v['reward'],
                               StepOutputInfo(v['ep_ret'], v['ep_step']),
                               v['done'],
                               (v['frames'], (v['instr_ids'],
                                              v['instr_len']))),
        agent_outputs=AgentOutput(v['action'], v['logits'], v['baseline']))


class WeightStore(object):
  """Seqlock weight snapshot: header [version u64][numel u64] + fp32 data."""

  HDR = 64

  def __init__(self, name, numel=0, create=False):
    import mmap
    import os
    self.name = name
    path = '/dev/shm' + name
    if create:
      size = self.HDR + 4 * numel
      fd = os.open(path, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o600)
      os.ftruncate(fd, size)
    else:
      fd = os.open(path, os.O_RDWR)
      size = os.fstat(fd).st_size
    self._mm = mmap.mmap(fd, size)
    os.close(fd)
    self._owner = create
    self._path = path
    if create:
      struct.pack_into('<QQ', self._mm, 0, 0, numel)
    self.numel = struct.unpack_from('<Q', self._mm, 8)[0]
    self.data = np.frombuffer(self._mm, dtype=np.float32, count=self.numel,
                              offset=self.HDR)

  def version(self):
    return struct.unpack_from('<Q', self._mm, 0)[0]

  def write(self, flat):
    v = self.version()
    struct.pack_into('<Q', self._mm, 0, v + 1)  # odd: writing
    self.data[...] = flat
    struct.pack_into('<Q', self._mm, 0, v + 2)

  def read(self, out):
    """Consistent copy into `out`; returns the version read."""
    while True:
      v0 = self.version()
      if v0 & 1:
        time.sleep(0.001)
        continue
      out[...] = self.data
      if self.version() == v0:
        return v0

  def close(self):
    import os
    del self.data
    self._mm.close()
    if self._owner:
      try:
        os.unlink(self._path)
      except OSError:
        pass


class LearnerTransport(object):
  """Learner side: creates the ring + weight store, pumps unrolls."""

  def __init__(self, flags, frame_shape, num_actions, learner):
    from ..experiment import level_names_for
    self.level_names = level_names_for(flags)
    self.layout = UnrollLayout(flags.unroll_length + 1, frame_shape,
                               num_actions)
    ring_name, w_name = segment_names(flags.logdir)
    self.ring = native.ShmRing(ring_name, max(4, 2 * flags.num_actors),
                               self.layout.nbytes, True)
    self.learner = learner
    self.weights = WeightStore(w_name, learner.flat.numel, create=True)
    self.publish_weights()

  def publish_weights(self):
    self.weights.write(self.learner.flat.params.detach().cpu().numpy())

  def pump(self, q, stop):
    import queue as queue_lib
    while not stop.is_set():
      slot = self.ring.acquire_read(200)
      if slot < 0:
        if slot == -2:
          return
        continue
      out = self.layout.decode(self.ring.slot_view(slot), self.level_names)
      self.ring.release(slot)
      while not stop.is_set():
        try:
          q.put(out, timeout=0.5)
          break
        except queue_lib.Full:
          pass

  def close(self):
    self.ring.close()
    self.weights.close()
    del self.ring


def run_actor_process(flags, level_names, action_set, frame_shape, use_instr):
  """`--job_name=actor --task=i`: one env + CPU agent, ships unrolls."""
  import torch
  from .. import environments
  from ..actor import Actor
  from ..experiment import create_environment
  from ..models import Agent
  from ..optim import FlatParams

  level = level_names[flags.task % len(level_names)]
  env = create_environment(flags, level, seed=flags.task + 1)
  env.start()
  from ..experiment import num_value_heads
  agent = Agent(len(action_set), torso=flags.torso, frame_shape=frame_shape,
                seed=flags.seed, num_value_heads=num_value_heads(flags))
  flat = FlatParams(agent)
  layout = UnrollLayout(flags.unroll_length + 1, frame_shape, len(action_set))
  ring_name, w_name = segment_names(flags.logdir)
  deadline = time.time() + 120
  while True:
    try:
      ring = native.ShmRing(ring_name)
      weights = WeightStore(w_name)
      break
    except (RuntimeError, OSError, FileNotFoundError):
      if time.time() > deadline:
        raise RuntimeError('learner segments %s not found' % ring_name)
      time.sleep(0.5)
  host = np.empty(weights.numel, np.float32)
  version = -1
  gen = torch.Generator().manual_seed(flags.seed + flags.task)

  @torch.no_grad()
  def infer(last_action, reward, done, frame, ids, n, c, h):
    t = torch.from_numpy
    instr = (t(ids), t(n)) if use_instr and int(n.max()) > 0 else None
    out, (c2, h2) = agent.step(
        t(last_action), StepOutput(t(reward), None, t(done), (t(frame), instr)),
        (t(c), t(h)), generator=gen)
    return (out.action.numpy(), out.policy_logits.numpy(),
            out.baseline.numpy(), c2.numpy(), h2.numpy())

  actor = Actor(environments.FlowEnvironment(env), infer, level, action_set,
                flags.unroll_length, len(action_set), use_instruction=use_instr)
  level_index = level_names.index(level)
  try:
    while not ring.closed:
      v = weights.version()
      if v != version:
        version = weights.read(host)
        flat.params.copy_(torch.from_numpy(host))
      out = actor.unroll()
      slot = ring.acquire_write(1000)
      if slot == -2:
        break
      if slot < 0:
        continue
      layout.encode(out, level_index, ring.slot_view(slot))
      ring.commit(slot)
  finally:
    env.close()
