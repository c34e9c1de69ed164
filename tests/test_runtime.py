"""Host runtime: shared-memory ring, weight snapshot, summaries, checkpoints,
DMLab-30 scoring, flags, timing/decay utilities."""

import glob
import os
import threading

import numpy as np
import pytest
import torch

from scalable_agent_amd import checkpoint as ckpt
from scalable_agent_amd import dmlab30
from scalable_agent_amd import flags as flags_lib
from scalable_agent_amd.runtime import native
from scalable_agent_amd.runtime.shm_transport import (UnrollLayout,
                                                      WeightStore)
from scalable_agent_amd.summary import SummaryWriter, read_events, crc32c


def test_shm_ring_fifo_and_cross_thread():
  name = '/sa_test_ring_%d' % os.getpid()
  ring = native.ShmRing(name, 4, 1000, True)
  attached = native.ShmRing(name)
  assert attached.num_slots == 4 and attached.slot_bytes >= 1000
  order = []
  for v in (7, 8, 9):
    s = attached.acquire_write(100)
    np.frombuffer(attached.slot_view(s), np.uint8)[0] = v
    attached.commit(s)
  for _ in range(3):
    s = ring.acquire_read(100)
    order.append(int(np.frombuffer(ring.slot_view(s), np.uint8)[0]))
    ring.release(s)
  assert order == [7, 8, 9]
  assert ring.acquire_read(50) == -1        # timeout
  got = []
  t = threading.Thread(target=lambda: got.append(ring.acquire_read(2000)))
  t.start()
  s = attached.acquire_write(100)
  attached.commit(s)
  t.join()
  assert got[0] >= 0
  ring.close()
  assert attached.acquire_write(10) == -2   # closed
  del attached, ring


def test_unroll_layout_roundtrip():
  from scalable_agent_amd.actor import INSTR_LEN
  from scalable_agent_amd.structs import (ActorOutput, AgentOutput,
                                          StepOutput, StepOutputInfo)
  T1, shape, A = 6, (8, 10, 3), 5
  rng = np.random.RandomState(0)
  out = ActorOutput(
      'lvl', (rng.randn(256).astype(np.float32),
              rng.randn(256).astype(np.float32)),
      StepOutput(rng.randn(T1).astype(np.float32),
                 StepOutputInfo(rng.randn(T1).astype(np.float32),
                                rng.randint(0, 9, T1).astype(np.int32)),
                 rng.rand(T1) < 0.5,
                 (rng.randint(0, 255, (T1,) + shape).astype(np.uint8),
                  (rng.randint(0, 999, (T1, INSTR_LEN)),
                   rng.randint(0, 5, T1)))),
      AgentOutput(rng.randint(0, A, T1), rng.randn(T1, A).astype(np.float32),
                  rng.randn(T1).astype(np.float32)))
  lay = UnrollLayout(T1, shape, A)
  buf = bytearray(lay.nbytes)
  lay.encode(out, 0, buf)
  back = lay.decode(buf, ['lvl'])
  for a, b in zip(
      [out.agent_state[0], out.env_outputs.reward, out.env_outputs.done,
       out.env_outputs.observation[0], out.agent_outputs.policy_logits],
      [back.agent_state[0], back.env_outputs.reward, back.env_outputs.done,
       back.env_outputs.observation[0], back.agent_outputs.policy_logits]):
    np.testing.assert_array_equal(a, b)


def test_weight_store_seqlock():
  name = '/sa_test_w_%d' % os.getpid()
  w = WeightStore(name, 100, create=True)
  r = WeightStore(name)
  w.write(np.arange(100, dtype=np.float32))
  out = np.zeros(100, np.float32)
  v = r.read(out)
  assert v == 2 and out[99] == 99
  r.close()
  w.close()


def test_summary_writer_roundtrip(tmp_path):
  assert crc32c(b'123456789') == 0xE3069283  # CRC32C check value
  w = SummaryWriter(str(tmp_path))
  w.add_scalars({'total_loss': 1.5, 'learning_rate': 0.1}, 10)
  w.add_histogram('action', np.array([0, 1, 1, 2]), 10)
  w.add_scalar('lvl/episode_return', 3.0, 20)
  w.close()
  ev = read_events(glob.glob(str(tmp_path / 'events.out.tfevents*'))[0])
  assert ev[1] == (10, {'total_loss': 1.5, 'learning_rate': pytest.approx(0.1)})
  assert ev[3] == (20, {'lvl/episode_return': 3.0})


def test_checkpoint_roundtrip_and_keep(tmp_path):
  from scalable_agent_amd.learner import Learner
  from scalable_agent_amd.models import Agent
  f = flags_lib.default_flags(batch_size=1, unroll_length=2)
  a = Agent(9, torso='shallow', frame_shape=(16, 16, 3), seed=1)
  learner = Learner(a, f, 'cpu')
  for i in range(7):
    learner.frames.fill_(100 * (i + 1))
    learner.opt.ms.add_(1.0)
    ckpt.save(str(tmp_path), learner, f, keep=5)
  files = sorted(glob.glob(str(tmp_path / 'checkpoint_*.pt')))
  assert len(files) == 5
  assert ckpt.latest_checkpoint(str(tmp_path)).endswith('checkpoint_700.pt')
  b = Agent(9, torso='shallow', frame_shape=(16, 16, 3), seed=2)
  learner2 = Learner(b, f, 'cpu')
  assert ckpt.restore(str(tmp_path), learner2) == 700
  torch.testing.assert_close(learner2.flat.params, learner.flat.params)
  torch.testing.assert_close(learner2.opt.ms, learner.opt.ms)
  st = ckpt.load_state(ckpt.latest_checkpoint(str(tmp_path)))
  assert 'agent/lstm_cell/kernel' in st['params']


def test_dmlab30_scores():
  levels = {l: [dmlab30.HUMAN_SCORES[dmlab30.LEVEL_MAPPING[l]]]
            for l in dmlab30.LEVEL_MAPPING}
  assert dmlab30.compute_human_normalized_score(levels, None) == \
      pytest.approx(100.0)
  levels = {l: [dmlab30.RANDOM_SCORES[dmlab30.LEVEL_MAPPING[l]]]
            for l in dmlab30.LEVEL_MAPPING}
  assert dmlab30.compute_human_normalized_score(levels, 100) == \
      pytest.approx(0.0)
  bad = dict(levels)
  bad.pop('rooms_watermaze')
  with pytest.raises(ValueError, match='Missing levels'):
    dmlab30.compute_human_normalized_score(bad, None)
  assert len(dmlab30.ALL_LEVELS) == 32


def test_flags_defaults_and_parsing():
  f = flags_lib.parse_flags([])
  assert (f.batch_size, f.unroll_length, f.num_action_repeats) == (2, 100, 4)
  assert f.learning_rate == 0.00048 and f.epsilon == .1 and f.decay == .99
  assert f.reward_clipping == 'abs_one' and f.level_name == \
      'explore_goal_locations_small'
  f = flags_lib.parse_flags(['--batch_size=32', '--torso', 'deep',
                             '--reward_clipping=soft_asymmetric'])
  assert f.batch_size == 32 and f.torso == 'deep'
  assert flags_lib.frames_per_step(f) == 32 * 100 * 4
  with pytest.raises(SystemExit):
    flags_lib.parse_flags(['--no_such_flag=1'])


def test_flags_reject_bf16_shallow_on_hip():
  # the shallow torso has exact-fp32 HIP kernels only: refused, not run fp32
  with pytest.raises(SystemExit, match='shallow torso has no bf16'):
    flags_lib.parse_flags(['--dtype=bf16', '--torso=shallow'])
  f = flags_lib.parse_flags(['--dtype=bf16', '--torso=shallow', '--backend=torch'])
  assert f.dtype == 'bf16' and f.torso == 'shallow'
  f = flags_lib.parse_flags(['--dtype=bf16', '--torso=deep'])
  assert f.dtype == 'bf16'


def test_timing_and_decay_utils():
  from scalable_agent_amd.utils.decay import LinearDecay
  from scalable_agent_amd.utils.timing import Timing, StepTimer
  d = LinearDecay([(0, 100), (1000, 50)])
  assert d.at(-5) == 100 and d.at(500) == 75 and d.at(2000) == 50
  d = LinearDecay([(0, 0), (1000, 100)], staircase=10)
  assert d.at(540) == 50
  t = Timing()
  with t.timeit('x'):
    pass
  assert t.x > 0
  st = StepTimer(100)
  st.step()
  st.step()
  assert st.frames_per_sec() > 0


def test_udp_port_probe():
  from scalable_agent_amd.utils.network import is_udp_port_available
  is_udp_port_available(50301)
