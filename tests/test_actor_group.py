"""Vectorised actor-group processes (runtime/actor_group.py): the shared
double-buffered weight snapshot, the actor split, VectorInfer against the
per-row InferenceModel, and CPU end-to-end training with --actor_groups
(including env-worker crashes inside a group)."""

import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from scalable_agent_amd.runtime.actor_group import (SharedWeights, board_geometry,
                                                   split_actors)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ['--level_name=synthetic', '--unroll_length=5', '--device=cpu',
          '--dtype=fp32', '--torso=shallow', '--synthetic_episode_length=6',
          '--height=24', '--width=32']


def test_split_actors():
  assert split_actors(5, 2) == [[0, 1, 2], [3, 4]]
  assert split_actors(3, 8) == [[0], [1], [2]]
  groups = split_actors(48, 7)
  assert sorted(sum(groups, [])) == list(range(48))
  assert max(map(len, groups)) - min(map(len, groups)) <= 1


def test_shared_weights_double_buffer_seqlock():
  name = '/sa_w_test_%d' % os.getpid()
  w = SharedWeights(name, 10, create=True)
  try:
    r = SharedWeights.attach(name, lambda: True, timeout_s=5)
    assert r is not None and r.numel == 10
    assert r.version() == 0 and r.latest() == -1
    w.publish(torch.arange(10, dtype=torch.float32))
    assert r.version() == 1 and r.latest() == 0 and r.seq(0) % 2 == 0
    out = np.zeros(10, np.float32)
    assert r.read_into(out) == 1 and np.array_equal(out, np.arange(10))
    w.publish(torch.full((10,), 7.0))
    assert r.latest() == 1 and r.version() == 2
    assert r.read_into(out) == 2 and np.all(out == 7)
    # a writer mid-update on the non-latest buffer leaves `latest` readable
    b = w._target()
    assert b == 0 and r.seq(0) % 2 == 1 and r.latest() == 1
    assert r.read_into(out) == 2 and np.all(out == 7)
    r.close()
  finally:
    w.close()
  assert not os.path.exists('/dev/shm' + name)


def test_vector_infer_matches_the_per_row_model():
  from scalable_agent_amd.inference import InferenceModel, VectorInfer
  from scalable_agent_amd.models import Agent
  M, shape, A = 3, (24, 32, 3), 9
  agent = Agent(A, torso='shallow', frame_shape=shape, seed=3)
  ref = Agent(A, torso='shallow', frame_shape=shape, seed=3)
  model = InferenceModel(agent, 'cpu', use_instruction=False, seed=5)
  ref_model = InferenceModel(ref, 'cpu', use_instruction=False, seed=5)
  vi = VectorInfer(model, M, shape, A)
  rng = np.random.RandomState(0)
  c = np.zeros((M, 256), np.float32)
  h = np.zeros((M, 256), np.float32)
  for step in range(3):
    frame = rng.randint(0, 256, (M,) + shape).astype(np.uint8)
    reward = rng.randn(M).astype(np.float32)
    done = np.array([step == 0, False, step == 2])
    la = rng.randint(0, A, M).astype(np.int64)
    vi.inputs['frame'][:] = frame
    vi.inputs['reward'][:] = reward
    vi.inputs['done'][:] = done
    vi.inputs['last_action'][:] = la
    _, logits, baseline, c2, h2 = vi.run()
    _, rl, rb, rc, rh = ref_model.infer(
        la, reward, done, frame, np.zeros((M, 16), np.int64),
        np.zeros(M, np.int64), c, h)
    np.testing.assert_allclose(logits, rl, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(baseline, rb, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(c2, rc, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(h2, rh, rtol=1e-5, atol=1e-6)
    c, h = rc, rh  # the vector path keeps its state; the reference threads it


def _run(args, timeout=240):
  env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS='2')
  return subprocess.run([sys.executable, os.path.join(ROOT, 'experiment.py')]
                        + COMMON + args, capture_output=True, text=True,
                        timeout=timeout, env=env)


def test_train_with_actor_groups(tmp_path):
  logdir = str(tmp_path / 'groups')
  r = _run(['--logdir=' + logdir, '--num_actors=5', '--batch_size=2',
            '--actor_groups=2', '--total_environment_frames=480',
            '--save_summaries_secs=0', '--log_every_frames=160'])
  assert r.returncode == 0, r.stderr[-3000:]
  assert '2 actor group(s) over 5 envs' in r.stderr
  assert 'Episode return' in r.stderr
  assert 'learner host' in r.stderr
  assert os.path.exists(os.path.join(logdir, 'checkpoint'))


def test_actor_groups_survive_env_crashes(tmp_path):
  logdir = str(tmp_path / 'crash')
  r = _run(['--logdir=' + logdir, '--num_actors=4', '--batch_size=2',
            '--actor_groups=2', '--total_environment_frames=640',
            '--fault_inject=env_crash:0.02', '--save_summaries_secs=0'])
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'episode truncated' in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_vector_infer_graph_on_gpu(cuda, dtype):
  """The captured VectorInfer graph (HIP agent) against the eager per-batch
  InferenceModel.infer of an identical agent on the same device."""
  from scalable_agent_amd.inference import InferenceModel, VectorInfer
  from scalable_agent_amd.models import Agent
  M, shape, A = 6, (72, 96, 3), 9
  mk = lambda: Agent(A, torso='deep', frame_shape=shape, seed=3,
                     backend='hip', compute_dtype=dtype)
  model = InferenceModel(mk(), 'cuda', use_instruction=False, seed=5)
  ref_model = InferenceModel(mk(), 'cuda', use_instruction=False, seed=5)
  vi = VectorInfer(model, M, shape, A)
  assert vi.use_graph
  rng = np.random.RandomState(0)
  c = np.zeros((M, 256), np.float32)
  h = np.zeros((M, 256), np.float32)
  tol = 2e-5 if dtype == torch.float32 else 2e-2
  for step in range(4):
    frame = rng.randint(0, 256, (M,) + shape).astype(np.uint8)
    reward = rng.randn(M).astype(np.float32)
    done = np.array([step == 0, False, step == 2, False, True, False])
    la = rng.randint(0, A, M).astype(np.int64)
    vi.inputs['frame'][:] = frame
    vi.inputs['reward'][:] = reward
    vi.inputs['done'][:] = done
    vi.inputs['last_action'][:] = la
    _, logits, baseline, c2, h2 = [x.copy() for x in vi.run()]
    _, rl, rb, rc, rh = ref_model.infer(
        la, reward, done, frame, np.zeros((M, 16), np.int64),
        np.zeros(M, np.int64), c, h)
    np.testing.assert_allclose(logits, rl, rtol=tol, atol=tol)
    np.testing.assert_allclose(baseline, rb, rtol=tol, atol=tol)
    np.testing.assert_allclose(h2, rh, rtol=tol, atol=tol)
    c, h = rc, rh


def _board_worker(board, slot, rows, n_steps, seed):
  import os as _os
  from scalable_agent_amd.runtime.inference_board import BoardClient
  cl = BoardClient(board, slot, rows)
  rng = np.random.RandomState(seed)
  for _ in range(n_steps):
    cl.inputs['frame'][:] = rng.randint(0, 256, cl.inputs['frame'].shape)
    cl.inputs['done'][:] = False
    cl.launch()
    a, lg, b, c, h = cl.wait()
    assert a.shape == (rows,) and np.all((a >= 0) & (a < 9))
    assert np.all(np.isfinite(lg)) and np.all(np.isfinite(c))
  _os._exit(0)


def test_inference_board_serves_forked_workers():
  """Two forked workers (different row counts) post to the shared board; a
  CPU server answers each with its own rows; the LSTM state of rows that
  were not in a batch does not move."""
  import multiprocessing as mp
  from scalable_agent_amd.inference import InferenceModel
  from scalable_agent_amd.models import Agent
  from scalable_agent_amd.runtime.inference_board import (BoardServer,
                                                          InferenceBoard)
  shape = (24, 32, 3)
  board = InferenceBoard(3, 4, shape, 9)
  model = InferenceModel(Agent(9, torso='shallow', frame_shape=shape, seed=2),
                         'cpu', use_instruction=False, seed=1)
  server = BoardServer(model, board, use_graph=False)
  ctx = mp.get_context('fork')
  procs = [ctx.Process(target=_board_worker, args=(board, s, r, 5, s))
           for s, r in ((0, 4), (2, 3))]
  for p in procs:
    p.start()
  served = 0
  deadline = __import__('time').time() + 60
  while any(p.is_alive() for p in procs) and __import__('time').time() < deadline:
    served += server.serve_once(timeout_ms=20)
  for p in procs:
    p.join(10)
    assert p.exitcode == 0
  assert served >= 5 and server.rows_served == 5 * (4 + 3)
  # slot 1 never asked: its rows' state is untouched; slot 2's 4th row is
  # padding (3 rows): untouched too
  assert float(server.c[4:8].abs().sum()) == 0.0
  assert float(server.c[8 + 3:].abs().sum()) == 0.0
  assert float(server.c[0:4].abs().sum()) > 0.0
  board.close()


@pytest.mark.parametrize('lanes', [1, 2])
def test_train_with_inference_server(tmp_path, lanes):
  logdir = str(tmp_path / 'board')
  r = _run(['--logdir=' + logdir, '--num_actors=6', '--batch_size=2',
            '--actor_groups=3', '--inference_server=true',
            '--inference_lanes=%d' % lanes,
            '--total_environment_frames=480', '--save_summaries_secs=0'])
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'board served by the learner process' in r.stderr
  assert 'Episode return' in r.stderr
  assert 'inference board:' in r.stderr
  assert os.path.exists(os.path.join(logdir, 'checkpoint'))


def test_board_geometry_lanes():
  # 3 groups x 2 splits: one board of 6 slots, or lane 0 (groups 0, 2) and
  # lane 1 (group 1) on boards of 4 slots; rows = the largest split
  assert board_geometry(150, 3, 2) == (6, 25)
  assert board_geometry(150, 3, 2, lanes=2) == (4, 25)
  assert board_geometry(48, 2, 2, lanes=2) == (2, 12)
  assert board_geometry(6, 3, 2, lanes=8) == (2, 1)  # lanes <= groups
