"""Learner on the GPU: the HIP-graph step matches the eager step (same
parameters after several updates), with and without PopArt."""

import pytest
import torch

from scalable_agent_amd import flags as flags_lib
from scalable_agent_amd.envs.synthetic import make_synthetic_batch
from scalable_agent_amd.learner import Learner, batch_to_device
from scalable_agent_amd.models import Agent

pytestmark = pytest.mark.gpu


def _learner(popart, device):
  from scalable_agent_amd import ops
  ops.load()
  f = flags_lib.default_flags(batch_size=4, unroll_length=8, popart=popart,
                              popart_beta=0.05)
  agent = Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=5,
                backend='hip', compute_dtype=torch.bfloat16,
                num_value_heads=2 if popart else 1)
  return Learner(agent, f, device)


@pytest.mark.parametrize('popart', [False, True])
def test_graph_step_matches_eager(cuda, popart):
  batches = []
  for i in range(3):
    b = make_synthetic_batch(4, 8, (72, 96, 3), 9, seed=i)
    if popart:
      b = b._replace(level_name=torch.tensor([0, 1, 0, 1]))
    batches.append(batch_to_device(b, cuda))
  eager = _learner(popart, cuda)
  graph = _learner(popart, cuda)
  graph.flat.params.copy_(eager.flat.params)
  for b in batches:
    le = eager.step(b)
    if graph._graph is None:
      graph.capture(b)
    graph.load_static(b)
    lg = graph.graph_step()
    torch.cuda.synchronize()
    assert torch.isfinite(le) and torch.isfinite(lg)
    torch.testing.assert_close(lg.float(), le.float(), rtol=2e-2, atol=1e-2)
  torch.testing.assert_close(graph.flat.params, eager.flat.params,
                             rtol=1e-3, atol=1e-4)
  if popart:
    torch.testing.assert_close(graph.popart.mu, eager.popart.mu)
    assert float(eager.popart.mu.abs().sum()) > 0


@pytest.mark.parametrize('dtype,instructions', [
    (torch.bfloat16, False), (torch.bfloat16, True),
    (torch.float32, False), (torch.float32, True)])
def test_pipelined_unroll_matches_serial(cuda, dtype, instructions):
  """The time-chunked torso || LSTM pipeline (side stream) computes the same
  loss and gradients as the serial unroll, eager and graph-captured; with
  instructions the side stream also reads the main-stream instruction
  encoding (agent.py record_stream)."""
  from scalable_agent_amd import ops
  from scalable_agent_amd.envs.synthetic import add_synthetic_instructions
  from scalable_agent_amd.learner import compute_loss
  ops.load()
  f = flags_lib.default_flags(batch_size=4, unroll_length=15)
  b = make_synthetic_batch(4, 15, (72, 96, 3), 9, seed=7)
  res = []
  for chunks in (1, 4):
    agent = Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=5,
                  backend='hip', compute_dtype=dtype,
                  pipeline_chunks=chunks)
    bb = b
    if instructions:
      bb = add_synthetic_instructions(b, agent.embed.shape[0], seed=3)
    bb = batch_to_device(bb, cuda)
    lrn = Learner(agent, f, cuda)
    lrn.flat.zero_grad()
    loss = compute_loss(agent, bb, f, use_fused=True)
    loss.backward()
    torch.cuda.synchronize()
    res.append((loss.detach().clone(), lrn.flat.grads.clone(), lrn, bb))
    del loss  # frees the eager autograd graph before the capture below
  (l1, g1, _, _), (l4, g4, lrn4, b4) = res
  cos = float(torch.dot(g4, g1) / (g4.norm() * g1.norm()))
  if dtype == torch.float32:
    # exact-fp32 kernels on both sides (per-step recurrence either way, the
    # chunked dfeats ReLU mask in the GEMM epilogue, dh0 through gemm_f32 at
    # each chunk boundary, the carried c_last): only the summation order of
    # the chunked GEMMs differs
    torch.testing.assert_close(l4, l1, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(g4, g1, rtol=1e-3,
                               atol=1e-4 * float(g1.abs().max()))
    assert cos > 0.999999, cos
  else:
    # chunks=1 runs the fused core with the bf16 gang recurrence, the
    # pipeline the same fused core per chunk with the per-step recurrence
    # kernels (never the gang next to a concurrent torso): same math,
    # different roundings
    torch.testing.assert_close(l4, l1, rtol=2e-3, atol=2e-2)
    assert cos > 0.999, cos
  if instructions:
    emb = lrn4.flat.view_of(g4, 'embed')
    assert float(emb.abs().sum()) > 0
  b = b4
  # graph capture of the pipelined step replays the same loss
  before = lrn4.flat.params.clone()
  lrn4.capture(b)
  lrn4.load_static(b)
  lg = lrn4.graph_step()
  torch.cuda.synchronize()
  torch.testing.assert_close(lg.float(), l4.float(), rtol=1e-3, atol=1e-3)
  assert not torch.equal(before, lrn4.flat.params)


@pytest.mark.parametrize('groups,server', [(0, False), (-1, False),
                                           (2, True)])
def test_experiment_train_and_test_on_gpu(tmp_path, groups, server):
  """The full driver on the GPU: actor threads with batched GPU inference
  (groups=0) or the default actor-group process (groups=-1: one group,
  pipelined splits, captured fixed-batch inference), the HIP-graph learner,
  checkpoint, then --mode=test from the checkpoint (reference Dockerfile
  smoke, deep torso)."""
  import os
  import subprocess
  import sys
  if not torch.cuda.is_available():
    pytest.skip('no GPU')
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  common = [sys.executable, os.path.join(root, 'experiment.py'),
            '--level_name=synthetic', '--torso=deep', '--unroll_length=8',
            '--synthetic_episode_length=10', '--logdir=' + str(tmp_path)]
  env = dict(os.environ, PYTHONPATH=root)
  r = subprocess.run(common + ['--num_actors=4', '--batch_size=4',
                               '--actor_groups=%d' % groups,
                               '--inference_server=%s' % server,
                               '--total_environment_frames=1280',
                               '--save_summaries_secs=0'],
                     capture_output=True, text=True, timeout=100, env=env)
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'Episode return' in r.stderr
  r = subprocess.run(common + ['--mode=test', '--test_num_episodes=2'],
                     capture_output=True, text=True, timeout=100, env=env)
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'Mean episode return' in r.stderr
