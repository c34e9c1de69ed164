"""Learner semantics on CPU (the reference has no learner/agent/loss tests;
SURVEY.md §4 item 2): loss = reference formula, step updates params with the
TF-RMSProp rule, frame counter / LR schedule, both torsos, agent semantics."""

import numpy as np
import pytest
import torch

from scalable_agent_amd import flags as flags_lib
from scalable_agent_amd import losses as L
from scalable_agent_amd import vtrace as V
from scalable_agent_amd.envs.synthetic import make_synthetic_batch
from scalable_agent_amd.learner import Learner, compute_loss
from scalable_agent_amd.models import Agent, layers
from scalable_agent_amd.optim import polynomial_decay


def _flags(**kw):
  d = dict(batch_size=2, unroll_length=6, total_environment_frames=10000)
  d.update(kw)
  return flags_lib.default_flags(**d)


@pytest.mark.parametrize('torso', ['shallow', 'deep'])
def test_learner_step_cpu(torso):
  torch.manual_seed(0)
  f = _flags(torso=torso)
  agent = Agent(9, torso=torso, frame_shape=(24, 32, 3), seed=1)
  learner = Learner(agent, f, 'cpu')
  batch = make_synthetic_batch(2, 6, (24, 32, 3), 9, seed=3)
  p0 = learner.flat.params.clone()
  loss = learner.step(batch)
  assert torch.isfinite(loss)
  assert not torch.equal(p0, learner.flat.params)
  assert int(learner.frames) == 2 * 6 * 4


def test_rmsprop_first_step_matches_tf_formula():
  torch.manual_seed(0)
  f = _flags(learning_rate=0.01, momentum=0.0)
  agent = Agent(9, torso='shallow', frame_shape=(24, 32, 3), seed=1)
  learner = Learner(agent, f, 'cpu')
  batch = make_synthetic_batch(2, 6, (24, 32, 3), 9, seed=3)
  p0 = learner.flat.params.clone()
  learner.flat.zero_grad()
  compute_loss(agent, batch, f).backward()
  g = learner.flat.grads.clone()
  learner.flat.params.copy_(p0)
  learner._apply()
  ms = 1.0 + (g * g - 1.0) * (1 - f.decay)
  expected = p0 - 0.01 * g / torch.sqrt(ms + f.epsilon)
  torch.testing.assert_close(learner.flat.params, expected, rtol=1e-5,
                             atol=1e-7)


def test_loss_matches_reference_formula():
  torch.manual_seed(0)
  f = _flags()
  agent = Agent(9, torso='shallow', frame_shape=(24, 32, 3), seed=1)
  batch = make_synthetic_batch(2, 6, (24, 32, 3), 9, seed=4)
  loss = compute_loss(agent, batch, f)
  # independent re-derivation (experiment.py:346-407)
  out, _ = agent.unroll(batch.agent_outputs.action, batch.env_outputs,
                        batch.agent_state, sample=False)
  bootstrap = out.baseline[-1]
  a = batch.agent_outputs.action[1:]
  r = torch.clamp(batch.env_outputs.reward[1:], -1, 1)
  disc = (~batch.env_outputs.done[1:]).float() * f.discounting
  vt = V.from_logits(batch.agent_outputs.policy_logits[1:],
                     out.policy_logits[:-1], a, disc, r, out.baseline[:-1],
                     bootstrap)
  ref = (L.compute_policy_gradient_loss(out.policy_logits[:-1], a,
                                        vt.pg_advantages) +
         f.baseline_cost * L.compute_baseline_loss(vt.vs - out.baseline[:-1]) +
         f.entropy_cost * L.compute_entropy_loss(out.policy_logits[:-1]))
  torch.testing.assert_close(loss, ref)


def test_polynomial_decay():
  assert polynomial_decay(1.0, 0, 100) == 1.0
  assert abs(polynomial_decay(1.0, 25, 100) - 0.75) < 1e-12
  assert polynomial_decay(1.0, 1000, 100) == 0.0


def test_same_padding_and_shapes():
  assert layers.same_pads(72, 8, 4) == (2, 2)
  assert layers.same_pads(18, 4, 2) == (1, 1)
  assert layers.same_pads(12, 3, 2) == (0, 1)   # asymmetric W pad (K4)
  assert layers.same_pads(72, 3, 2) == (0, 1)   # deep maxpool
  agent = Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=0)
  assert agent.flat_size == 9 * 12 * 32
  agent = Agent(9, torso='shallow', frame_shape=(72, 96, 3), seed=0)
  assert agent.flat_size == 5 * 6 * 128
  agent = Agent(9, torso='shallow', frame_shape=(72, 128, 3), seed=0)
  assert agent.flat_size == 5 * 8 * 128  # Doom 128x72


def test_core_resets_state_on_done():
  torch.manual_seed(0)
  agent = Agent(4, torso='shallow', frame_shape=(16, 16, 3), seed=0)
  T, B = 3, 2
  x = torch.randn(T, B, agent.core_input_size)
  done = torch.tensor([[False, False], [True, False], [False, False]])
  state = (torch.randn(B, 256), torch.randn(B, 256))
  out, _ = agent.core_unroll(x, done, state)
  # row 0 at t=1 must equal a fresh unroll of steps 1.. from zero state
  out2, _ = agent.core_unroll(x[1:, :1], torch.zeros(2, 1, dtype=torch.bool),
                              (torch.zeros(1, 256), torch.zeros(1, 256)))
  torch.testing.assert_close(out[1:, 0], out2[:, 0])


def test_instruction_encoder_last_valid_output():
  torch.manual_seed(0)
  from scalable_agent_amd.models import tokenize
  agent = Agent(4, torso='shallow', frame_shape=(16, 16, 3), seed=0)
  ids, lens = tokenize(['go to the red ball', '', 'left'])
  out = agent.instruction_encoding((torch.from_numpy(ids),
                                    torch.from_numpy(lens)), 3, 'cpu')
  assert out.shape == (3, 64)
  assert torch.all(out[1] == 0)           # empty instruction -> zeros
  single = agent.instruction_encoding(
      (torch.from_numpy(ids[2:3, :1]), torch.from_numpy(lens[2:3])), 1, 'cpu')
  torch.testing.assert_close(out[2:3], single)


def test_agent_step_sampling_shapes():
  agent = Agent(9, torso='shallow', frame_shape=(24, 32, 3), seed=0)
  B = 5
  from scalable_agent_amd.structs import StepOutput
  eo = StepOutput(torch.zeros(B), None, torch.ones(B, dtype=torch.bool),
                  (torch.zeros(B, 24, 32, 3, dtype=torch.uint8), None))
  out, (c, h) = agent.step(torch.zeros(B, dtype=torch.long), eo,
                           agent.initial_state(B))
  assert out.action.shape == (B,) and out.policy_logits.shape == (B, 9)
  assert out.baseline.shape == (B,) and c.shape == (B, 256)
  assert int(out.action.max()) < 9


def test_popart_preserves_outputs_and_normalises():
  """PopArt: the statistics move towards the targets and the value head is
  rescaled so unnormalised outputs are preserved exactly."""
  import torch
  from scalable_agent_amd.popart import PopArt
  torch.manual_seed(0)
  pa = PopArt(3, beta=0.5)
  w = torch.randn(8, 3)
  b = torch.randn(3)
  x = torch.randn(5, 8)

  def unnorm(w, b):
    return (x @ w + b) * pa.sigma() + pa.mu

  before = unnorm(w, b)
  targets = torch.randn(4, 6) * 10 + 50  # [T, B]
  tasks = torch.tensor([0, 0, 1, 1, 0, 1])
  pa.update(targets, tasks, w, b)
  torch.testing.assert_close(unnorm(w, b), before, rtol=1e-4, atol=1e-3)
  assert pa.mu[0] > 10 and pa.mu[1] > 10 and pa.mu[2] == 0  # task 2 absent
  assert pa.sigma()[2] == 1.0


def test_learner_popart_step_cpu():
  import torch
  from scalable_agent_amd import flags as flags_lib
  from scalable_agent_amd.envs.synthetic import make_synthetic_batch
  from scalable_agent_amd.learner import Learner
  from scalable_agent_amd.models import Agent
  f = flags_lib.default_flags(batch_size=2, unroll_length=4, popart=True,
                              popart_beta=0.1)
  agent = Agent(9, torso='shallow', frame_shape=(24, 32, 3), seed=1,
                num_value_heads=2)
  learner = Learner(agent, f, 'cpu')
  batch = make_synthetic_batch(2, 4, (24, 32, 3), 9, seed=0)
  batch = batch._replace(level_name=torch.tensor([0, 1]))
  for _ in range(3):
    loss = learner.step(batch)
    assert torch.isfinite(loss)
  assert float(learner.popart.mu.abs().sum()) > 0
  sd = learner.state_dict()
  assert 'popart' in sd


def test_flat_staging_roundtrip():
  from scalable_agent_amd.learner import FlatStaging, _map_tensors
  b1 = make_synthetic_batch(3, 5, (8, 10, 3), 4, seed=1)
  b2 = make_synthetic_batch(3, 5, (8, 10, 3), 4, seed=2)
  host = FlatStaging(b1, 'cpu').load(b1)
  dev = FlatStaging(b1, 'cpu')
  leaves = []
  _map_tensors(dev.views, lambda t: leaves.append(t) or t)
  assert all(t.data_ptr() % 256 == 0 for t in leaves)
  assert all(t.untyped_storage().data_ptr() ==
             dev.flat.untyped_storage().data_ptr() for t in leaves)
  dev.copy_from(host, non_blocking=False)
  got, want = [], []
  _map_tensors(dev.views, lambda t: got.append(t) or t)
  _map_tensors(b1, lambda t: want.append(t) or t)
  assert len(got) == len(want) and all(torch.equal(a, b)
                                       for a, b in zip(got, want))
  host.load(b2)  # reusing the slab changes every view in place
  dev.copy_from(host, non_blocking=False)
  got2, want2 = [], []
  _map_tensors(dev.views, lambda t: got2.append(t) or t)
  _map_tensors(b2, lambda t: want2.append(t) or t)
  assert all(torch.equal(a, b) for a, b in zip(got2, want2))
  assert got2[0].data_ptr() == got[0].data_ptr()
