"""--deterministic on the HIP learner: two identical learner steps from the
same initial state and batch are bitwise identical (gradients and updated
parameters).  The bf16 torso switches its weight-gradient flush from float
atomics to per-workgroup slots summed in a fixed order
(conv_tune('deterministic', 1)); the fp32 torso, the learner heads and the
column-sum kernels always reduce in a fixed order."""

import pytest
import torch

from scalable_agent_amd import flags as flags_lib
from scalable_agent_amd import ops
from scalable_agent_amd.envs.synthetic import make_synthetic_batch
from scalable_agent_amd.learner import Learner, _map_tensors
from scalable_agent_amd.models import Agent

pytestmark = pytest.mark.gpu


def _two_steps(device, dtype, torso, det=True):
  cdt = torch.bfloat16 if dtype == 'bf16' else torch.float32
  flags = flags_lib.default_flags(batch_size=8, unroll_length=20, torso=torso,
                                  dtype=dtype, deterministic=det)
  agent = Agent(9, torso=torso, seed=11, backend='hip', compute_dtype=cdt)
  learner = Learner(agent, flags, device)
  batch = _map_tensors(make_synthetic_batch(8, 20, (72, 96, 3), 9, seed=5),
                       lambda t: t.to(device))
  grads = []
  for _ in range(2):
    learner.step(batch)
    grads.append(learner.flat.grads.clone())
  torch.cuda.synchronize()
  return grads, learner.flat.params.clone()


@pytest.mark.parametrize('dtype,torso', [('bf16', 'deep'), ('fp32', 'deep'),
                                         ('fp32', 'shallow')])
def test_learner_steps_are_bitwise_reproducible(cuda, dtype, torso):
  C = ops.load()
  old = C.conv_tune('deterministic', -1)
  try:
    g1, p1 = _two_steps(cuda, dtype, torso)
    g2, p2 = _two_steps(cuda, dtype, torso)
  finally:
    C.conv_tune('deterministic', old)
  for a, b in zip(g1, g2):
    assert torch.equal(a, b)
  assert torch.equal(p1, p2)
  assert float(g1[0].abs().sum()) > 0


def test_deterministic_bf16_wgrad_matches_the_atomic_flush(cuda):
  """Slot mode computes the same weight gradients as the atomic flush (up to
  fp32 summation order)."""
  C = ops.load()
  old = C.conv_tune('deterministic', -1)
  try:
    C.conv_tune('deterministic', 0)
    g_atomic, _ = _two_steps(cuda, 'bf16', 'deep', det=False)
    C.conv_tune('deterministic', 1)
    g_slots, _ = _two_steps(cuda, 'bf16', 'deep')
  finally:
    C.conv_tune('deterministic', old)
  a, b = g_atomic[0].double(), g_slots[0].double()
  assert ((a - b).norm() / a.norm()).item() < 1e-5
