"""One whole HIP learner step against the pure-PyTorch fp32 learner.

Same init, same batch, one `Learner.step` each (re-unroll, V-trace, losses,
backward, TF-RMSProp; reference experiment.py:346-427).  The fp32 HIP path
(exact-fp32 MFMA conv kernels, fp32 LSTM recurrence, fused V-trace/loss,
fused RMSProp) must match the torch learner to fp32 accuracy; the bf16 path
to bf16-operand accuracy.  Also: a cooperative-LSTM timeout (fault-injected)
skips the update and is counted instead of applying stale gradients.
"""

import pytest
import torch

from scalable_agent_amd import flags as flags_lib
from scalable_agent_amd.envs.synthetic import make_synthetic_batch
from scalable_agent_amd.learner import Learner, batch_to_device
from scalable_agent_amd.models import Agent

pytestmark = pytest.mark.gpu


def _step(backend, torso, dtype, cuda, shape=(72, 96, 3), B=4, T=8):
  flags = flags_lib.default_flags(batch_size=B, unroll_length=T, torso=torso)
  agent = Agent(9, torso=torso, frame_shape=shape, seed=3, backend=backend,
                compute_dtype=dtype)
  learner = Learner(agent, flags, cuda)
  batch = batch_to_device(make_synthetic_batch(B, T, shape, 9, seed=4), cuda)
  p0 = learner.flat.params.clone()
  loss = learner.step(batch)
  torch.cuda.synchronize()
  return dict(loss=float(loss), grads=learner.flat.grads.clone(), p0=p0,
              p1=learner.flat.params.clone(), flat=learner.flat,
              health=learner.health())


def _compare(ref, hip, cos_min, rel_max):
  assert torch.equal(ref['p0'], hip['p0']), 'different init'
  assert abs(hip['loss'] - ref['loss']) <= rel_max * max(abs(ref['loss']), 1.0)
  worst = []
  for name, _ in ref['flat'].named:
    gr = ref['flat'].view_of(ref['grads'], name).double()
    gh = hip['flat'].view_of(hip['grads'], name).double()
    if gr.abs().max() == 0:
      assert gh.abs().max() == 0, name
      continue
    cos = torch.nn.functional.cosine_similarity(gr.reshape(1, -1),
                                                gh.reshape(1, -1)).item()
    rel = ((gh - gr).norm() / gr.norm()).item()
    worst.append((rel, name, cos))
    assert cos >= cos_min, (name, cos)
    assert rel <= rel_max, (name, rel)
  # the RMSProp update itself (same formula on both sides)
  dr = (ref['p1'] - ref['p0']).double()
  dh = (hip['p1'] - hip['p0']).double()
  assert ((dh - dr).norm() / dr.norm()).item() <= rel_max
  return max(worst)


@pytest.mark.parametrize('torso', ['deep', 'shallow'])
def test_fp32_hip_learner_step_matches_torch(cuda, torso):
  ref = _step('torch', torso, torch.float32, cuda)
  hip = _step('hip', torso, torch.float32, cuda)
  worst = _compare(ref, hip, cos_min=0.999999, rel_max=1e-4)
  print('fp32 %s worst relative gradient error %.3g (%s)' % (torso, worst[0], worst[1]))
  assert hip['health'] == {'skipped_updates': 0, 'lstm_timeouts': 0}


def test_fp32_hip_learner_step_atari_shape(cuda):
  """Atari-shaped 84x84x4 frames (BASELINE config #2) on the HIP learner."""
  ref = _step('torch', 'deep', torch.float32, cuda, shape=(84, 84, 4))
  hip = _step('hip', 'deep', torch.float32, cuda, shape=(84, 84, 4))
  _compare(ref, hip, cos_min=0.999999, rel_max=1e-4)


def test_bf16_hip_learner_step_tracks_torch_fp32(cuda):
  ref = _step('torch', 'deep', torch.float32, cuda)
  hip = _step('hip', 'deep', torch.bfloat16, cuda)
  worst = _compare(ref, hip, cos_min=0.999, rel_max=0.05)
  print('bf16 deep worst relative gradient error %.3g (%s)' % (worst[0], worst[1]))


def test_gang_lstm_timeout_skips_update(cuda):
  from scalable_agent_amd.ops import lstm as lstm_ops
  flags = flags_lib.default_flags(batch_size=4, unroll_length=8, torso='deep')
  agent = Agent(9, torso='deep', seed=3, backend='hip', compute_dtype=torch.bfloat16)
  learner = Learner(agent, flags, cuda)
  batch = batch_to_device(make_synthetic_batch(4, 8, (72, 96, 3), 9, seed=4), cuda)
  prev_gang = lstm_ops.set_gang(True)
  prev_fault = lstm_ops.set_gang_fault(True)
  try:
    p0 = learner.flat.params.clone()
    learner.step(batch)
    torch.cuda.synchronize()
    assert torch.equal(learner.flat.params, p0), 'stale-gradient update applied'
    assert learner.health() == {'skipped_updates': 1, 'lstm_timeouts': 1}
  finally:
    lstm_ops.set_gang_fault(prev_fault)
  try:
    # the word was consumed: the next healthy step applies normally
    assert lstm_ops.persistent_error(cuda) == 0
    learner.step(batch)
    torch.cuda.synchronize()
    assert not torch.equal(learner.flat.params, p0)
    assert learner.health() == {'skipped_updates': 1, 'lstm_timeouts': 1}
  finally:
    lstm_ops.set_gang(prev_gang)
