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
from scalable_agent_amd.learner import (Learner, batch_to_device, compute_loss,
                                        _map_tensors)
from scalable_agent_amd.models import Agent

pytestmark = pytest.mark.gpu


def _oracle64(torso, cuda, shape=(72, 96, 3), B=4, T=8, aseed=3, bseed=4):
  """float64 loss gradients of the same step (torch ops, no HIP kernels)."""
  flags = flags_lib.default_flags(batch_size=B, unroll_length=T, torso=torso)
  agent = Agent(9, torso=torso, frame_shape=shape, seed=aseed, backend='torch',
                compute_dtype=torch.float64).to(cuda).double()
  batch = batch_to_device(make_synthetic_batch(B, T, shape, 9, seed=bseed), cuda)
  batch = _map_tensors(batch, lambda t: t.double() if t.is_floating_point() else t)
  names, params = zip(*agent.named_parameters())
  loss = compute_loss(agent, batch, flags, use_fused=False)
  grads = torch.autograd.grad(loss, params, allow_unused=True)
  return float(loss), {n: (torch.zeros_like(p) if g is None else g)
                       for n, p, g in zip(names, params, grads)}


def _vs_oracle(res, oracle, name_filter=None):
  """-> {param: relative L2 error of res's gradient vs the fp64 oracle}."""
  out = {}
  for name, _ in res['flat'].named:
    g64 = oracle[1][name]
    g = res['flat'].view_of(res['grads'], name).double()
    if g64.abs().max() == 0:
      continue
    out[name] = ((g - g64).norm() / g64.norm()).item()
  return out


def _step(backend, torso, dtype, cuda, shape=(72, 96, 3), B=4, T=8, aseed=3,
          bseed=4):
  flags = flags_lib.default_flags(batch_size=B, unroll_length=T, torso=torso)
  agent = Agent(9, torso=torso, frame_shape=shape, seed=aseed, backend=backend,
                compute_dtype=dtype)
  learner = Learner(agent, flags, cuda)
  batch = batch_to_device(make_synthetic_batch(B, T, shape, 9, seed=bseed), cuda)
  p0 = learner.flat.params.clone()
  loss = learner.step(batch)
  torch.cuda.synchronize()
  return dict(loss=float(loss), grads=learner.flat.grads.clone(), p0=p0,
              p1=learner.flat.params.clone(), flat=learner.flat,
              health=learner.health())


def _compare(ref, hip, cos_min, rel_max, loss_rel=None):
  assert torch.equal(ref['p0'], hip['p0']), 'different init'
  loss_rel = rel_max if loss_rel is None else loss_rel
  assert abs(hip['loss'] - ref['loss']) <= loss_rel * max(abs(ref['loss']), 1.0)
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
  # the RMSProp update itself (same formula on both sides).  The first
  # update is ~lr * g (~1e-8) on weights of ~1e-1, so p1 - p0 carries fp32
  # quantisation of p1 (ulp ~4e-9): gradients equal to 1e-7 still round a
  # few updates differently, hence the looser bound
  dr = (ref['p1'] - ref['p0']).double()
  dh = (hip['p1'] - hip['p0']).double()
  assert ((dh - dr).norm() / dr.norm()).item() <= max(rel_max, 1e-3)
  return max(worst)


@pytest.mark.parametrize('torso,aseed,bseed', [('deep', 7, 35), ('shallow', 3, 2)])
def test_fp32_hip_learner_step_matches_torch(cuda, torso, aseed, bseed):
  # discontinuity-free (agent, batch) seeds (tests/_discontinuity.py, the
  # ones of test_fp32_hip_learner_matches_fp64): with a max-pool near-tie or
  # a ReLU near-zero in the batch, fp32 torch (MIOpen direct conv) and the
  # HIP kernels (Winograd 3x3 convs) round differently, may branch
  # differently there, and one flip moves a whole local gradient term
  from tests import _discontinuity
  shape = (72, 96, 3)
  probe = Agent(9, torso=torso, frame_shape=shape, seed=aseed)
  frames = make_synthetic_batch(2, 3, shape, 9, seed=bseed).env_outputs.observation[0]
  assert _discontinuity.count(probe, frames.reshape((-1,) + shape)) == 0
  kw = dict(B=2, T=3, aseed=aseed, bseed=bseed)
  ref = _step('torch', torso, torch.float32, cuda, **kw)
  hip = _step('hip', torso, torch.float32, cuda, **kw)
  worst = _compare(ref, hip, cos_min=0.999999, rel_max=1e-4)
  print('fp32 %s worst relative gradient error %.3g (%s)' % (torso, worst[0], worst[1]))
  assert hip['health'] == {'skipped_updates': 0, 'lstm_timeouts': 0,
                                'conv_timeouts': 0}


# (agent seed, batch seed) whose float64 forward has no pool near-tie /
# ReLU near-zero (tests/_discontinuity.py): fp32 and float64 may branch
# differently there, and one flip moves a whole local gradient
@pytest.mark.parametrize('torso,shape,aseed,bseed', [
    ('deep', (72, 96, 3), 7, 35), ('shallow', (72, 96, 3), 3, 2),
    ('deep', (84, 84, 4), 3, 30), ('shallow', (84, 84, 4), 3, 0)])
def test_fp32_hip_learner_matches_fp64(cuda, torso, shape, aseed, bseed):
  """One fp32 HIP learner step against the float64 oracle of the same step:
  loss and every parameter gradient to fp32 accuracy (<= 2e-5 relative L2),
  next to the torch fp32 learner's own error for comparison."""
  from tests import _discontinuity
  kw = dict(shape=shape, B=2, T=3, aseed=aseed, bseed=bseed)
  probe = Agent(9, torso=torso, frame_shape=shape, seed=aseed)
  frames = make_synthetic_batch(2, 3, shape, 9, seed=bseed).env_outputs.observation[0]
  assert _discontinuity.count(probe, frames.reshape((-1,) + shape)) == 0
  oracle = _oracle64(torso, cuda, **kw)
  ref = _step('torch', torso, torch.float32, cuda, **kw)
  hip = _step('hip', torso, torch.float32, cuda, **kw)
  assert abs(hip['loss'] - oracle[0]) <= 1e-5 * max(1.0, abs(oracle[0]))
  e_hip, e_ref = _vs_oracle(hip, oracle), _vs_oracle(ref, oracle)
  for name in e_hip:
    print('%-40s hip %.2e  torch %.2e' % (name, e_hip[name], e_ref[name]))
  for name in e_hip:
    # a flip both fp32 learners share (rounding of the uint8/255 input or of
    # a long sum) bounds fp32-vs-fp64 agreement from below
    assert e_hip[name] <= max(2e-5, 1.5 * e_ref[name]), (name, e_hip[name], e_ref[name])


def test_bf16_hip_learner_step_tracks_fp64(cuda):
  """bf16 operands (fp32 accumulation/state): every gradient keeps cosine
  >= 0.99 to the float64 oracle.  The heavily cancelling early-conv weight
  gradients are the loosest (that is why the headline runs fp32)."""
  oracle = _oracle64('deep', cuda)
  hip = _step('hip', 'deep', torch.bfloat16, cuda)
  worst = 1.0
  for name, _ in hip['flat'].named:
    g64 = oracle[1][name]
    if g64.abs().max() == 0:
      continue
    g = hip['flat'].view_of(hip['grads'], name).double()
    cos = torch.nn.functional.cosine_similarity(g.reshape(1, -1),
                                                g64.reshape(1, -1)).item()
    print('%-40s cos %.5f' % (name, cos))
    worst = min(worst, cos)
    assert cos >= 0.99, (name, cos)


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
    assert learner.health() == {'skipped_updates': 1, 'lstm_timeouts': 1,
                                'conv_timeouts': 0}
  finally:
    lstm_ops.set_gang_fault(prev_fault)
  try:
    # the word was consumed: the next healthy step applies normally
    assert lstm_ops.persistent_error(cuda) == 0
    learner.step(batch)
    torch.cuda.synchronize()
    assert not torch.equal(learner.flat.params, p0)
    assert learner.health() == {'skipped_updates': 1, 'lstm_timeouts': 1,
                                'conv_timeouts': 0}
  finally:
    lstm_ops.set_gang(prev_gang)


def test_conv_handoff_timeout_skips_update(cuda):
  """The fused Winograd backward's bounded LDS hand-off wait (the 16->32
  stage head, conv_wino.hip) fails loud: with the fault injected every wait
  'expires', the sticky conv error word is set, the RMSProp guard skips the
  update and counts it as a conv timeout; the next healthy step applies."""
  from scalable_agent_amd.ops import _ext
  flags = flags_lib.default_flags(batch_size=4, unroll_length=8, torso='deep')
  agent = Agent(9, torso='deep', seed=3, backend='hip',
                compute_dtype=torch.float32)
  learner = Learner(agent, flags, cuda)
  batch = batch_to_device(make_synthetic_batch(4, 8, (72, 96, 3), 9, seed=4), cuda)
  prev = _ext.ext().cf32_wino_fault(1)
  try:
    p0 = learner.flat.params.clone()
    learner.step(batch)
    torch.cuda.synchronize()
    assert torch.equal(learner.flat.params, p0), 'stale-gradient update applied'
    assert learner.health() == {'skipped_updates': 1, 'lstm_timeouts': 0,
                                'conv_timeouts': 1}
  finally:
    _ext.ext().cf32_wino_fault(prev)
  learner.step(batch)
  torch.cuda.synchronize()
  assert not torch.equal(learner.flat.params, p0)
  assert learner.health() == {'skipped_updates': 1, 'lstm_timeouts': 0,
                              'conv_timeouts': 1}
