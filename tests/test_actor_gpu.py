"""Actor inference on the GPU: the fused heads + Gumbel-max sampler
(csrc/kernels/actor_io.hip) against an fp32 reference and a host Philox, and
the pinned-slab inference server against per-call inference."""

import threading

import numpy as np
import pytest
import torch

from scalable_agent_amd import inference
from scalable_agent_amd.models import Agent

pytestmark = pytest.mark.gpu

M32 = np.uint64(0xFFFFFFFF)


def _philox_u(rows, lanes, offset, seed):
  """Host Philox4x32-10, first output word -> uniform in (0,1) (float64)."""
  c0 = rows.astype(np.uint64)
  c1 = lanes.astype(np.uint64)
  c2 = np.full_like(c0, np.uint64(offset & 0xFFFFFFFF))
  c3 = np.full_like(c0, np.uint64(offset >> 32))
  k0 = np.uint64(seed & 0xFFFFFFFF)
  k1 = np.uint64(seed >> 32)
  for _ in range(10):
    p0 = np.uint64(0xD2511F53) * c0
    p1 = np.uint64(0xCD9E8D57) * c2
    c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ k0, p1 & M32,
                      (p0 >> np.uint64(32)) ^ c3 ^ k1, p0 & M32)
    k0 = (k0 + np.uint64(0x9E3779B9)) & M32
    k1 = (k1 + np.uint64(0xBB67AE85)) & M32
  return ((c0 >> np.uint64(8)).astype(np.float64) + 0.5) / float(1 << 24)


def _ops():
  from scalable_agent_amd import ops
  ops.load()
  return ops


@pytest.mark.parametrize('B,A', [(1, 9), (37, 9), (1024, 18), (5, 32),
                                 (3, 1)])
def test_actor_head_sample_matches_reference(cuda, B, A):
  ops = _ops()
  g = torch.Generator(device=cuda).manual_seed(B * 100 + A)
  h = torch.randn(B, 256, device=cuda, generator=g)
  wp = torch.randn(256, A, device=cuda, generator=g) * 0.1
  bp = torch.randn(A, device=cuda, generator=g)
  wb = torch.randn(256, 1, device=cuda, generator=g) * 0.1
  bb = torch.randn(1, device=cuda, generator=g)
  stream = ops.PhiloxStream(1234567890123)
  stream.offset = 5
  action, logits, baseline = ops.actor_heads_sample(h, wp, bp, wb, bb, stream)
  assert stream.offset == 6
  ref_logits = h.double() @ wp.double() + bp.double()
  ref_base = (h.double() @ wb.double() + bb.double()).squeeze(-1)
  torch.testing.assert_close(logits.double(), ref_logits, atol=1e-4,
                             rtol=1e-4)
  torch.testing.assert_close(baseline.double(), ref_base, atol=1e-4,
                             rtol=1e-4)
  rows = np.repeat(np.arange(B), A)
  lanes = np.tile(np.arange(A), B)
  u = _philox_u(rows, lanes, 5, 1234567890123).reshape(B, A)
  keys = logits.double().cpu().numpy() - np.log(-np.log(u))
  want = keys.argmax(-1)
  got = action.cpu().numpy()
  assert action.dtype == torch.int64 and got.min() >= 0 and got.max() < A
  assert (got == want).mean() >= 0.995
  # same (seed, offset) -> same sample; next offset -> a different draw
  stream.offset = 5
  a2, _, _ = ops.actor_heads_sample(h, wp, bp, wb, bb, stream)
  assert torch.equal(a2, action)


def test_actor_head_sample_distribution(cuda):
  ops = _ops()
  A, B = 6, 8192
  logits_row = torch.tensor([0.5, -1.0, 2.0, 0.0, 1.0, -3.0], device=cuda)
  # h = e_0 and W row 0 = the logits: every row has the same distribution
  h = torch.zeros(B, 256, device=cuda)
  h[:, 0] = 1.0
  wp = torch.zeros(256, A, device=cuda)
  wp[0] = logits_row
  bp = torch.zeros(A, device=cuda)
  wb = torch.zeros(256, 1, device=cuda)
  bb = torch.zeros(1, device=cuda)
  stream = ops.PhiloxStream(7)
  counts = torch.zeros(A, device=cuda)
  for _ in range(8):
    a, _, _ = ops.actor_heads_sample(h, wp, bp, wb, bb, stream)
    counts += torch.bincount(a, minlength=A).float()
  n = float(counts.sum())
  p = torch.softmax(logits_row.double(), 0).cpu().numpy()
  obs = counts.double().cpu().numpy()
  chi2 = float((((obs - n * p) ** 2) / (n * p)).sum())
  assert chi2 < 25.0, (chi2, obs / n, p)  # 5 dof: p(chi2 > 25) < 2e-4


def test_agent_step_fused_sampler(cuda):
  ops = _ops()
  torch.manual_seed(0)
  agent = Agent(9, torso='deep', backend='hip',
                compute_dtype=torch.bfloat16).to(cuda)
  B = 12
  g = torch.Generator(device=cuda).manual_seed(1)
  frame = torch.randint(0, 255, (B, 72, 96, 3), device=cuda,
                        dtype=torch.uint8)
  reward = torch.randn(B, device=cuda)
  done = torch.rand(B, device=cuda) < 0.3
  last = torch.randint(0, 9, (B,), device=cuda)
  state = (torch.randn(B, 256, device=cuda), torch.randn(B, 256, device=cuda))
  from scalable_agent_amd.structs import StepOutput
  eo = StepOutput(reward, None, done, (frame, None))
  with torch.no_grad():
    out_t, st_t = agent.step(last, eo, state, generator=g)
    out_f, st_f = agent.step(last, eo, state,
                             generator=ops.PhiloxStream(3))
  torch.testing.assert_close(out_f.policy_logits, out_t.policy_logits,
                             atol=1e-4, rtol=1e-4)
  torch.testing.assert_close(out_f.baseline, out_t.baseline, atol=1e-4,
                             rtol=1e-4)
  torch.testing.assert_close(st_f[1], st_t[1])
  assert out_f.action.shape == (B,) and out_f.action.dtype == torch.int64


def test_device_counter_stream(cuda):
  ops = _ops()
  h = torch.randn(63, 256, device=cuda)  # a partial last workgroup
  wp = torch.randn(256, 9, device=cuda)
  bp, wb, bb = (torch.zeros(9, device=cuda), torch.zeros(256, 1, device=cuda),
                torch.zeros(1, device=cuda))
  s = ops.PhiloxStream(5, device=cuda)
  a1, _, _ = ops.actor_heads_sample(h, wp, bp, wb, bb, s)
  a2, _, _ = ops.actor_heads_sample(h, wp, bp, wb, bb, s)
  # the kernel advanced its own counter: offset 2, wave count re-armed
  assert s.device_offset == 2 and int(s.counter[1].item()) == 0
  assert s.offset == 0
  host = ops.PhiloxStream(5)
  b1, _, _ = ops.actor_heads_sample(h, wp, bp, wb, bb, host)
  b2, _, _ = ops.actor_heads_sample(h, wp, bp, wb, bb, host)
  assert torch.equal(a1, b1) and torch.equal(a2, b2)
  assert not torch.equal(a1, a2)


@pytest.mark.parametrize('graphs', [True, False])
def test_staged_server_gpu(cuda, graphs):
  torch.manual_seed(0)
  agent = Agent(9, torso='deep', backend='hip', compute_dtype=torch.bfloat16)
  model = inference.InferenceModel(agent, cuda, True, seed=3)
  srv = inference.make_batched_infer(model, 1, 16, 5, graphs=graphs)
  assert isinstance(srv, inference.StagedBatchedInfer)
  assert srv.graphs == graphs
  errors = []

  def actor(i):
    rng = np.random.RandomState(i)
    try:
      for k in range(6):
        ids = np.zeros((1, 16), np.int64)
        n = np.zeros(1, np.int64)
        if i % 3 == 0 and k % 2 == 1:  # some batches carry instructions
          n[0] = 1 + k % 4
          ids[0, :n[0]] = rng.randint(0, 1000, n[0])
        a = (np.array([k % 9], np.int64), np.array([0.5], np.float32),
             np.array([k == 3]),
             rng.randint(0, 255, (1, 72, 96, 3)).astype(np.uint8),
             ids, n,
             rng.rand(1, 256).astype(np.float32),
             rng.rand(1, 256).astype(np.float32))
        o = srv(*a)
        r = model.infer(*a)
        for got, want in zip(o[1:], r[1:]):
          np.testing.assert_allclose(got, want, atol=2e-3, rtol=2e-3)
        assert 0 <= int(o[0][0]) < 9
    except Exception as e:  # pylint: disable=broad-except
      errors.append(e)

  ts = [threading.Thread(target=actor, args=(i,)) for i in range(8)]
  for t in ts:
    t.start()
  for t in ts:
    t.join(120)
  st = srv.stats()
  srv.close()
  srv.join(30)
  assert not errors, errors[0]
  assert st['requests'] == 48


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
def test_inference_weight_cache_tracks_publish(cuda, dtype):
  """An inference agent packs W_h (and on the bf16 path casts the core's FC
  / W_x weights) once per publish (Agent.inference_cache) instead of on
  every step: its step is bitwise that of an uncached agent with the same
  weights, before and after a publish of new weights."""
  _ops()
  from scalable_agent_amd.optim import FlatParams
  from scalable_agent_amd.structs import StepOutput
  mk = lambda seed: Agent(9, torso='deep', backend='hip', seed=seed,
                          compute_dtype=dtype)
  model = inference.InferenceModel(mk(1), cuda, False, seed=3)
  cache = model.agent._inference_cache
  assert cache['w4'] is not None
  assert (cache['w16'] is not None) == (dtype == torch.bfloat16)
  assert (cache['w0pad'] is not None) == (dtype == torch.float32)
  ref, other = mk(1).to(cuda), mk(2).to(cuda)
  assert ref._inference_cache is None
  B = 10
  g = torch.Generator().manual_seed(4)
  frame = torch.randint(0, 255, (B, 72, 96, 3), generator=g,
                        dtype=torch.uint8).to(cuda)
  eo = StepOutput(torch.randn(B, generator=g).to(cuda), None,
                  torch.zeros(B, dtype=torch.bool, device=cuda), (frame, None))
  last = torch.randint(0, 9, (B,), generator=g).to(cuda)
  state = (torch.randn(B, 256, generator=g).to(cuda),
           torch.randn(B, 256, generator=g).to(cuda))

  def run(agent):
    with torch.no_grad():
      out, (c2, h2) = agent.step(last, eo, state,
                                 generator=torch.Generator(cuda).manual_seed(0))
    torch.cuda.synchronize()
    return out.policy_logits, out.baseline, c2, h2

  for a, b in zip(run(model.agent), run(ref)):
    assert torch.equal(a, b)
  model.publish(FlatParams(other).params)
  torch.cuda.synchronize()
  for a, b in zip(run(model.agent), run(other)):
    assert torch.equal(a, b)
