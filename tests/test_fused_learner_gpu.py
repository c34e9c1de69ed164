"""Fused learner ops (csrc/kernels/learner_io.hip, ops/core.py, ops/heads.py)
against fp32 PyTorch references of the same math."""

import pytest
import torch
import torch.nn.functional as F

from scalable_agent_amd import flags as flags_lib
from scalable_agent_amd import losses as losses_lib
from scalable_agent_amd import vtrace as vtrace_lib
from scalable_agent_amd.envs.synthetic import (add_synthetic_instructions,
                                                make_synthetic_batch)
from scalable_agent_amd.learner import Learner, batch_to_device, compute_loss
from scalable_agent_amd.models import Agent

pytestmark = pytest.mark.gpu


def _ops():
  from scalable_agent_amd import ops
  ops.load()
  return ops


def _cos(a, b):
  a, b = a.detach().float().reshape(-1), b.detach().float().reshape(-1)
  return float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-12))


def _ref_loss(core, wp, bp, wb, bb, beh, act, rew, done, clip, bc, ec):
  logits = core @ wp + bp
  values = (core @ wb + bb).squeeze(-1)
  discounts = (~done[1:]).float() * 0.99
  vt = vtrace_lib.from_logits(
      behaviour_policy_logits=beh[1:], target_policy_logits=logits[:-1],
      actions=act[1:], discounts=discounts,
      rewards=losses_lib.clip_rewards(rew[1:], clip), values=values[:-1],
      bootstrap_value=values[-1])
  total = losses_lib.compute_policy_gradient_loss(logits[:-1], act[1:],
                                                  vt.pg_advantages)
  total = total + bc * losses_lib.compute_baseline_loss(vt.vs - values[:-1])
  return total + ec * losses_lib.compute_entropy_loss(logits[:-1])


@pytest.mark.parametrize('T,B,A,clip', [(100, 32, 9, 'abs_one'),
                                        (7, 3, 5, 'soft_asymmetric'),
                                        (300, 2, 18, 'abs_one')])
def test_heads_vtrace_loss_matches_reference(cuda, T, B, A, clip):
  ops = _ops()
  torch.manual_seed(11)
  T1 = T + 1
  core = torch.randn(T1, B, 256, device=cuda, requires_grad=True)
  wp = (torch.randn(256, A, device=cuda) * 0.05).requires_grad_()
  bp = (torch.randn(A, device=cuda) * 0.1).requires_grad_()
  wb = (torch.randn(256, 1, device=cuda) * 0.05).requires_grad_()
  bb = (torch.randn(1, device=cuda) * 0.1).requires_grad_()
  beh = torch.randn(T1, B, A, device=cuda)
  act = torch.randint(0, A, (T1, B), device=cuda)
  rew = torch.randn(T1, B, device=cuda) * 2
  done = torch.rand(T1, B, device=cuda) < 0.05
  leaves = [core, wp, bp, wb, bb]
  ref = _ref_loss(core, wp, bp, wb, bb, beh, act, rew, done, clip, 0.5, 0.01)
  (2.0 * ref).backward()
  gref = [t.grad.clone() for t in leaves]
  for t in leaves:
    t.grad = None
  loss = ops.heads_vtrace_loss(core, wp, bp, wb, bb, beh, act, rew, done,
                               0.99, clip, 0.5, 0.01)
  torch.testing.assert_close(loss, ref, rtol=1e-4, atol=1e-3)
  (2.0 * loss).backward()
  for t, g in zip(leaves, gref):
    torch.testing.assert_close(t.grad, g, rtol=1e-3, atol=1e-4)
  # deterministic loss (fixed-order ticket reduction), repeatable launches
  l2 = ops.heads_vtrace_loss(core, wp, bp, wb, bb, beh, act, rew, done, 0.99,
                             clip, 0.5, 0.01)
  assert torch.equal(l2, loss)
  # direct accumulation into existing .grad buffers
  for t in (wp, bp, wb, bb):
    t.grad = torch.ones_like(t)
  core.grad = None
  with ops.direct_grads():
    ops.heads_vtrace_loss(core, wp, bp, wb, bb, beh, act, rew, done, 0.99,
                          clip, 0.5, 0.01).backward()
  for t, g in zip(leaves[1:], gref[1:]):
    torch.testing.assert_close(t.grad, 1.0 + 0.5 * g, rtol=1e-3, atol=1e-4)


def _ref_popart_loss(core, wp, bp, wb, bb, beh, act, rew, done, task, popart,
                     bc, ec):
  """compute_loss's generic PopArt path (learner.py) on given core outputs."""
  logits = core @ wp + bp
  values_all = core @ wb + bb                      # [T1, B, K]
  idx = task.view(1, -1, 1).expand(values_all.shape[0], -1, 1)
  n = values_all.gather(-1, idx).squeeze(-1)       # normalised values
  sigma, mu = popart.stats_for(task)
  sigma, mu = sigma.to(core.dtype), mu.to(core.dtype)
  values = n[:-1] * sigma + mu
  boot = n[-1] * sigma + mu
  discounts = (~done[1:]).to(core.dtype) * 0.99
  vt = vtrace_lib.from_logits(
      behaviour_policy_logits=beh[1:], target_policy_logits=logits[:-1],
      actions=act[1:], discounts=discounts,
      rewards=losses_lib.clip_rewards(rew[1:], 'abs_one'), values=values,
      bootstrap_value=boot)
  err = (vt.vs - mu) / sigma - n[:-1]
  total = losses_lib.compute_policy_gradient_loss(
      logits[:-1], act[1:], vt.pg_advantages / sigma)
  total = total + bc * losses_lib.compute_baseline_loss(err)
  return total + ec * losses_lib.compute_entropy_loss(logits[:-1]), vt.vs


@pytest.mark.parametrize('T,B,K', [(100, 32, 30), (9, 5, 3)])
def test_heads_vtrace_loss_popart_matches_reference(cuda, T, B, K):
  """Multi-task PopArt in the fused head kernels (K value heads, the task
  column of each batch column, de-normalised V-trace, normalised baseline
  error and advantages) against the generic torch path in float64."""
  from scalable_agent_amd.popart import PopArt
  ops = _ops()
  torch.manual_seed(5)
  T1, A = T + 1, 9
  pa = PopArt(K, device=cuda)
  pa.mu.copy_(torch.randn(K, device=cuda) * 3)
  pa.nu.copy_(pa.mu * pa.mu + torch.rand(K, device=cuda) * 20 + 0.5)
  core = torch.randn(T1, B, 256, device=cuda)
  wp = torch.randn(256, A, device=cuda) * 0.05
  bp = torch.randn(A, device=cuda) * 0.1
  wb = torch.randn(256, K, device=cuda) * 0.05
  bb = torch.randn(K, device=cuda) * 0.1
  beh = torch.randn(T1, B, A, device=cuda)
  act = torch.randint(0, A, (T1, B), device=cuda)
  rew = torch.randn(T1, B, device=cuda) * 2
  done = torch.rand(T1, B, device=cuda) < 0.05
  task = torch.randint(0, K, (B,), device=cuda)
  leaves64 = [t.double().requires_grad_() for t in (core, wp, bp, wb, bb)]
  ref, vs_ref = _ref_popart_loss(*leaves64, beh.double(), act, rew.double(),
                                 done, task, pa, 0.5, 0.01)
  (2.0 * ref).backward()
  leaves = [t.clone().requires_grad_() for t in (core, wp, bp, wb, bb)]
  aux = {}
  loss = ops.heads_vtrace_loss(*leaves, beh, act, rew, done, 0.99, 'abs_one',
                               0.5, 0.01, task_ids=task, popart=pa, aux=aux)
  torch.testing.assert_close(loss.double(), ref.detach(), rtol=1e-4, atol=1e-3)
  torch.testing.assert_close(aux['targets'].double(), vs_ref, rtol=1e-4, atol=1e-4)
  (2.0 * loss).backward()
  for t, r in zip(leaves, leaves64):
    g, gr = t.grad.double(), r.grad
    assert ((g - gr).norm() / gr.norm().clamp_min(1e-30)).item() <= 1e-4
  # only the heads the batch uses get a value-head gradient
  unused = torch.ones(K, dtype=torch.bool, device=cuda)
  unused[task] = False
  assert torch.all(leaves[3].grad[:, unused] == 0)
  assert torch.all(leaves[4].grad[unused] == 0)


def test_popart_learner_uses_fused_heads(cuda):
  """A --popart HIP learner step runs the fused head kernels (no torch
  V-trace) and keeps PopArt's statistics and preserved outputs updating."""
  flags = flags_lib.default_flags(batch_size=4, unroll_length=8, torso='deep',
                                  popart=True)
  agent = Agent(9, torso='deep', seed=1, backend='hip', num_value_heads=5)
  learner = Learner(agent, flags, cuda)
  batch = make_synthetic_batch(4, 8, (72, 96, 3), 9, seed=3)
  batch = batch._replace(level_name=torch.tensor([0, 3, 3, 1]))
  batch = batch_to_device(batch, cuda)
  calls = []
  from scalable_agent_amd.ops import heads as heads_mod
  orig = heads_mod.heads_vtrace_loss
  import scalable_agent_amd.ops as ops_pkg
  def spy(*a, **k):
    calls.append(k.get('popart') is not None)
    return orig(*a, **k)
  ops_pkg.heads_vtrace_loss = spy
  try:
    mu0 = learner.popart.mu.clone()
    loss = learner.step(batch)
    torch.cuda.synchronize()
  finally:
    ops_pkg.heads_vtrace_loss = orig
  assert calls == [True]
  assert torch.isfinite(loss).item()
  changed = (learner.popart.mu != mu0).cpu()
  assert changed.tolist() == [True, True, False, True, False]


def _ref_lstm(x, done, c, h, kernel, bias):
  F_in = x.shape[-1]
  kx, kh = kernel[:F_in], kernel[F_in:]
  outs = []
  for t in range(x.shape[0]):
    keep = (~done[t]).float().unsqueeze(-1)
    c = c * keep
    h = h * keep
    g = x[t] @ kx + bias + h @ kh
    i, ci, f, o = g.chunk(4, -1)
    c = torch.tanh(ci) * torch.sigmoid(i) + c * torch.sigmoid(f + 1.0)
    h = torch.tanh(c) * torch.sigmoid(o)
    outs.append(h)
  return torch.stack(outs), c


@pytest.mark.parametrize('T,B,A', [(26, 32, 9), (5, 3, 4)])
def test_core_lstm_matches_reference(cuda, T, B, A):
  """relu(feats W_fc + b) -> [h, clip(r), one_hot(a), 0] -> LSTM: the fused
  op (bf16 GEMMs, fp32 recurrence) against the fp32 reference on the same
  bf16-rounded inputs."""
  ops = _ops()
  torch.manual_seed(5)
  N, Fd = T * B, 3456
  f_in = 256 + 1 + A + 64
  feats = torch.randn(N, Fd, device=cuda).relu().bfloat16().requires_grad_()
  w_fc = (torch.randn(Fd, 256, device=cuda) * 0.02).requires_grad_()
  b_fc = (torch.randn(256, device=cuda) * 0.1).requires_grad_()
  kernel = (torch.randn(f_in + 256, 1024, device=cuda) * 0.05).requires_grad_()
  bias = (torch.randn(1024, device=cuda) * 0.1).requires_grad_()
  rew = torch.randn(N, device=cuda) * 2
  act = torch.randint(0, A, (N,), device=cuda)
  done = torch.rand(T, B, device=cuda) < 0.1
  c0 = torch.randn(B, 256, device=cuda) * 0.3
  h0 = torch.randn(B, 256, device=cuda) * 0.3
  leaves = [feats, w_fc, b_fc, kernel, bias]
  bfr = lambda t: t.bfloat16().float()
  h = F.relu(feats.float() @ bfr(w_fc) + bfr(b_fc))
  x = torch.cat([h, rew.clamp(-1, 1).unsqueeze(1),
                 F.one_hot(act, A).float(),
                 torch.zeros(N, 64, device=cuda)], 1).view(T, B, -1)
  kx = torch.cat([bfr(kernel[:f_in]), kernel[f_in:]], 0)
  hs_ref, c_ref = _ref_lstm(x, done, c0, h0, kx, bias)
  go = torch.randn_like(hs_ref)
  (hs_ref * go).sum().backward()
  gref = [t.grad.clone() for t in leaves]
  for t in leaves:
    t.grad = None
  hs, (c_last, _) = ops.core_lstm(feats, w_fc, b_fc, kernel, bias, rew, act,
                                  done, (c0, h0), A)
  assert (hs - hs_ref).abs().max() < 2e-2
  assert _cos(hs, hs_ref) > 0.9999
  (hs * go).sum().backward()
  for name, t, g in zip(['feats', 'w_fc', 'b_fc', 'kernel', 'bias'], leaves,
                        gref):
    assert _cos(t.grad, g) > 0.999, (name, _cos(t.grad, g))
  # the instruction rows past the aug padding get no gradient at all
  K = ops.core.aug_width(A)
  assert torch.count_nonzero(kernel.grad[257 + A:f_in]) == 0
  assert K <= f_in


@pytest.mark.parametrize('T,B,A', [(26, 32, 9), (5, 3, 4)])
def test_core_lstm_with_instructions_matches_reference(cuda, T, B, A):
  """The fused core with the 64 language-LSTM columns in the core input
  (instruction levels): outputs, every weight gradient and the gradient
  into the instruction encoding against the fp32 reference."""
  ops = _ops()
  torch.manual_seed(7)
  N, Fd = T * B, 3456
  f_in = 256 + 1 + A + 64
  feats = torch.randn(N, Fd, device=cuda).relu().bfloat16().requires_grad_()
  w_fc = (torch.randn(Fd, 256, device=cuda) * 0.02).requires_grad_()
  b_fc = (torch.randn(256, device=cuda) * 0.1).requires_grad_()
  kernel = (torch.randn(f_in + 256, 1024, device=cuda) * 0.05).requires_grad_()
  bias = (torch.randn(1024, device=cuda) * 0.1).requires_grad_()
  enc = (torch.randn(N, 64, device=cuda) * 0.5).tanh().requires_grad_()
  rew = torch.randn(N, device=cuda) * 2
  act = torch.randint(0, A, (N,), device=cuda)
  done = torch.rand(T, B, device=cuda) < 0.1
  c0 = torch.randn(B, 256, device=cuda) * 0.3
  h0 = torch.randn(B, 256, device=cuda) * 0.3
  leaves = [feats, w_fc, b_fc, kernel, bias, enc]
  bfr = lambda t: t.bfloat16().float()
  h = F.relu(feats.float() @ bfr(w_fc) + bfr(b_fc))
  x = torch.cat([h, rew.clamp(-1, 1).unsqueeze(1), F.one_hot(act, A).float(),
                 bfr(enc)], 1).view(T, B, -1)
  kx = torch.cat([bfr(kernel[:f_in]), kernel[f_in:]], 0)
  hs_ref, _ = _ref_lstm(x, done, c0, h0, kx, bias)
  go = torch.randn_like(hs_ref)
  (hs_ref * go).sum().backward()
  gref = [t.grad.clone() for t in leaves]
  for t in leaves:
    t.grad = None
  hs, _ = ops.core_lstm(feats, w_fc, b_fc, kernel, bias, rew, act, done,
                        (c0, h0), A, instr_enc=enc)
  assert _cos(hs, hs_ref) > 0.9999
  (hs * go).sum().backward()
  for name, t, g in zip(['feats', 'w_fc', 'b_fc', 'kernel', 'bias', 'enc'],
                        leaves, gref):
    assert _cos(t.grad, g) > 0.999, (name, _cos(t.grad, g))
  # the instruction rows of W_x do receive gradient now
  assert torch.count_nonzero(kernel.grad[257 + A:f_in]) > 0


@pytest.mark.parametrize('instructions', [False, True])
def test_fused_learner_loss_matches_generic_hip_path(cuda, instructions):
  """compute_loss on the fused path vs the per-op HIP path (torso + torch FC
  + lstm_unroll + fused V-trace kernel) on the same agent."""
  _ops()
  f = flags_lib.default_flags(batch_size=4, unroll_length=12)
  b = make_synthetic_batch(4, 12, (72, 96, 3), 9, seed=2)
  agent = Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=4,
                backend='hip', compute_dtype=torch.bfloat16)
  if instructions:
    b = add_synthetic_instructions(b, agent.embed.shape[0], seed=3)
  b = batch_to_device(b, cuda)
  lrn = Learner(agent, f, cuda)
  out = []
  for fused in (True, False):
    lrn.flat.zero_grad()
    if fused:
      loss = compute_loss(agent, b, f, use_fused=True)
    else:
      agent.fused_core_ready = lambda instr=None: False
      loss = compute_loss(agent, b, f, use_fused=True)
      del agent.fused_core_ready
    loss.backward()
    torch.cuda.synchronize()
    out.append((loss.detach().clone(), lrn.flat.grads.clone()))
  (l1, g1), (l2, g2) = out
  torch.testing.assert_close(l1, l2, rtol=2e-3, atol=2e-2)
  assert _cos(g1, g2) > 0.999
  if instructions:  # the language LSTM and embedding get gradient
    emb = lrn.flat.view_of(lrn.flat.grads, 'embed')
    assert float(emb.abs().sum()) > 0


@pytest.mark.parametrize('N,C,ld', [(3232, 256, 272), (37, 16, 16), (5, 64, 80)])
def test_glue_kernels_match_torch(cuda, N, C, ld):
  """relu_bwd_colsum_ (masked in place + column sums, strided y), relu_mask,
  colsum and core_aug against plain PyTorch."""
  C_ = _ops().ext()
  torch.manual_seed(N)
  dy = torch.randn(N, C, device=cuda).bfloat16()
  yfull = torch.randn(N, ld, device=cuda).bfloat16()
  y = yfull[:, :C]
  ref = dy.float() * (y.float() > 0)
  out = torch.ones(C, device=cuda)
  C_.relu_bwd_colsum_(dy, y, out)
  torch.testing.assert_close(dy.float(), ref)
  torch.testing.assert_close(out, 1 + ref.sum(0), rtol=1e-4, atol=1e-3)
  x = torch.randn(N, C, device=cuda)
  s = torch.zeros(C, device=cuda)
  C_.colsum_f32_(x, s)
  torch.testing.assert_close(s, x.sum(0), rtol=1e-4, atol=1e-3)
  if (N * C) % 8 == 0:
    d2 = torch.randn(N, C, device=cuda).bfloat16()
    r2 = d2 * (yfull[:, :C].contiguous() > 0)
    C_.relu_mask_bf16_(d2, yfull[:, :C].contiguous())
    assert torch.equal(d2, r2)
  h = torch.randn(N, C, device=cuda).bfloat16()
  rw = torch.randn(N, device=cuda) * 3
  act = torch.randint(0, 5, (N,), device=cuda)
  aug = C_.core_aug_fwd(h, rw, act, C + 16, 0)
  assert torch.equal(aug[:, :C], h)
  assert torch.equal(aug[:, C].float(), rw.clamp(-1, 1).bfloat16().float())
  oh = torch.nn.functional.one_hot(act, 15).bfloat16()
  assert torch.equal(aug[:, C + 1:], oh)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_instruction_learner_graph_replay_matches_eager(cuda, dtype):
  """Instruction levels under hipGraph capture (more than 3072 word lookups:
  the embedding gradient must be a fixed-size scatter, not a data-sized
  sort/compact): replayed steps match eager steps from the same state."""
  _ops()
  f = flags_lib.default_flags(batch_size=8, unroll_length=30)
  mk = lambda: Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=4,
                     backend='hip', compute_dtype=dtype)
  ref_agent = mk()
  b = make_synthetic_batch(8, 30, (72, 96, 3), 9, seed=2)
  b = batch_to_device(add_synthetic_instructions(b, ref_agent.embed.shape[0],
                                                 seed=3), cuda)
  eager = Learner(ref_agent, f, cuda)
  graph = Learner(mk(), f, cuda)
  graph.capture(b)
  losses = []
  for _ in range(2):
    le = eager.step(b)
    lg = graph.graph_step()
    losses.append((float(le), float(lg)))
  torch.cuda.synchronize()
  for le, lg in losses:
    assert abs(le - lg) <= 1e-3 * max(1.0, abs(le)), losses
  emb_e = eager.flat.view_of(eager.flat.params, 'embed')
  emb_g = graph.flat.view_of(graph.flat.params, 'embed')
  assert torch.allclose(emb_e, emb_g, rtol=1e-4, atol=1e-6)
