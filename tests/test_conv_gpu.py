"""Fused NHWC conv-torso kernels vs fp32 PyTorch references.

Inputs/weights are rounded to bf16 first so the comparison isolates the
kernels' accumulation order and their (bf16) output rounding.
"""

import pytest
import torch
import torch.nn.functional as F

from scalable_agent_amd.models import layers

pytestmark = pytest.mark.gpu


def _C():
  from scalable_agent_amd import ops
  return ops.ext()


def bf(t):
  return t.to(torch.bfloat16).to(torch.float32)


def conv_ref(x, w, b):
  return layers.conv2d_same_nhwc(x, w, b, 1)


def pads(h, w):
  return layers.same_pads(h, 3, 2)[0], layers.same_pads(w, 3, 2)[0]


def scatter_pool_grad(dP, arg, H, W, pb_h, pb_w):
  N, Hp, Wo, C = dP.shape
  dev = dP.device
  a = arg.long()
  i = torch.arange(Hp, device=dev).view(1, Hp, 1, 1)
  j = torch.arange(Wo, device=dev).view(1, 1, Wo, 1)
  r = 2 * i - pb_h + a // 3
  c = 2 * j - pb_w + a % 3
  n = torch.arange(N, device=dev).view(N, 1, 1, 1).expand_as(a)
  ch = torch.arange(C, device=dev).view(1, 1, 1, C).expand_as(a)
  dY = torch.zeros(N, H, W, C, device=dev)
  dY.index_put_((n.reshape(-1), r.reshape(-1), c.reshape(-1), ch.reshape(-1)),
                dP.float().reshape(-1), accumulate=True)
  return dY


def close(a, b, tol):
  a, b = a.float(), b.float()
  err = (a - b).abs().max().item()
  scale = max(b.abs().max().item(), 1e-6)
  assert err <= tol * scale, 'max err %.4g vs scale %.4g' % (err, scale)


@pytest.mark.parametrize('C,H,W,resid,post,relu_in', [
    (16, 36, 48, False, False, True), (16, 36, 48, True, False, True),
    (32, 18, 24, True, True, True), (32, 9, 12, False, False, True),
    (32, 18, 24, False, False, True),
    # block forms used by the torso: conv1 = relu-in + post-relu, conv2 =
    # plain input + residual (+ post-relu on the last block)
    (16, 36, 48, False, True, True), (16, 36, 48, True, False, False),
    (32, 18, 24, False, True, True), (32, 9, 12, True, True, False),
    (16, 10, 14, True, False, False)])
def test_res_conv_fwd(cuda, C, H, W, resid, post, relu_in):
  torch.manual_seed(0)
  N = 3
  x = torch.randn(N, H, W, C, device=cuda).to(torch.bfloat16)
  w = bf(torch.randn(3, 3, C, C, device=cuda) * 0.1)
  b = torch.randn(C, device=cuda) * 0.1
  r = torch.randn(N, H, W, C, device=cuda).to(torch.bfloat16) if resid else None
  y = _C().res_conv_fwd(x, w, b, r, post, relu_in)
  ref = conv_ref(F.relu(x.float()) if relu_in else x.float(), w, b)
  if resid:
    ref = ref + r.float()
  if post:
    ref = F.relu(ref)
  close(y, ref, 1e-2)


@pytest.mark.parametrize('CIN,COUT,H,W', [(16, 32, 36, 48), (32, 32, 18, 24),
                                          (32, 32, 9, 12), (16, 16, 10, 14)])
def test_conv_pool_fwd(cuda, CIN, COUT, H, W):
  torch.manual_seed(1)
  N = 2
  x = torch.randn(N, H, W, CIN, device=cuda).to(torch.bfloat16)
  w = bf(torch.randn(3, 3, CIN, COUT, device=cuda) * 0.1)
  b = torch.randn(COUT, device=cuda) * 0.1
  pb_h, pb_w = pads(H, W)
  pooled, arg = _C().conv_pool_fwd(x, w, b, pb_h, pb_w)
  y = bf(conv_ref(x.float(), w, b))
  ref = layers.maxpool_same_nhwc(y, 3, 2)
  close(pooled, ref, 1e-2)
  # argmax points at a conv output equal to the pooled value (bf16 rounded)
  Hp, Wo = pooled.shape[1], pooled.shape[2]
  a = arg.long()
  i = torch.arange(Hp, device=cuda).view(1, Hp, 1, 1)
  j = torch.arange(Wo, device=cuda).view(1, 1, Wo, 1)
  rr = (2 * i - pb_h + a // 3).clamp(0, H - 1)
  cc = (2 * j - pb_w + a % 3).clamp(0, W - 1)
  n = torch.arange(N, device=cuda).view(N, 1, 1, 1).expand_as(a)
  ch = torch.arange(COUT, device=cuda).view(1, 1, 1, COUT).expand_as(a)
  picked = y[n, rr, cc, ch]
  close(picked, pooled.float(), 1e-2)


@pytest.mark.parametrize('H,W,C', [(72, 96, 3), (20, 26, 3), (84, 84, 4),
                                   (21, 19, 4)])
def test_conv1_pool_fwd(cuda, H, W, C):
  torch.manual_seed(2)
  N = 3
  frames = torch.randint(0, 256, (N, H, W, C), device=cuda, dtype=torch.uint8)
  w = torch.randn(3, 3, C, 16, device=cuda) * 0.2
  b = torch.randn(16, device=cuda) * 0.1
  pb_h, pb_w = pads(H, W)
  pooled, arg = _C().conv1_pool_fwd(frames, w, b, pb_h, pb_w)
  y = conv_ref(frames.float() / 255.0, w, b)
  ref = layers.maxpool_same_nhwc(y, 3, 2)
  close(pooled, ref, 2e-2)


@pytest.mark.parametrize('C,H,W,skip,relu_act', [
    (16, 36, 48, False, True), (16, 36, 48, True, True),
    (32, 18, 24, True, True), (32, 9, 12, False, True),
    (16, 36, 48, False, False), (32, 18, 24, False, False),
    (32, 9, 12, False, False), (16, 10, 14, False, False)])
def test_res_conv_bwd(cuda, C, H, W, skip, relu_act):
  torch.manual_seed(3)
  N = 3
  act = torch.randn(N, H, W, C, device=cuda).to(torch.bfloat16)
  dy = torch.randn(N, H, W, C, device=cuda).to(torch.bfloat16)
  sk = torch.randn(N, H, W, C, device=cuda).to(torch.bfloat16) if skip else None
  w = bf(torch.randn(3, 3, C, C, device=cuda) * 0.1)
  dw = torch.zeros(3, 3, C, C, device=cuda)
  db = torch.zeros(C, device=cuda)
  if not relu_act:
    act = F.relu(act.float()).to(torch.bfloat16)  # stored post-ReLU
  dx = _C().res_conv_bwd(dy, act, sk, w, dw, db, relu_act)
  a = act.float().requires_grad_(True)
  wr = w.clone().requires_grad_(True)
  br = torch.zeros(C, device=cuda, requires_grad=True)
  out = conv_ref(F.relu(a), wr, br)
  out.backward(dy.float())
  ref_dx = a.grad + (sk.float() if skip else 0)
  close(dx, ref_dx, 1e-2)
  close(dw, wr.grad, 1e-3)
  close(db, br.grad, 1e-3)


@pytest.mark.parametrize('CIN,COUT,H,W', [(16, 32, 36, 48), (32, 32, 18, 24),
                                          (32, 32, 9, 12)])
def test_pool_conv_bwd(cuda, CIN, COUT, H, W):
  torch.manual_seed(4)
  N = 2
  x = torch.randn(N, H, W, CIN, device=cuda).to(torch.bfloat16)
  w = bf(torch.randn(3, 3, CIN, COUT, device=cuda) * 0.1)
  b = torch.randn(COUT, device=cuda) * 0.1
  pb_h, pb_w = pads(H, W)
  pooled, arg = _C().conv_pool_fwd(x, w, b, pb_h, pb_w)
  dP = torch.randn_like(pooled.float()).to(torch.bfloat16)
  dw = torch.zeros(3, 3, CIN, COUT, device=cuda)
  db = torch.zeros(COUT, device=cuda)
  dx = _C().pool_conv_bwd(dP, arg, x, w, dw, db, True, pb_h, pb_w)
  dY = bf(scatter_pool_grad(dP, arg, H, W, pb_h, pb_w))
  xr = x.float().requires_grad_(True)
  wr = w.clone().requires_grad_(True)
  br = torch.zeros(COUT, device=cuda, requires_grad=True)
  conv_ref(xr, wr, br).backward(dY)
  close(dx, xr.grad, 1e-2)
  close(dw, wr.grad, 1e-3)
  close(db, br.grad, 1e-3)


@pytest.mark.parametrize('H,W,C', [(72, 96, 3), (20, 26, 3), (84, 84, 4),
                                   (21, 19, 4)])
def test_conv1_pool_bwd(cuda, H, W, C):
  torch.manual_seed(5)
  N = 2
  frames = torch.randint(0, 256, (N, H, W, C), device=cuda, dtype=torch.uint8)
  w = torch.randn(3, 3, C, 16, device=cuda) * 0.2
  b = torch.randn(16, device=cuda) * 0.1
  pb_h, pb_w = pads(H, W)
  pooled, arg = _C().conv1_pool_fwd(frames, w, b, pb_h, pb_w)
  dP = torch.randn_like(pooled.float()).to(torch.bfloat16)
  dw = torch.zeros(3, 3, C, 16, device=cuda)
  db = torch.zeros(16, device=cuda)
  _C().conv1_pool_bwd(dP, arg, frames, dw, db, pb_h, pb_w)
  dY = bf(scatter_pool_grad(dP, arg, H, W, pb_h, pb_w))
  wr = w.clone().requires_grad_(True)
  br = torch.zeros(16, device=cuda, requires_grad=True)
  conv_ref(frames.float() / 255.0, wr, br).backward(dY)
  close(dw, wr.grad, 5e-3)
  close(db, br.grad, 1e-3)


def _cos(a, b):
  a, b = a.float().reshape(-1), b.float().reshape(-1)
  a, b = a.detach(), b.detach()
  return float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-12))


@pytest.mark.parametrize('shape', [(72, 96, 3), (84, 84, 4)])
def test_deep_torso_matches_fp32_reference(cuda, shape):
  """Whole torso fwd+bwd: the HIP bf16 path must track the fp32 oracle at
  least as well as PyTorch's own bf16 path (MIOpen) does - on DMLab RGB
  frames and on Atari 84x84 4-frame stacks (BASELINE config #2)."""
  from scalable_agent_amd.models import Agent
  from scalable_agent_amd.models.agent import torso_precision
  torch.manual_seed(6)
  mk = lambda **kw: Agent(9, torso='deep', frame_shape=shape, seed=3,
                          **kw).to(cuda)
  ref = mk()
  tbf = mk(compute_dtype=torch.bfloat16)
  hip = mk(backend='hip', compute_dtype=torch.bfloat16)
  assert torso_precision(hip) == 'bf16'
  frames = torch.randint(0, 256, (6,) + shape, device=cuda, dtype=torch.uint8)
  feats = [m.conv_features(frames) for m in (ref, tbf, hip)]
  assert feats[2].shape == feats[0].shape
  assert _cos(feats[2], feats[0]) > 0.999
  g = torch.randn_like(feats[0])
  for f in feats:
    (f.float() * g).sum().backward()
  named = [dict(m.convnet.named_parameters()) for m in (ref, tbf, hip)]
  for n in named[0]:
    c_hip = _cos(named[2][n].grad, named[0][n].grad)
    c_tbf = _cos(named[1][n].grad, named[0][n].grad)
    assert c_hip > min(0.99, c_tbf - 0.01), (n, c_hip, c_tbf)


@pytest.mark.parametrize('frame', [(72, 96, 3), (72, 128, 3), (84, 84, 4)])
def test_specialized_geometry_matches_generic(cuda, frame):
  """Compile-time-geometry kernels (IMPALA 72x96, Doom 72x128 and Atari
  84x84x4 stages, the last with odd 21 / 11 maps and a pool pad-before of 1)
  give the same results as the runtime-geometry kernels."""
  C = _C()
  torch.manual_seed(7)
  N = 2
  H0, W0, CH = frame
  frames = torch.randint(0, 256, (N, H0, W0, CH), device=cuda, dtype=torch.uint8)
  w1 = torch.randn(3, 3, CH, 16, device=cuda) * 0.2
  b16 = torch.randn(16, device=cuda) * 0.1
  b32 = torch.randn(32, device=cuda) * 0.1
  w16 = bf(torch.randn(3, 3, 16, 16, device=cuda) * 0.1)
  w1632 = bf(torch.randn(3, 3, 16, 32, device=cuda) * 0.1)
  w32 = bf(torch.randn(3, 3, 32, 32, device=cuda) * 0.1)
  half = lambda n: (n + 1) // 2
  pb = lambda n: max((half(n) - 1) * 2 + 3 - n, 0) // 2  # SAME pool pad-before
  H1, W1 = half(H0), half(W0)
  H2, W2 = half(H1), half(W1)
  x16 = torch.randn(N, H1, W1, 16, device=cuda).to(torch.bfloat16)
  x32 = torch.randn(N, H2, W2, 32, device=cuda).to(torch.bfloat16)
  x9 = torch.randn(N, half(H2), half(W2), 32, device=cuda).to(torch.bfloat16)

  def run():
    out = []
    p1, a1 = C.conv1_pool_fwd(frames, w1, b16, pb(H0), pb(W0))
    out += [p1, a1]
    out.append(C.res_conv_fwd(x16, w16, b16, x16, False))
    out.append(C.res_conv_fwd(x32, w32, b32, None, False))
    out.append(C.res_conv_fwd(x9, w32, b32, x9, True))
    out.append(C.res_conv_fwd(x16, w16, b16, None, True, True))
    out.append(C.res_conv_fwd(x32, w32, b32, x32, False, False))
    p2, a2 = C.conv_pool_fwd(x16, w1632, b32, pb(H1), pb(W1))
    p3, a3 = C.conv_pool_fwd(x32, w32, b32, pb(H2), pb(W2))
    out += [p2, a2, p3, a3]
    for x, w, b in ((x16, w16, b16), (x32, w32, b32), (x9, w32, b32)):
      dw, db = torch.zeros_like(w, dtype=torch.float32), torch.zeros_like(b)
      out += [C.res_conv_bwd(x, x, x, w, dw, db), dw, db]
      dw2, db2 = torch.zeros_like(dw), torch.zeros_like(db)
      out += [C.res_conv_bwd(x, x, None, w, dw2, db2, False), dw2, db2]
    for (pp, aa, x, w, b, hh, ww) in ((p2, a2, x16, w1632, b32, H1, W1),
                                      (p3, a3, x32, w32, b32, H2, W2)):
      dw, db = torch.zeros_like(w, dtype=torch.float32), torch.zeros_like(b)
      out += [C.pool_conv_bwd(pp, aa, x, w, dw, db, True, pb(hh), pb(ww)), dw, db]
    dw1, db1 = torch.zeros_like(w1), torch.zeros_like(b16)
    C.conv1_pool_bwd(p1, a1, frames, dw1, db1, pb(H0), pb(W0))
    out += [dw1, db1]
    return out

  spec = run()
  old = C.conv_tune('specialize', 0)
  try:
    gen = run()
  finally:
    C.conv_tune('specialize', old)
  for a, b in zip(spec, gen):
    if a.dtype == torch.float32:  # atomically accumulated weight grads
      close(a, b, 1e-4)
    else:
      assert torch.equal(a, b)


@pytest.mark.parametrize('C,H,W,last', [(16, 36, 48, False), (32, 18, 24, False),
                                        (32, 9, 12, True), (16, 10, 14, False),
                                        (32, 7, 5, True)])
def test_res_block_fwd_matches_two_convs(cuda, C, H, W, last):
  """The fused residual-block forward reproduces the two-launch form
  (conv1 with ReLU-in/ReLU-out, conv2 with the skip) exactly."""
  torch.manual_seed(C + H)
  x = torch.randn(3, H, W, C, device=cuda).to(torch.bfloat16)
  w1 = torch.randn(3, 3, C, C, device=cuda) * 0.2
  w2 = torch.randn(3, 3, C, C, device=cuda) * 0.2
  b1 = torch.randn(C, device=cuda) * 0.1
  b2 = torch.randn(C, device=cuda) * 0.1
  t_ref = _C().res_conv_fwd(x, w1, b1, None, True, True)
  y_ref = _C().res_conv_fwd(t_ref, w2, b2, x, last, False)
  t, y = _C().res_block_fwd(x, w1, b1, w2, b2, last)
  assert torch.equal(t, t_ref)
  assert torch.equal(y, y_ref)


@pytest.mark.parametrize('shape', [(72, 96, 3), (84, 84, 4)])
def test_inference_torso_fused_blocks_match_learner_path(cuda, shape):
  """Small no-grad batches (actor inference) run the bf16 torso with the
  fused residual-block kernel (ops/conv.py _DeepTorsoInfer); the learner's
  autograd path runs two convs per block: bitwise the same features."""
  from scalable_agent_amd.models import Agent
  from scalable_agent_amd.ops import conv
  agent = Agent(9, torso='deep', frame_shape=shape, seed=4, backend='hip',
                compute_dtype=torch.bfloat16).to(cuda)
  g = torch.Generator().manual_seed(6)
  frames = torch.randint(0, 256, (37,) + shape, generator=g,
                         dtype=torch.uint8).to(cuda)
  with torch.no_grad():
    f_inf = conv.torso_forward(agent, frames)
  with torch.enable_grad():
    f_lrn = conv.torso_forward(agent, frames)
  assert f_lrn.requires_grad and not f_inf.requires_grad
  assert torch.equal(f_inf, f_lrn.detach())
