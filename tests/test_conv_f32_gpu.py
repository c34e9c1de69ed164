"""Exact-fp32 conv kernels (csrc/kernels/conv_f32.hip) vs float64 PyTorch.

Every layer shape of both torsos (reference experiment.py:156-189: shallow
8x8/4, 4x4/2, 3x3/2 with the asymmetric W pad; deep 3x3/1 stages, 3x3/2
max-pool) plus the Atari-shaped 84x84x4 and Doom-shaped 72x128x3 inputs:
forward (with the fused ReLU-in / residual / ReLU-out), data gradient (fused
mask + skip add), weight + bias gradient (deterministic reduction) and the
pool.  The oracle is the float64 TF-SAME reference of models/layers.py on
the CPU; the fp32 kernels must agree to <= 1e-5 of the output scale.
"""

import pytest
import torch

from scalable_agent_amd.models import layers

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _C():
  from scalable_agent_amd import ops
  return ops.ext()


def rel_err(a, ref):
  a = a.detach().double().cpu()
  ref = ref.detach().double().cpu()
  return (a - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)


# (N, H, W, Cin, Cout, K, S, uint8 source)
SHAPES = {
    'shallow1': (3, 72, 96, 3, 32, 8, 4, True),
    'shallow2': (3, 18, 24, 32, 64, 4, 2, False),
    'shallow3': (3, 9, 12, 64, 128, 3, 2, False),   # W pad 0/1
    'deep_conv1': (3, 72, 96, 3, 16, 3, 1, True),
    'deep_conv2': (3, 36, 48, 16, 32, 3, 1, False),
    'deep_res16': (3, 36, 48, 16, 16, 3, 1, False),
    'deep_res32': (3, 18, 24, 32, 32, 3, 1, False),
    'deep_res32_s3': (3, 9, 12, 32, 32, 3, 1, False),
    'atari_deep_conv1': (2, 84, 84, 4, 16, 3, 1, True),
    'atari_deep_res32': (2, 11, 11, 32, 32, 3, 1, False),
    'atari_shallow1': (2, 84, 84, 4, 32, 8, 4, True),
    'atari_shallow2': (2, 21, 21, 32, 64, 4, 2, False),
    'atari_shallow3': (2, 11, 11, 64, 128, 3, 2, False),
    'doom_deep_conv1': (2, 72, 128, 3, 16, 3, 1, True),
}


def _make(name, cuda, seed=0):
  N, H, W, Cin, Cout, K, S, u8 = SHAPES[name]
  g = torch.Generator().manual_seed(seed)
  if u8:
    x = torch.randint(0, 256, (N, H, W, Cin), generator=g, dtype=torch.uint8)
    x64 = x.double() / 255.0
  else:
    x = torch.randn(N, H, W, Cin, generator=g)
    x64 = x.double()
  w = torch.randn(K, K, Cin, Cout, generator=g) / (K * K * Cin) ** 0.5
  b = torch.randn(Cout, generator=g) * 0.1
  pt, pl = layers.same_pads(H, K, S)[0], layers.same_pads(W, K, S)[0]
  Ho, Wo = layers.same_out(H, S), layers.same_out(W, S)
  return dict(x=x, x64=x64, w=w, b=b, K=K, S=S, pt=pt, pl=pl, Ho=Ho, Wo=Wo,
              H=H, W=W, u8=u8, g=g, dev=cuda)


@pytest.mark.parametrize('name', sorted(SHAPES))
@pytest.mark.parametrize('relu_in,resid,relu_out', [
    (False, False, False), (True, False, True), (False, True, True)])
def test_conv_f32_forward(cuda, name, relu_in, resid, relu_out):
  d = _make(name, cuda)
  if d['u8'] and relu_in:
    pytest.skip('frames are never ReLU\'d')
  C = _C()
  N = d['x'].shape[0]
  Cout = d['w'].shape[3]
  add = torch.randn(N, d['Ho'], d['Wo'], Cout, generator=d['g']) if resid else None
  xin = d['x64'].clamp(min=0) if relu_in else d['x64']
  ref = layers.conv2d_same_nhwc(xin, d['w'].double(), d['b'].double(), d['S'])
  if resid:
    ref = ref + add.double()
  if relu_out:
    ref = ref.clamp(min=0)
  y = C.cf32_conv_fwd(d['x'].to(cuda), d['w'].to(cuda), d['b'].to(cuda), d['S'],
                      d['pt'], d['pl'], d['Ho'], d['Wo'], relu_in=relu_in,
                      add=None if add is None else add.to(cuda), relu_out=relu_out)
  assert y.dtype == torch.float32 and y.shape == ref.shape
  assert rel_err(y, ref) <= TOL


@pytest.mark.parametrize('name', sorted(k for k, v in SHAPES.items() if not v[7]))
@pytest.mark.parametrize('masked', [False, True])
def test_conv_f32_dgrad(cuda, name, masked):
  d = _make(name, cuda, seed=1)
  C = _C()
  N = d['x'].shape[0]
  Cout = d['w'].shape[3]
  dy = torch.randn(N, d['Ho'], d['Wo'], Cout, generator=d['g'])
  x64 = d['x64'].clone().requires_grad_(True)
  y = layers.conv2d_same_nhwc(x64, d['w'].double(), None, d['S'])
  (ref,) = torch.autograd.grad(y, x64, dy.double())
  mask = add = None
  if masked:
    mask = torch.randn(d['x'].shape, generator=d['g'])
    add = torch.randn(d['x'].shape, generator=d['g'])
    ref = torch.where(mask.double() > 0, ref, torch.zeros_like(ref)) + add.double()
  dx = C.cf32_conv_dgrad(dy.to(cuda), d['w'].to(cuda), d['S'], d['pt'], d['pl'],
                         d['H'], d['W'],
                         mask=None if mask is None else mask.to(cuda),
                         add=None if add is None else add.to(cuda))
  assert dx.shape == ref.shape
  assert rel_err(dx, ref) <= TOL


@pytest.mark.parametrize('name', sorted(SHAPES))
@pytest.mark.parametrize('relu_in', [False, True])
def test_conv_f32_wgrad(cuda, name, relu_in):
  d = _make(name, cuda, seed=2)
  if d['u8'] and relu_in:
    pytest.skip('frames are never ReLU\'d')
  C = _C()
  N = d['x'].shape[0]
  Cout = d['w'].shape[3]
  dy = torch.randn(N, d['Ho'], d['Wo'], Cout, generator=d['g'])
  w64 = d['w'].double().requires_grad_(True)
  b64 = d['b'].double().requires_grad_(True)
  xin = d['x64'].clamp(min=0) if relu_in else d['x64']
  y = layers.conv2d_same_nhwc(xin, w64, b64, d['S'])
  rw, rb = torch.autograd.grad(y, (w64, b64), dy.double())
  # the kernels ACCUMULATE: start from a known non-zero gradient
  dw0 = torch.randn(d['w'].shape, generator=d['g'])
  db0 = torch.randn(Cout, generator=d['g'])
  dw, db = dw0.to(cuda), db0.to(cuda)
  x, dyc = d['x'].to(cuda), dy.to(cuda)
  C.cf32_conv_wgrad(x, dyc, d['S'], d['pt'], d['pl'], relu_in, dw, db)
  assert rel_err(dw - dw0.to(cuda), rw) <= TOL
  assert rel_err(db - db0.to(cuda), rb) <= TOL
  # deterministic: a second accumulation adds bitwise the same amount
  dw2, db2 = torch.zeros_like(dw), torch.zeros_like(db)
  dw3, db3 = torch.zeros_like(dw), torch.zeros_like(db)
  C.cf32_conv_wgrad(x, dyc, d['S'], d['pt'], d['pl'], relu_in, dw2, db2)
  C.cf32_conv_wgrad(x, dyc, d['S'], d['pt'], d['pl'], relu_in, dw3, db3)
  assert torch.equal(dw2, dw3) and torch.equal(db2, db3)


@pytest.mark.parametrize('N,H,W,C', [(3, 72, 96, 16), (3, 36, 48, 32),
                                     (3, 18, 24, 32), (2, 84, 84, 16),
                                     (2, 21, 21, 32)])
def test_maxpool_f32(cuda, N, H, W, C):
  g = torch.Generator().manual_seed(3)
  x = torch.randn(N, H, W, C, generator=g)
  dy = torch.randn(N, (H + 1) // 2, (W + 1) // 2, C, generator=g)
  x64 = x.double().requires_grad_(True)
  ref = layers.maxpool_same_nhwc(x64, 3, 2)
  (rdx,) = torch.autograd.grad(ref, x64, dy.double())
  pbh, pbw = layers.same_pads(H, 3, 2)[0], layers.same_pads(W, 3, 2)[0]
  C_ = _C()
  y, arg = C_.cf32_maxpool_fwd(x.to(cuda), pbh, pbw)
  assert torch.equal(y.cpu().double(), ref.detach())  # max is exact
  dx = C_.cf32_maxpool_bwd(dy.to(cuda), arg, H, W, pbh, pbw)
  assert rel_err(dx, rdx) <= 1e-6


def _ref_features(agent, frames):
  """float64 replica of Agent.conv_features (the torch oracle)."""
  x = frames.double() / 255.0
  P = {k: v.detach().double().cpu().requires_grad_(True) for k, v in agent.convnet.items()}
  for sp in agent.specs:
    if sp['kind'] == 'conv':
      x = layers.conv2d_same_nhwc(x, P[sp['name'] + '__w'], P[sp['name'] + '__b'], sp['s'])
      if sp['relu_out']:
        x = x.clamp(min=0)
    elif sp['kind'] == 'pool':
      x = layers.maxpool_same_nhwc(x, 3, 2)
    else:
      block_in = x
      for sub in ('conv_2d', 'conv_2d_1'):
        x = x.clamp(min=0)
        x = layers.conv2d_same_nhwc(x, P[sp['name'] + '__' + sub + '__w'],
                                    P[sp['name'] + '__' + sub + '__b'], 1)
      x = x + block_in
  x = x.clamp(min=0)
  return x.reshape(x.shape[0], -1), P


# frame seeds whose float64 forward has no pool near-tie / ReLU near-zero
# (tests/_discontinuity.py): there fp32 and float64 may branch differently
# and a single flip moves a whole local gradient
@pytest.mark.parametrize('torso,shape,fseed', [('deep', (72, 96, 3), 2),
                                               ('shallow', (72, 96, 3), 0),
                                               ('deep', (84, 84, 4), 8),
                                               ('shallow', (84, 84, 4), 0),
                                               ('deep', (72, 128, 3), 3)])
def test_torso_f32_matches_float64(cuda, torso, shape, fseed):
  """Whole fp32 HIP torso (features and every conv weight/bias gradient)
  against the float64 oracle; the bf16 kernels are not involved."""
  from scalable_agent_amd.models import Agent
  from scalable_agent_amd.models.agent import torso_precision
  from tests import _discontinuity
  agent = Agent(9, torso=torso, frame_shape=shape, seed=5, backend='hip',
                compute_dtype=torch.float32)
  g = torch.Generator().manual_seed(fseed)
  frames = torch.randint(0, 256, (2,) + shape, generator=g, dtype=torch.uint8)
  assert _discontinuity.count(agent, frames) == 0
  agent = agent.to(cuda)
  assert torso_precision(agent) == 'fp32'
  feats = agent.conv_features(frames.to(cuda))
  assert feats.dtype == torch.float32
  ref, P = _ref_features(agent, frames)
  assert rel_err(feats, ref) <= TOL
  r = torch.randn(ref.shape, generator=g)
  (feats * r.to(cuda)).sum().backward()
  (ref * r.double()).sum().backward()
  for k, p in agent.convnet.items():
    assert rel_err(p.grad, P[k].grad) <= 5 * TOL, k


def test_bf16_agent_atari_stack_takes_bf16_kernels(cuda):
  """The Atari 4-channel stack (BASELINE config #2) runs the fused bf16
  torso at bf16 (conv1 takes C = 3 or 4 uint8 channels); other channel
  counts take the exact-fp32 kernels instead of failing."""
  from scalable_agent_amd.models import Agent
  from scalable_agent_amd.models.agent import torso_precision
  agent = Agent(6, torso='deep', frame_shape=(84, 84, 4), seed=1, backend='hip',
                compute_dtype=torch.bfloat16).to(cuda)
  assert torso_precision(agent) == 'bf16'
  frames = torch.randint(0, 256, (4, 84, 84, 4), dtype=torch.uint8, device=cuda)
  feats = agent.conv_features(frames)
  assert feats.shape == (4, 11 * 11 * 32) and torch.isfinite(feats).all()
  gray = Agent(6, torso='deep', frame_shape=(84, 84, 1), seed=1, backend='hip',
               compute_dtype=torch.bfloat16).to(cuda)
  assert torso_precision(gray) == 'fp32'


def _torso_run(agent, frames, r, max_frames):
  """Features and conv-parameter gradients of sum(features * r) with the
  torso chunked at max_frames frames per launch sequence."""
  from scalable_agent_amd.ops import conv_f32
  old = conv_f32.MAX_FRAMES
  conv_f32.MAX_FRAMES = max_frames
  try:
    for p in agent.parameters():
      p.grad = None
    f = agent.conv_features(frames)
    (f.float() * r).sum().backward()
    return f.detach(), {k: p.grad.clone() for k, p in agent.convnet.items()}
  finally:
    conv_f32.MAX_FRAMES = old


@pytest.mark.parametrize('torso,dtype', [('deep', torch.float32), ('shallow', torch.float32),
                                         ('deep', torch.bfloat16)])
def test_torso_chunking_matches_whole_batch(cuda, torso, dtype):
  """Large learner batches run the torso in frame chunks (ops/conv_f32.py
  MAX_FRAMES): per-frame features are bitwise those of one launch sequence,
  and the chunks' weight gradients add up to the whole batch's."""
  from scalable_agent_amd.models import Agent
  agent = Agent(9, torso=torso, frame_shape=(72, 96, 3), seed=3, backend='hip',
                compute_dtype=dtype).to(cuda)
  g = torch.Generator(device=cuda).manual_seed(4)
  frames = torch.randint(0, 256, (150, 72, 96, 3), generator=g, dtype=torch.uint8,
                         device=cuda)
  r = torch.randn(150, agent.flat_size, generator=g, device=cuda)
  f1, g1 = _torso_run(agent, frames, r, 1 << 20)
  f3, g3 = _torso_run(agent, frames, r, 64)  # 3 chunks of 50 frames
  assert torch.equal(f1, f3)
  tol = 1e-5 if dtype == torch.float32 else 2e-3
  for k in g1:
    assert rel_err(g3[k], g1[k]) <= tol, k


def test_torso_f32_learner_scale_batch(cuda):
  """The single-learner equivalent of 8 data-parallel ranks (B=256, T=100:
  25856 frames, past the Winograd launchers' 2^22-tile / 4 GB limits for one
  launch): 4 chunks of 6464 frames vs 8 chunks of 3232 (the headline batch)
  - bitwise features, gradients within fp32 summation order - and the first
  frames against the float64 oracle."""
  from scalable_agent_amd.models import Agent
  from scalable_agent_amd.ops import conv_f32
  agent = Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=5, backend='hip',
                compute_dtype=torch.float32).to(cuda)
  N = 256 * 101
  g = torch.Generator(device=cuda).manual_seed(2)
  frames = torch.randint(0, 256, (N, 72, 96, 3), generator=g, dtype=torch.uint8,
                         device=cuda)
  r = torch.randn(N, agent.flat_size, generator=g, device=cuda)
  assert -(-N // conv_f32.MAX_FRAMES) == 4
  fa, ga = _torso_run(agent, frames, r, conv_f32.MAX_FRAMES)
  fb, gb = _torso_run(agent, frames, r, 3232)
  assert torch.isfinite(fa).all()
  assert torch.equal(fa, fb)
  for k in ga:
    assert torch.isfinite(ga[k]).all(), k
    assert rel_err(ga[k], gb[k]) <= 1e-5, k
  cpu_agent = Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=5)
  ref, _ = _ref_features(cpu_agent, frames[-2:].cpu())
  assert rel_err(fa[-2:], ref) <= 1e-4


@pytest.mark.parametrize('N,H,W,zero_w,cin', [(256, 36, 48, False, 16), (5, 36, 48, False, 16),
                                               (3, 16, 32, False, 16), (2, 8, 64, False, 16),
                                               (7, 36, 48, True, 16), (300, 18, 24, False, 32),
                                               (3, 18, 24, True, 32),
                                               # odd tile-row counts (H % 4 == 2):
                                               # the Atari 42x42 head, and 10 rows at 48
                                               (64, 42, 42, False, 16), (5, 42, 42, False, 16),
                                               (3, 42, 42, True, 16), (4, 10, 48, False, 16)])
def test_wino_conv_pool_matches_conv_then_pool(cuda, N, H, W, zero_w, cin):
  """The 16 -> 32 stage head with the max-pool in the Winograd epilogue
  (wino_conv_pool_kernel): pooled values and argmax codes bitwise those of
  the Winograd conv followed by maxpool_fwd.  N = 256: long contiguous runs
  per workgroup (the register carry between tile-row pairs); N = 5: one
  range per workgroup, so every pooled odd row goes through the run-boundary
  merge; zero weights: every tap ties, the first one must win everywhere.
  cin 32: the stage-2 head (18x24, whole-image ranges, opt-in bit 2)."""
  C = _C()
  g = torch.Generator().manual_seed(11)
  x = torch.randn(N, H, W, cin, generator=g).to(cuda)
  w = (torch.zeros(3, 3, cin, 32) if zero_w else
       torch.randn(3, 3, cin, 32, generator=g) / 12.0).to(cuda)
  b = torch.randn(32, generator=g).to(cuda)
  out = C.cf32_wino_conv_pool_fwd(x, w, b, stages=15)  # 15: the 42-wide head too
  assert len(out) == 2
  y, arg = out
  conv = C.cf32_conv_fwd(x, w, b, 1, 1, 1, H, W)
  ry, rarg = C.cf32_maxpool_fwd(conv, 0, 0)
  assert y.shape == ry.shape == (N, H // 2, W // 2, 32)
  assert torch.equal(y, ry)
  assert torch.equal(arg, rarg)
  if zero_w:
    assert int(arg.max()) == 0


@pytest.mark.parametrize('N,H,W,zero_w', [(6, 72, 96, False), (120, 72, 96, False),
                                           (3, 8, 64, False), (5, 72, 96, True),
                                           (7, 84, 84, False), (3, 84, 84, True),
                                           (5, 72, 128, False), (3, 72, 128, True)])
def test_wino_conv_pool_stage0_matches_float64(cuda, N, H, W, zero_w):
  """Stage-0 head (4-channel image -> 16) with the pool in the Winograd
  epilogue against the float64 conv + 3x3/2 max-pool: values to fp32
  rounding, argmax codes wherever the float64 window has a clear maximum
  (gap > 1e-5: elsewhere fp32 and float64 may legitimately pick another
  tap); zero weights: every tap ties and the first must win."""
  C = _C()
  g = torch.Generator().manual_seed(13)
  x = torch.rand(N, H, W, 4, generator=g)
  w = (torch.zeros(3, 3, 4, 16) if zero_w else
       torch.randn(3, 3, 4, 16, generator=g) / 6.0)
  if W != 84:  # RGB: the image's pad channel; 84x84 Atari stacks: 4 frames
    x[..., 3] = 0
    w[:, :, 3] = 0
  b = torch.randn(16, generator=g) * 0.1
  # stage 0 is opt-in (SA_F32_WINO_POOL bit 1): enabled explicitly here
  out = C.cf32_wino_conv_pool_fwd(x.to(cuda), w.to(cuda), b.to(cuda), stages=3)
  assert len(out) == 2
  y, arg = out[0].cpu().double(), out[1].cpu().long()
  conv = layers.conv2d_same_nhwc(x.double(), w.double(), b.double(), 1)
  # windows (3x3, stride 2, pad-before 0, -inf beyond the bottom/right edge)
  cp = torch.nn.functional.pad(conv.permute(0, 3, 1, 2), (0, 1, 0, 1), value=float('-inf'))
  win = cp.unfold(2, 3, 2).unfold(3, 3, 2)            # [N, C, Hp, Wp, 3, 3]
  win = win.reshape(*win.shape[:4], 9).permute(0, 2, 3, 1, 4)  # [N, Hp, Wp, C, 9]
  ref = win.max(-1).values
  first = (win == ref.unsqueeze(-1)).double().argmax(-1)       # first maximal tap
  assert rel_err(y, ref) <= 1e-5
  top2 = win.topk(2, dim=-1).values
  clear = (top2[..., 0] - top2[..., 1]) > 1e-5 * ref.abs().max()
  assert torch.equal(arg[clear], first[clear])
  if zero_w:
    assert int(arg.max()) == 0
  else:
    assert clear.float().mean() > 0.99


def test_wino_conv_pool_declines_other_shapes(cuda):
  C = _C()
  x = torch.randn(2, 20, 24, 32, device=cuda)  # 32 -> 32 off the 18x24 instance
  assert C.cf32_wino_conv_pool_fwd(x, torch.zeros(3, 3, 32, 32, device=cuda),
                                   torch.zeros(32, device=cuda), stages=7) == []
  x = torch.randn(2, 42, 44, 16, device=cuda)  # a width with no instance
  assert C.cf32_wino_conv_pool_fwd(x, torch.zeros(3, 3, 16, 32, device=cuda),
                                   torch.zeros(32, device=cuda)) == []


@pytest.mark.parametrize('shape', [(3232 // 101, 72, 96, 3), (3, 5, 7, 3), (2, 84, 84, 4),
                                   (3, 5, 7, 1), (2, 6, 5, 2),
                                   (1300, 72, 96, 3)])  # > 8192 tiles: grid stride
@pytest.mark.parametrize('misaligned', [False, True])
def test_frames_f32_is_exact_division(cuda, shape, misaligned):
  """uint8 frames -> the 4-channel fp32 x / 255 image: bitwise torch's
  correctly rounded division, zero pad channels, any pixel count (tail) and
  a frame pointer that is not word aligned."""
  C = _C()
  g = torch.Generator().manual_seed(17)
  n = 1
  for d in shape:
    n *= d
  buf = torch.randint(0, 256, (n + 1,), generator=g, dtype=torch.uint8).to(cuda)
  fr = (buf[1:] if misaligned else buf[:n]).view(shape)
  y = C.cf32_frames_f32(fr).cpu()
  # correctly rounded fp32 quotients (the reference's IEEE division; the
  # GPU torch scalar division multiplies by a rounded reciprocal instead)
  table = (torch.arange(256, dtype=torch.float64) / 255.0).float()
  ref = torch.zeros(shape[:3] + (4,))
  ref[..., :shape[3]] = table[fr.cpu().long()]
  assert y.shape == ref.shape and torch.equal(y, ref)


def test_oversized_conv_call_fails_loudly(cuda):
  """A conv tensor of >= 4 GB (past the validated sizes) raises instead of
  running: the learner chunks such batches (ops/conv_f32.py MAX_FRAMES)."""
  C = _C()
  x = torch.empty(10000, 72, 96, 16, device=cuda)  # 4.4 GB, never written
  w = torch.zeros(3, 3, 16, 16, device=cuda)
  b = torch.zeros(16, device=cuda)
  with pytest.raises(RuntimeError, match='4 GB'):
    C.cf32_conv_fwd(x, w, b, 1, 1, 1, 72, 96)
  del x


@pytest.mark.parametrize('N,H,W,Cin,Cout,u8', [
    (3, 72, 96, 3, 16, True), (3, 36, 48, 16, 32, False), (3, 18, 24, 32, 32, False),
    (2, 84, 84, 4, 16, True), (2, 42, 42, 16, 32, False), (2, 21, 21, 32, 32, False)])
def test_fused_stage_head_matches_unfused(cuda, N, H, W, Cin, Cout, u8):
  """Fused conv+pool forward == conv then maxpool (bitwise: same MFMA order);
  the backward that gathers the pre-pool gradient from (dP, argmax) inside
  the conv kernels == maxpool_bwd then the plain conv kernels."""
  C = _C()
  g = torch.Generator().manual_seed(7)
  if u8:
    x = torch.randint(0, 256, (N, H, W, Cin), generator=g, dtype=torch.uint8).to(cuda)
  else:
    x = torch.randn(N, H, W, Cin, generator=g).to(cuda)
  w = (torch.randn(3, 3, Cin, Cout, generator=g) / (9 * Cin) ** 0.5).to(cuda)
  b = (torch.randn(Cout, generator=g) * 0.1).to(cuda)
  pbh, pbw = layers.same_pads(H, 3, 2)[0], layers.same_pads(W, 3, 2)[0]
  conv = C.cf32_conv_fwd(x, w, b, 1, 1, 1, H, W)
  ref_p, ref_a = C.cf32_maxpool_fwd(conv, pbh, pbw)
  p, a = C.cf32_conv_pool_fwd(x, w, b, pbh, pbw)
  # the stand-alone 3x3/1 conv of the 16/32-channel stages runs the Winograd
  # kernels (different rounding than the fused direct conv+pool): values to
  # fp32 accuracy, argmax codes equal except at fp32-level near-ties
  assert rel_err(p, ref_p) <= 1e-6
  assert (a != ref_a).float().mean().item() <= 1e-4
  ref_a = a
  dP = torch.randn(p.shape, generator=g).to(cuda)
  dconv = C.cf32_maxpool_bwd(dP, a, H, W, pbh, pbw)
  dw1, db1 = torch.zeros_like(w), torch.zeros_like(b)
  dw2, db2 = torch.zeros_like(w), torch.zeros_like(b)
  C.cf32_conv_wgrad(x, dconv, 1, 1, 1, False, dw1, db1)
  C.cf32_conv_wgrad(x, dP, 1, 1, 1, False, dw2, db2, pool_arg=a, pool_pbh=pbh, pool_pbw=pbw)
  assert rel_err(dw2, dw1) <= 1e-6 and rel_err(db2, db1) <= 1e-6
  if not u8:
    dx1 = C.cf32_conv_dgrad(dconv, w, 1, 1, 1, H, W)
    dx2 = C.cf32_conv_dgrad(dP, w, 1, 1, 1, H, W, pool_arg=a, pool_pbh=pbh, pool_pbw=pbw)
    assert rel_err(dx2, dx1) <= 1e-6


@pytest.mark.parametrize('N,H,W,Cs', [(5, 72, 96, 3), (3, 84, 84, 4), (4, 9, 13, 1),
                                      (2, 10, 136, 3)])
def test_stage0_scatter_wgrad(cuda, N, H, W, Cs):
  """Stage-0 weight gradient in scatter form straight from (dP, argmax)
  (pool_wgrad_kernel) == the float64 weight gradient of the dense pre-pool
  gradient; bitwise reproducible run to run (fixed-order partials).  W = 136
  (pooled width 68 > 64) takes the dense-gather MFMA fallback instead."""
  C = _C()
  g = torch.Generator().manual_seed(11)
  fr = torch.randint(0, 256, (N, H, W, Cs), generator=g, dtype=torch.uint8).to(cuda)
  x = C.cf32_frames_f32(fr)
  w = (torch.randn(3, 3, 4, 16, generator=g) / 6.0).to(cuda)
  b = (torch.randn(16, generator=g) * 0.1).to(cuda)
  pbh, pbw = layers.same_pads(H, 3, 2)[0], layers.same_pads(W, 3, 2)[0]
  p, a = C.cf32_conv_pool_fwd(x, w, b, pbh, pbw)
  dP = torch.randn(p.shape, generator=g).to(cuda)
  dconv = C.cf32_maxpool_bwd(dP, a, H, W, pbh, pbw)
  ref = torch.nn.grad.conv2d_weight(
      x.permute(0, 3, 1, 2).double(), (16, 4, 3, 3),
      dconv.permute(0, 3, 1, 2).double(), padding=1).permute(2, 3, 1, 0)
  outs = []
  for _ in range(2):
    dw, db = torch.zeros_like(w), torch.zeros_like(b)
    C.cf32_conv_wgrad(x, dP, 1, 1, 1, False, dw, db, pool_arg=a, pool_pbh=pbh,
                      pool_pbw=pbw)
    outs.append((dw, db))
  assert rel_err(outs[0][0].double(), ref) <= 1e-5
  assert rel_err(outs[0][1].double(), dconv.double().sum((0, 1, 2))) <= 1e-5
  assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize('env', [{'SA_F32_DGRAD_STACK': '1'},
                                 {'SA_F32_DGRAD_PHASE': '0'}])
def test_strided_dgrad_alternative_paths(cuda, env):
  """The opt-in strided-dgrad forms (phase-stacked single launch; the
  correlation over the stride-dilated dY) pass the same dgrad tests (the
  switches are read once per process, hence a subprocess)."""
  import os
  import subprocess
  import sys
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  r = subprocess.run(
      [sys.executable, '-m', 'pytest', '-q', '-p', 'no:cacheprovider',
       os.path.abspath(__file__), '-k', 'test_conv_f32_dgrad and shallow'],
      capture_output=True, text=True, timeout=240, cwd=root,
      env=dict(os.environ, PYTHONPATH=root, **env))
  assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
  assert ' passed' in r.stdout


@pytest.mark.parametrize('H,W,Cin,Cout', [(36, 48, 16, 16), (36, 48, 16, 32),
                                          (18, 24, 32, 32), (9, 12, 32, 32)])
def test_conv_f32_many_tiles(cuda, H, W, Cin, Cout):
  """The deep torso's 3x3/1 layers at N = 256 frames: every persistent
  workgroup walks several tiles/ranges (cross-tile register prefetch, LDS
  double use, range/image boundaries, slot-capped weight-gradient loops),
  which the N <= 3 shape tests above never reach.  Forward with ReLU-in +
  residual + ReLU-out, data gradient with mask + skip add, weight + bias
  gradient with ReLU-in, all against float64."""
  C = _C()
  N = 256
  g = torch.Generator().manual_seed(H * Cin + Cout)
  x = torch.randn(N, H, W, Cin, generator=g)
  w = torch.randn(3, 3, Cin, Cout, generator=g) / (9 * Cin) ** 0.5
  b = torch.randn(Cout, generator=g) * 0.1
  add = torch.randn(N, H, W, Cout, generator=g)
  xr = x.double().clamp(min=0)
  ref = (layers.conv2d_same_nhwc(xr, w.double(), b.double(), 1) +
         add.double()).clamp(min=0)
  y = C.cf32_conv_fwd(x.to(cuda), w.to(cuda), b.to(cuda), 1, 1, 1, H, W,
                      relu_in=True, add=add.to(cuda), relu_out=True)
  assert rel_err(y, ref) <= TOL
  dy = torch.randn(N, H, W, Cout, generator=g)
  mask = torch.randn(N, H, W, Cin, generator=g)
  sk = torch.randn(N, H, W, Cin, generator=g)
  x64 = x.double().requires_grad_(True)
  (dref,) = torch.autograd.grad(
      layers.conv2d_same_nhwc(x64, w.double(), None, 1), x64, dy.double())
  dref = torch.where(mask.double() > 0, dref, torch.zeros_like(dref)) + sk.double()
  dx = C.cf32_conv_dgrad(dy.to(cuda), w.to(cuda), 1, 1, 1, H, W,
                         mask=mask.to(cuda), add=sk.to(cuda))
  assert rel_err(dx, dref) <= TOL
  w64 = w.double().requires_grad_(True)
  b64 = b.double().requires_grad_(True)
  rw, rb = torch.autograd.grad(layers.conv2d_same_nhwc(xr, w64, b64, 1),
                               (w64, b64), dy.double())
  dw, db = torch.zeros(3, 3, Cin, Cout, device=cuda), torch.zeros(Cout, device=cuda)
  C.cf32_conv_wgrad(x.to(cuda), dy.to(cuda), 1, 1, 1, True, dw, db)
  assert rel_err(dw, rw) <= TOL
  assert rel_err(db, rb) <= TOL


@pytest.mark.parametrize('N,H,W,Cx,Cy,mask', [
    (256, 36, 48, 16, 16, True), (256, 18, 24, 32, 32, True), (256, 9, 12, 32, 32, True),
    (5, 11, 11, 16, 16, True), (5, 11, 11, 32, 32, True),
    (256, 36, 48, 16, 32, False), (256, 18, 24, 32, 32, False), (5, 11, 11, 16, 32, False),
    (256, 36, 48, 16, 16, False),
    (7, 42, 42, 16, 32, False), (3, 36, 64, 16, 32, False),
    # the 72x128 Doom ladder: ranges on tile-row boundaries (tight row bound)
    (40, 36, 64, 16, 16, True), (40, 36, 64, 16, 32, False),
    (40, 18, 32, 32, 32, True), (40, 18, 32, 32, 32, False), (40, 9, 16, 32, 32, True),
    # ranges that never straddle images but start mid-row (per_img % RT == 0)
    (40, 16, 48, 16, 16, True), (40, 16, 48, 32, 32, True)])
@pytest.mark.parametrize('relu_x,use_add', [(False, False), (True, True)])
def test_conv_bwd_fused(cuda, N, H, W, Cx, Cy, mask, relu_x, use_add):
  """A 3x3/1 conv's backward in one pass (conv_wino.hip
  wino_bwd_fused_kernel for the 16-channel residual convs,
  wino_bwd_fused32_kernel for 32 -> 32 and the 16 -> 32 stage head, whose
  data gradient splits each task over a wave pair and hands the partial
  output transform through LDS): dX = dgrad(dY, W) [* (x > 0)] [+ add],
  dW += relu?(x)^T dY, db += sum dY, against float64.  At N = 256 every
  persistent workgroup walks many ranges (contiguous range runs, cross-range
  prefetch, image boundaries inside a range); 11x11 / 42x42 exercise odd
  tile counts and partial 2x2 tiles; 36x64 / 18x32 / 9x16 are the 72x128
  Doom frame's maps, whose ranges start on tile-row boundaries."""
  C = _C()
  g = torch.Generator().manual_seed(N * H + Cx + Cy)
  x = torch.randn(N, H, W, Cx, generator=g)
  w = torch.randn(3, 3, Cx, Cy, generator=g) / (9 * Cx) ** 0.5
  dy = torch.randn(N, H, W, Cy, generator=g)
  add = torch.randn(N, H, W, Cx, generator=g)
  x64 = x.double().requires_grad_(True)
  xin = x64.clamp(min=0) if relu_x else x64
  w64 = w.double().requires_grad_(True)
  b64 = torch.zeros(Cy, dtype=torch.float64, requires_grad=True)
  _, gw, gb = torch.autograd.grad(layers.conv2d_same_nhwc(xin, w64, b64, 1),
                                  (x64, w64, b64), dy.double())
  x2 = x.double().requires_grad_(True)
  (gx,) = torch.autograd.grad(layers.conv2d_same_nhwc(x2, w.double(), None, 1), x2,
                              dy.double())
  ref = torch.where(x.double() > 0, gx, torch.zeros_like(gx)) if mask else gx
  if use_add:
    ref = ref + add.double()
  dw = torch.zeros(3, 3, Cx, Cy, device=cuda)
  db = torch.zeros(Cy, device=cuda)
  dx = C.cf32_conv_bwd_fused(dy.to(cuda), w.to(cuda), x.to(cuda), relu_x, dw, db,
                             add=add.to(cuda) if use_add else None, mask=mask)
  assert rel_err(dx, ref) <= TOL
  assert rel_err(dw, gw) <= TOL
  assert rel_err(db, gb) <= TOL


@pytest.mark.parametrize('H,W,C', [(36, 48, 16), (18, 24, 32), (11, 11, 16)])
@pytest.mark.parametrize('block_conv', [1, 2])
def test_residual_block_forward_flags(cuda, H, W, C, block_conv):
  """The two forward flag sets of a residual block at N = 160 frames: conv 1
  = ReLU on the input + ReLU on the output + bias, conv 2 = bias + skip add
  (the sets that have compile-time kernel instances, conv_wino.hip)."""
  Cmod = _C()
  N = 160
  g = torch.Generator().manual_seed(H * C + block_conv)
  x = torch.randn(N, H, W, C, generator=g)
  w = torch.randn(3, 3, C, C, generator=g) / (9 * C) ** 0.5
  b = torch.randn(C, generator=g) * 0.1
  if block_conv == 1:
    ref = layers.conv2d_same_nhwc(x.double().clamp(min=0), w.double(), b.double(), 1)
    ref = ref.clamp(min=0)
    y = Cmod.cf32_conv_fwd(x.to(cuda), w.to(cuda), b.to(cuda), 1, 1, 1, H, W,
                           relu_in=True, relu_out=True)
  else:
    add = torch.randn(N, H, W, C, generator=g)
    ref = layers.conv2d_same_nhwc(x.double(), w.double(), b.double(), 1) + add.double()
    y = Cmod.cf32_conv_fwd(x.to(cuda), w.to(cuda), b.to(cuda), 1, 1, 1, H, W,
                           add=add.to(cuda))
  assert rel_err(y, ref) <= TOL


GEO_FWD = [(36, 48, 16, 16), (42, 42, 16, 16), (36, 48, 16, 32), (42, 42, 16, 32),
           (18, 24, 32, 32), (9, 12, 32, 32), (21, 21, 32, 32), (11, 11, 32, 32),
           (36, 64, 16, 16), (36, 64, 16, 32), (18, 32, 32, 32), (9, 16, 32, 32)]


@pytest.mark.parametrize('H,W,Cin,Cout', GEO_FWD)
@pytest.mark.parametrize('flags', ['plain', 'resblock1', 'resblock2'])
def test_wino_geometry_instances_match_runtime_fwd(cuda, H, W, Cin, Cout, flags):
  """Compile-time-geometry Winograd forward instances (conv_wino.hip
  TileGeo, every map of the IMPALA and Atari ladders) are bitwise the
  runtime-geometry kernel: same ranges, same arithmetic.  N = 37 frames:
  ranges cross images, the batch's last range is partial."""
  C = _C()
  N = 37
  g = torch.Generator().manual_seed(H * W + Cin + Cout)
  x = torch.randn(N, H, W, Cin, generator=g).to(cuda)
  w = (torch.randn(3, 3, Cin, Cout, generator=g) / (9 * Cin) ** 0.5).to(cuda)
  b = (torch.randn(Cout, generator=g) * 0.1).to(cuda)
  add = torch.randn(N, H, W, Cout, generator=g).to(cuda)
  kw = {'plain': {}, 'resblock1': dict(relu_in=True, relu_out=True),
        'resblock2': dict(add=add)}[flags]
  if flags == 'resblock2' and Cin != Cout:
    pytest.skip('the skip add needs Cin == Cout')
  outs = []
  prev = C.cf32_wino_geo(1)
  try:
    for geo in (1, 0):
      C.cf32_wino_geo(geo)
      outs.append(C.cf32_conv_fwd(x, w, b, 1, 1, 1, H, W, **kw))
  finally:
    C.cf32_wino_geo(prev)
  assert torch.equal(outs[0], outs[1])


GEO_BWD = [(36, 48, 16, 16, True), (42, 42, 16, 16, True), (36, 48, 16, 32, False),
           (42, 42, 16, 32, False), (18, 24, 32, 32, True), (18, 24, 32, 32, False),
           (9, 12, 32, 32, True), (21, 21, 32, 32, True), (21, 21, 32, 32, False),
           (11, 11, 32, 32, True), (36, 64, 16, 16, True), (36, 64, 16, 32, False),
           (18, 32, 32, 32, True), (18, 32, 32, 32, False), (9, 16, 32, 32, True)]


@pytest.mark.parametrize('H,W,Cx,Cy,mask', GEO_BWD)
@pytest.mark.parametrize('relu_x', [False, True])
def test_wino_geometry_instances_match_runtime_bwd(cuda, H, W, Cx, Cy, mask, relu_x):
  """Compile-time-geometry fused backward instances (wino_bwd_fused_kernel,
  wino_bwd_fused32_kernel) are bitwise the runtime-geometry kernels: dX, dW
  and db, N = 37 frames."""
  if relu_x and not mask:
    pytest.skip('stage heads: no ReLU on the operand')
  C = _C()
  N = 37
  g = torch.Generator().manual_seed(H * W + Cx + 3 * Cy)
  x = torch.randn(N, H, W, Cx, generator=g).to(cuda)
  w = (torch.randn(3, 3, Cx, Cy, generator=g) / (9 * Cx) ** 0.5).to(cuda)
  dy = torch.randn(N, H, W, Cy, generator=g).to(cuda)
  add = torch.randn(N, H, W, Cx, generator=g).to(cuda) if mask else None
  res = []
  prev = C.cf32_wino_geo(1)
  try:
    for geo in (1, 0):
      C.cf32_wino_geo(geo)
      dw = torch.zeros(3, 3, Cx, Cy, device=cuda)
      db = torch.zeros(Cy, device=cuda)
      dx = C.cf32_conv_bwd_fused(dy, w, x, relu_x, dw, db, add=add, mask=mask)
      res.append((dx, dw, db))
  finally:
    C.cf32_wino_geo(prev)
  for a, b_ in zip(*res):
    assert torch.equal(a, b_)
