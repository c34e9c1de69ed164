"""Isolates which fp32 op breaks inside the deep torso backward (debug)."""
import sys
import torch
sys.path.insert(0, '.')
from tests.test_conv_f32_gpu import rel_err
from scalable_agent_amd.models import Agent, layers
from scalable_agent_amd import ops

C = ops.ext()
cuda = torch.device('cuda')
shape, n = (72, 96, 3), int(sys.argv[1]) if len(sys.argv) > 1 else 6
agent = Agent(9, torso='deep', frame_shape=shape, seed=5)
g = torch.Generator().manual_seed(6)
frames = torch.randint(0, 256, (n,) + shape, generator=g, dtype=torch.uint8)
P = {k: v.detach().double() for k, v in agent.convnet.items()}
# fp64 forward of stage 0/1 up to block (1,1)
x = frames.double() / 255
acts = {}
for s in range(2):
  name = 'conv_2d' if s == 0 else 'conv_2d_%d' % s
  x = layers.conv2d_same_nhwc(x, P[name + '__w'], P[name + '__b'], 1)
  x = layers.maxpool_same_nhwc(x, 3, 2)
  for b in range(2):
    rn = 'residual_%d_%d' % (s, b)
    xa = x
    t = layers.conv2d_same_nhwc(xa.clamp(min=0), P[rn + '__conv_2d__w'], P[rn + '__conv_2d__b'], 1).clamp(min=0)
    y = layers.conv2d_same_nhwc(t, P[rn + '__conv_2d_1__w'], P[rn + '__conv_2d_1__b'], 1) + xa
    acts[(s, b)] = (xa, t, y)
    x = y
for (s, b), (xa, t, y) in acts.items():
  rn = 'residual_%d_%d' % (s, b)
  h, w = xa.shape[1], xa.shape[2]
  dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
  w2 = P[rn + '__conv_2d_1__w']
  w1 = P[rn + '__conv_2d__w']
  # fp64 refs
  tt = t.clone().requires_grad_(True)
  yy = layers.conv2d_same_nhwc(tt, w2, None, 1)
  (dt_ref,) = torch.autograd.grad(yy, tt, dy)
  dt_ref = dt_ref * (t > 0)
  w1v = w1.clone().requires_grad_(True)
  yy = layers.conv2d_same_nhwc(xa.clamp(min=0), w1v, None, 1)
  (dw1_ref,) = torch.autograd.grad(yy, w1v, dt_ref)
  # fp32 kernels on the same (rounded) inputs
  f = lambda a: a.float().contiguous().to(cuda)
  dt = C.cf32_conv_dgrad(f(dy), f(w2), 1, 1, 1, h, w, mask=f(t))
  dw1 = torch.zeros(w1.shape, device=cuda)
  db1 = torch.zeros(w1.shape[3], device=cuda)
  C.cf32_conv_wgrad(f(xa), f(dt_ref), 1, 1, 1, True, dw1, db1)
  y2 = C.cf32_conv_fwd(f(t), f(w2), f(P[rn + '__conv_2d_1__b']), 1, 1, 1, h, w, add=f(xa))
  print(s, b, 'fwd %.2e dgrad %.2e wgrad %.2e' % (rel_err(y2, y), rel_err(dt, dt_ref), rel_err(dw1, dw1_ref)))
