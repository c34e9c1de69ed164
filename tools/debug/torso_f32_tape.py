"""Compares the deep fp32 torso's backward intermediates with float64 (debug)."""
import sys
import torch
sys.path.insert(0, '.')
from tests.test_conv_f32_gpu import rel_err
from scalable_agent_amd.models import Agent, layers
from scalable_agent_amd.ops import conv_f32

cuda = torch.device('cuda')
shape = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]))
n = int(sys.argv[4])
agent = Agent(9, torso='deep', frame_shape=shape, seed=5, backend='hip',
              compute_dtype=torch.float32).to(cuda)
g = torch.Generator().manual_seed(6)
frames = torch.randint(0, 256, (n,) + shape, generator=g, dtype=torch.uint8)
conv_f32.DEBUG_TAPE = {}
feats = agent.conv_features(frames.to(cuda))
P = {k: v.detach().double().cpu().requires_grad_(True) for k, v in agent.convnet.items()}
x = frames.double() / 255
ref = {}
def keep(key, t):
  t.retain_grad(); ref[key] = t; return t
for s in range(3):
  name = 'conv_2d' if s == 0 else 'conv_2d_%d' % s
  c = keep(('dconv', s), layers.conv2d_same_nhwc(x, P[name + '__w'], P[name + '__b'], 1))
  x = keep(('dpool', s), layers.maxpool_same_nhwc(c, 3, 2))
  for b in range(2):
    rn = 'residual_%d_%d' % (s, b)
    xa = x
    t = keep(('dt', s, b), layers.conv2d_same_nhwc(xa.clamp(min=0), P[rn + '__conv_2d__w'], P[rn + '__conv_2d__b'], 1).clamp(min=0))
    y = layers.conv2d_same_nhwc(t, P[rn + '__conv_2d_1__w'], P[rn + '__conv_2d_1__b'], 1) + xa
    x = keep(('dy', s, b), y)
out = x.clamp(min=0).reshape(n, -1)
r = torch.randn(out.shape, generator=g)
(feats * r.to(cuda)).sum().backward()
(out * r.double()).sum().backward()
print('feats %.2e' % rel_err(feats, out))
for s in reversed(range(3)):
  for b in reversed(range(2)):
    for k in (('dy', s, b), ('dt', s, b)):
      print(k, '%.2e' % rel_err(conv_f32.DEBUG_TAPE[k], ref[k].grad))
  for k in (('dpool', s), ('dconv', s)):
    print(k, '%.2e' % rel_err(conv_f32.DEBUG_TAPE[k], ref[k].grad))
for s in reversed(range(3)):
  print('saved intact before stage', s, conv_f32.DEBUG_TAPE[('intact', s)])
