"""Per-parameter gradient error of the fp32 HIP torso vs float64 (debug)."""
import sys
import torch
sys.path.insert(0, '.')
from tests.test_conv_f32_gpu import _ref_features, rel_err
from scalable_agent_amd.models import Agent

cuda = torch.device('cuda')
for shape in [(72, 96, 3), (84, 84, 4), (72, 128, 3)]:
  for n in (3, 6):
    agent = Agent(9, torso='deep', frame_shape=shape, seed=5, backend='hip',
                  compute_dtype=torch.float32).to(cuda)
    g = torch.Generator().manual_seed(6)
    frames = torch.randint(0, 256, (n,) + shape, generator=g, dtype=torch.uint8)
    feats = agent.conv_features(frames.to(cuda))
    ref, P = _ref_features(agent, frames)
    r = torch.randn(ref.shape, generator=g)
    (feats * r.to(cuda)).sum().backward()
    (ref * r.double()).sum().backward()
    print(shape, n, 'feats %.2e' % rel_err(feats, ref))
    for k, p in agent.convnet.items():
      e = rel_err(p.grad, P[k].grad)
      print('   %-36s %.2e %s' % (k, e, '<<<' if e > 5e-5 else ''))
