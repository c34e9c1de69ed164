#!/usr/bin/env python3
"""One large-N torso launch sequence vs the same frames in headline-sized
chunks (ops/conv_f32.py MAX_FRAMES): features and conv-weight gradients.
usage: torso_size_check.py N [dtype fp32|bf16]"""
import sys

import torch

sys.path.insert(0, '.')
from scalable_agent_amd.models import Agent  # noqa: E402
from scalable_agent_amd.ops import conv_f32  # noqa: E402

N = int(sys.argv[1])
dt = torch.bfloat16 if len(sys.argv) > 2 and sys.argv[2] == 'bf16' else torch.float32
cuda = torch.device('cuda')
agent = Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=5, backend='hip',
              compute_dtype=dt).to(cuda)
g = torch.Generator(device=cuda).manual_seed(2)
frames = torch.randint(0, 256, (N, 72, 96, 3), generator=g, dtype=torch.uint8, device=cuda)
r = torch.randn(N, agent.flat_size, generator=g, device=cuda)


def run(mf):
  conv_f32.MAX_FRAMES = mf
  for p in agent.parameters():
    p.grad = None
  f = agent.conv_features(frames)
  (f.float() * r).sum().backward()
  torch.cuda.synchronize()
  return f.detach().float(), {k: p.grad.clone() for k, p in agent.convnet.items()}


fa, ga = run(1 << 30)
fb, gb = run(3232)
fd = (fa - fb).abs().max().item()
worst = max(((ga[k] - gb[k]).abs().max() / gb[k].abs().max().clamp(min=1e-30)).item()
            for k in ga)
bad = [i for i in range(0, N, max(1, N // 64)) if not torch.equal(fa[i], fb[i])]
print('N=%d %s: feature max|diff| %.3g, worst grad rel diff %.3g, first mismatching '
      'sampled frames %s' % (N, dt, fd, worst, bad[:8]), flush=True)
