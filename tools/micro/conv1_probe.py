#!/usr/bin/env python3
"""bf16 stage-0 kernels (conv1_pool_fwd / conv1_pool_bwd, conv_torso.hip) at
the learner batch for several frame shapes: us per call and per-pixel cost,
to separate frame size, channel count and tile geometry.
usage: python tools/micro/conv1_probe.py [N] [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
from scalable_agent_amd import ops  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 3232
IT = int(sys.argv[2]) if len(sys.argv) > 2 else 10
C = ops.ext()


def timeit(fn):
  fn()
  torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record()
  for _ in range(IT):
    fn()
  e.record()
  torch.cuda.synchronize()
  return s.elapsed_time(e) * 1e3 / IT


for H, W, Ch in [(72, 96, 3), (72, 96, 4), (84, 84, 3), (84, 84, 4)]:
  fr = torch.randint(0, 256, (N, H, W, Ch), dtype=torch.uint8, device='cuda')
  w = torch.randn(3, 3, Ch, 16, device='cuda') * 0.2
  b = torch.zeros(16, device='cuda')
  p, a = C.conv1_pool_fwd(fr, w, b, 0, 0)
  dp = (torch.randn(p.shape, device='cuda') * 0.5).to(torch.bfloat16)
  dw, db = torch.zeros_like(w), torch.zeros_like(b)
  tf = timeit(lambda: C.conv1_pool_fwd(fr, w, b, 0, 0))
  tb = timeit(lambda: C.conv1_pool_bwd(dp, a, fr, dw, db, 0, 0))
  px = N * H * W
  print('%dx%dx%d  fwd %7.1f us (%.2f ps/px)  bwd %7.1f us (%.2f ps/px)' % (
      H, W, Ch, tf, tf * 1e6 / px, tb, tb * 1e6 / px), flush=True)

if os.environ.get('SWEEP'):
  # tile-height sweep at 84x84x4 (non-default knobs run the runtime-geometry
  # kernels, so compare the rows with each other, not with the lines above)
  H, W, Ch = 84, 84, 4
  fr = torch.randint(0, 256, (N, H, W, Ch), dtype=torch.uint8, device='cuda')
  w = torch.randn(3, 3, Ch, 16, device='cuda') * 0.2
  b = torch.zeros(16, device='cuda')
  p, a = C.conv1_pool_fwd(fr, w, b, 0, 0)
  dp = (torch.randn(p.shape, device='cuda') * 0.5).to(torch.bfloat16)
  dw, db = torch.zeros_like(w), torch.zeros_like(b)
  C.conv_tune('specialize', 0)
  for rp in (3, 4, 5, 6, 7):
    old = C.conv_tune('px_conv1_fwd', (2 * rp + 1) * W + W // 2)
    t = timeit(lambda: C.conv1_pool_fwd(fr, w, b, 0, 0))
    C.conv_tune('px_conv1_fwd', old)
    print('fwd Rp=%d (runtime geometry) %7.1f us' % (rp, t), flush=True)
  for r in (8, 10, 11, 12, 13, 14):
    old = C.conv_tune('px_conv1_bwd', r * W + W // 2)
    t = timeit(lambda: C.conv1_pool_bwd(dp, a, fr, dw, db, 0, 0))
    C.conv_tune('px_conv1_bwd', old)
    print('bwd R=%d (runtime geometry) %7.1f us' % (r, t), flush=True)
  C.conv_tune('specialize', 1)
