#!/usr/bin/env python3
"""Tile-height sweep of the bf16 torso kernels (conv_torso.hip) per map:
res_conv_fwd / res_conv_bwd / conv_pool_fwd / pool_conv_bwd at the learner
batch, every tile height R the staging allows, on the runtime-geometry
kernels (conv_tune specialize=0), next to the default R.
usage: python tools/micro/torso_rows_sweep.py [N] [iters] [maps: impala,atari]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
from scalable_agent_amd import ops  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 3232
IT = int(sys.argv[2]) if len(sys.argv) > 2 else 5
WHICH = sys.argv[3] if len(sys.argv) > 3 else 'impala,atari'
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


def bf(*shape):
  return (torch.randn(*shape, device='cuda') * 0.5).to(torch.bfloat16)


def w32(cin, cout):
  return torch.randn(3, 3, cin, cout, device='cuda') * (2.0 / (9 * cin)) ** .5


def sweep(name, knob, W, rows, fn, rows_of_px):
  default = C.conv_tune(knob, -1)
  out = []
  for r in rows:
    px = rows_of_px(r)
    C.conv_tune(knob, px)
    try:
      out.append('%d:%.1f' % (r, timeit(fn)))
    except Exception as e:  # a height the launcher rejects
      out.append('%d:--' % r)
    C.conv_tune(knob, default)
  print('%-28s %s' % (name, '  '.join(out)), flush=True)


MAPS = {'impala': [(36, 48), (18, 24), (9, 12)], 'atari': [(42, 42), (21, 21), (11, 11)]}
C.conv_tune('specialize', 0)
for which in WHICH.split(','):
  (h1, w1), (h2, w2), (h3, w3) = MAPS[which]
  x16, d16 = bf(N, h1, w1, 16), bf(N, h1, w1, 16)
  w16, b16 = w32(16, 16), torch.zeros(16, device='cuda')
  dw16, db16 = torch.zeros_like(w16), torch.zeros_like(b16)
  rows1 = range(2, 17)
  pxr = lambda W: (lambda r: r * W + W // 2)
  sweep('%s res_fwd16 %dx%d' % (which, h1, w1), 'px_res_fwd', w1, rows1,
        lambda: C.res_conv_fwd(x16, w16, b16, None, True, True), pxr(w1))
  sweep('%s res_bwd16 %dx%d' % (which, h1, w1), 'px_res_bwd', w1, rows1,
        lambda: C.res_conv_bwd(d16, x16, d16, w16, dw16, db16), pxr(w1))
  w1632, b32 = w32(16, 32), torch.zeros(32, device='cuda')
  p2, a2 = C.conv_pool_fwd(x16, w1632, b32, 0, 0)
  dp2 = bf(*p2.shape)
  dw1632 = torch.zeros_like(w1632)
  pxp = lambda W: (lambda rp: (2 * rp + 1) * W + W // 2)
  sweep('%s pool_fwd16_32 %dx%d' % (which, h1, w1), 'px_pool_fwd', w1, range(1, 9),
        lambda: C.conv_pool_fwd(x16, w1632, b32, 0, 0), pxp(w1))
  sweep('%s pool_bwd16_32 %dx%d' % (which, h1, w1), 'px_pool_bwd', w1, rows1,
        lambda: C.pool_conv_bwd(dp2, a2, x16, w1632, dw1632, b32, True, 0, 0), pxr(w1))
  for (h, w) in ((h2, w2), (h3, w3)):
    x32, d32 = bf(N, h, w, 32), bf(N, h, w, 32)
    w32_ = w32(32, 32)
    dw32, db32 = torch.zeros_like(w32_), torch.zeros(32, device='cuda')
    rr = range(2, h + 1)
    sweep('%s res_fwd32 %dx%d' % (which, h, w), 'px_res_fwd', w, rr,
          lambda: C.res_conv_fwd(x32, w32_, b32, None, True, True), pxr(w))
    sweep('%s res_bwd32 %dx%d' % (which, h, w), 'px_res_bwd', w, rr,
          lambda: C.res_conv_bwd(d32, x32, d32, w32_, dw32, db32), pxr(w))
    if h in (h2,):
      p3, a3 = C.conv_pool_fwd(x32, w32_, b32, 0, 0)
      dp3 = bf(*p3.shape)
      sweep('%s pool_fwd32 %dx%d' % (which, h, w), 'px_pool_fwd', w, range(1, 7),
            lambda: C.conv_pool_fwd(x32, w32_, b32, 0, 0), pxp(w))
      sweep('%s pool_bwd32 %dx%d' % (which, h, w), 'px_pool_bwd', w, rr,
            lambda: C.pool_conv_bwd(dp3, a3, x32, w32_, dw32, db32, True, 0, 0), pxr(w))
C.conv_tune('specialize', 1)
