#!/usr/bin/env python3
"""Times every fused conv-torso kernel on the benchmark shapes (N = B*(T+1)
= 3232 frames of 72x96x3) and reports per-call time, per-step time (calls per
learner step x time) and effective HBM bandwidth; sweeps launch knobs
(`_C.conv_tune`).

usage: python tools/conv_bench.py [--n 3232] [--iters 10]
           [--sweep '[{"xcd":0}, {"xcd":1, "cap_bwd":4}]' | --sweep @file.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scalable_agent_amd import ops  # noqa: E402


def bf(*shape):
  return (torch.randn(*shape, device='cuda') * 0.5).to(torch.bfloat16)


def w32(cin, cout):
  return torch.randn(3, 3, cin, cout, device='cuda') * (2.0 / (9 * cin)) ** .5


def cases(n):
  C = ops.ext()
  dev = 'cuda'
  frames = torch.randint(0, 256, (n, 72, 96, 3), dtype=torch.uint8, device=dev)
  w1, b1 = w32(3, 16), torch.zeros(16, device=dev)
  p1, a1 = C.conv1_pool_fwd(frames, w1, b1, 0, 0)
  x16 = bf(n, 36, 48, 16)
  w16, b16 = w32(16, 16), torch.zeros(16, device=dev)
  w1632, b32 = w32(16, 32), torch.zeros(32, device=dev)
  p2, a2 = C.conv_pool_fwd(x16, w1632, b32, 0, 0)
  x32 = bf(n, 18, 24, 32)
  w32_ = w32(32, 32)
  p3, a3 = C.conv_pool_fwd(x32, w32_, b32, 0, 0)
  x9 = bf(n, 9, 12, 32)
  dw16, db16 = torch.zeros_like(w16), torch.zeros(16, device=dev)
  dw1632 = torch.zeros_like(w1632)
  dw32, db32 = torch.zeros_like(w32_), torch.zeros(32, device=dev)
  dw1, db1 = torch.zeros_like(w1), torch.zeros(16, device=dev)
  d16, d32, d9 = bf(n, 36, 48, 16), bf(n, 18, 24, 32), bf(n, 9, 12, 32)
  dp1, dp2, dp3 = bf(*p1.shape), bf(*p2.shape), bf(*p3.shape)
  B16 = n * 36 * 48 * 16 * 2
  B32 = n * 18 * 24 * 32 * 2
  B9 = n * 9 * 12 * 32 * 2
  F = n * 72 * 96 * 3
  # (name, calls per step, bytes moved (ideal), fn)
  return [
      ('conv1_pool_fwd', 1, F + B16 + B16 // 2,
       lambda: C.conv1_pool_fwd(frames, w1, b1, 0, 0)),
      ('res_fwd16', 2, 2 * B16, lambda: C.res_conv_fwd(x16, w16, b16, None, True, True)),
      ('res_fwd16_resid', 2, 3 * B16,
       lambda: C.res_conv_fwd(x16, w16, b16, x16, False, False)),
      ('block_fwd16 (fused)', 0, 3 * B16,
       lambda: C.res_block_fwd(x16, w16, b16, w16, b16, False)),
      ('conv_pool_fwd16_32', 1, B16 + B32 * 3 // 2,
       lambda: C.conv_pool_fwd(x16, w1632, b32, 0, 0)),
      ('res_fwd32', 2, 2 * B32, lambda: C.res_conv_fwd(x32, w32_, b32, None, True, True)),
      ('res_fwd32_resid', 2, 3 * B32,
       lambda: C.res_conv_fwd(x32, w32_, b32, x32, False, False)),
      ('block_fwd32 (fused)', 0, 3 * B32,
       lambda: C.res_block_fwd(x32, w32_, b32, w32_, b32, False)),
      ('conv_pool_fwd32_32', 1, B32 + B9 * 3 // 2,
       lambda: C.conv_pool_fwd(x32, w32_, b32, 0, 0)),
      ('res_fwd9', 2, 2 * B9, lambda: C.res_conv_fwd(x9, w32_, b32, None, True, True)),
      ('res_fwd9_resid', 2, 3 * B9,
       lambda: C.res_conv_fwd(x9, w32_, b32, x9, True, False)),
      ('block_fwd9 (fused)', 0, 3 * B9,
       lambda: C.res_block_fwd(x9, w32_, b32, w32_, b32, True)),
      ('res_bwd9', 2, 3 * B9,
       lambda: C.res_conv_bwd(d9, x9, None, w32_, dw32, db32, False)),
      ('res_bwd9_skip', 2, 4 * B9,
       lambda: C.res_conv_bwd(d9, x9, d9, w32_, dw32, db32)),
      ('pool_bwd32_32', 1, B9 * 3 // 2 + 2 * B32,
       lambda: C.pool_conv_bwd(dp3, a3, x32, w32_, dw32, db32, True, 0, 0)),
      ('res_bwd32', 2, 3 * B32,
       lambda: C.res_conv_bwd(d32, x32, None, w32_, dw32, db32, False)),
      ('res_bwd32_skip', 2, 4 * B32,
       lambda: C.res_conv_bwd(d32, x32, d32, w32_, dw32, db32)),
      ('pool_bwd16_32', 1, B32 * 3 // 2 + 2 * B16,
       lambda: C.pool_conv_bwd(dp2, a2, x16, w1632, dw1632, db32, True, 0, 0)),
      ('res_bwd16', 2, 3 * B16,
       lambda: C.res_conv_bwd(d16, x16, None, w16, dw16, db16, False)),
      ('res_bwd16_skip', 2, 4 * B16,
       lambda: C.res_conv_bwd(d16, x16, d16, w16, dw16, db16)),
      ('conv1_pool_bwd', 1, B16 * 3 // 4 + F,
       lambda: C.conv1_pool_bwd(dp1, a1, frames, dw1, db1, 0, 0)),
  ]


def time_fn(fn, iters):
  fn()
  torch.cuda.synchronize()
  ts = []
  for _ in range(iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(
        enable_timing=True)
    s.record()
    fn()
    e.record()
    e.synchronize()
    ts.append(s.elapsed_time(e) * 1e3)
  ts.sort()
  return ts[len(ts) // 2]


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--n', type=int, default=3232)
  ap.add_argument('--iters', type=int, default=10)
  ap.add_argument('--sweep', type=str, default='[{}]')
  ap.add_argument('--only', type=str, default='')
  args = ap.parse_args()
  C = ops.ext()
  cs = cases(args.n)
  if args.only:
    cs = [c for c in cs if args.only in c[0]]
  results = {}
  sweep = args.sweep
  if sweep.startswith('@'):
    sweep = open(sweep[1:]).read()
  for cfg in json.loads(sweep):
    old = {k: C.conv_tune(k, v) for k, v in cfg.items()}
    tot = 0.0
    rows = []
    for name, calls, nbytes, fn in cs:
      us = time_fn(fn, args.iters)
      tot += calls * us
      rows.append((name, calls, us, nbytes / us / 1e3))
    print('config %s: torso kernels %.1f us/step' % (json.dumps(cfg), tot),
          flush=True)
    for name, calls, us, gbs in rows:
      print('  %-20s x%d %8.1f us  %6.0f GB/s' % (name[:20], calls, us, gbs))
    results[json.dumps(cfg)] = tot
    for k, v in old.items():
      C.conv_tune(k, v)
  best = min(results, key=results.get)
  print('best: %s %.1f us/step' % (best, results[best]))


if __name__ == '__main__':
  main()
