#!/usr/bin/env python3
"""Per-layer timing of the exact-fp32 conv kernels at learner-batch size.

Deep-ResNet layers at N = (T+1) * B = 3232 frames (72x96x3 input): forward,
data gradient and weight gradient of every distinct layer shape, with the
achieved TFLOP/s against the 157 TF fp32 MFMA peak.  Usage:
  python tools/conv_f32_bench.py [N] [reps]
"""
import sys
import torch

sys.path.insert(0, '.')
from scalable_agent_amd import ops  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 3232
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ONLY = sys.argv[3] if len(sys.argv) > 3 else ''  # substring filter on layer names
C = ops.ext()
dev = torch.device('cuda')
# name, H, W, Cin, Cout, K, S, pt, pl, uint8 source, relu_in, resid
LAYERS = [
    ('deep conv1 3->16 72x96', 72, 96, 3, 16, 3, 1, 1, 1, True),
    ('deep res16 36x48', 36, 48, 16, 16, 3, 1, 1, 1, False),
    ('deep conv2 16->32 36x48', 36, 48, 16, 32, 3, 1, 1, 1, False),
    ('deep res32 18x24', 18, 24, 32, 32, 3, 1, 1, 1, False),
    ('deep res32 9x12', 9, 12, 32, 32, 3, 1, 1, 1, False),
    ('shallow1 8x8/4', 72, 96, 3, 32, 8, 4, 2, 2, True),
    ('shallow2 4x4/2', 18, 24, 32, 64, 4, 2, 1, 1, False),
    ('shallow3 3x3/2', 9, 12, 64, 128, 3, 2, 1, 0, False),
]


def timeit(fn):
  fn()
  torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record()
  for _ in range(REPS):
    fn()
  e.record()
  torch.cuda.synchronize()
  return s.elapsed_time(e) / REPS * 1e3


for name, H, W, Ci, Co, K, S, pt, pl, u8 in LAYERS:
  if ONLY and ONLY not in name:
    continue
  Ho, Wo = -(-H // S), -(-W // S)
  x = (torch.randint(0, 256, (N, H, W, Ci), dtype=torch.uint8, device=dev) if u8
       else torch.randn(N, H, W, Ci, device=dev))
  w = torch.randn(K, K, Ci, Co, device=dev) * 0.1
  b = torch.randn(Co, device=dev)
  dy = torch.randn(N, Ho, Wo, Co, device=dev)
  dw = torch.zeros_like(w)
  db = torch.zeros_like(b)
  flop = 2.0 * N * Ho * Wo * K * K * Ci * Co
  tf = timeit(lambda: C.cf32_conv_fwd(x, w, b, S, pt, pl, Ho, Wo))
  tw = timeit(lambda: C.cf32_conv_wgrad(x, dy, S, pt, pl, False, dw, db))
  line = '%-26s fwd %8.1f us %6.1f TF | wgrad %8.1f us %6.1f TF' % (
      name, tf, flop / tf / 1e6, tw, flop / tw / 1e6)
  if not u8:
    td = timeit(lambda: C.cf32_conv_dgrad(dy, w, S, pt, pl, H, W))
    line += ' | dgrad %8.1f us %6.1f TF' % (td, flop / td / 1e6)
  print(line, flush=True)
# residual-conv backward: fused (one pass) vs separate wgrad + masked dgrad
# (stage heads: 16 -> 32 and 32 -> 32 without mask / skip, relu_x off)
for name, H, W, Cc, Cy, res in [('res16 36x48', 36, 48, 16, 16, True),
                                ('res32 18x24', 18, 24, 32, 32, True),
                                ('res32 9x12', 9, 12, 32, 32, True),
                                ('head conv2 16->32 36x48', 36, 48, 16, 32, False),
                                ('head conv3 32->32 18x24', 18, 24, 32, 32, False)]:
  if ONLY and ONLY not in name and ONLY not in ('bwd', 'deep'):
    continue
  x = torch.randn(N, H, W, Cc, device=dev)
  w = torch.randn(3, 3, Cc, Cy, device=dev) * 0.1
  dy = torch.randn(N, H, W, Cy, device=dev)
  add = torch.randn(N, H, W, Cc, device=dev) if res else None
  dw = torch.zeros_like(w)
  db = torch.zeros(Cy, device=dev)
  tf = timeit(lambda: C.cf32_conv_bwd_fused(dy, w, x, res, dw, db, add=add, mask=res))

  def sep():
    C.cf32_conv_wgrad(x, dy, 1, 1, 1, res, dw, db)
    C.cf32_conv_dgrad(dy, w, 1, 1, 1, H, W, mask=x if res else None, add=add)
  ts = timeit(sep)
  bflop = 2 * 2.0 * N * H * W * 9 * Cc * Cy  # dgrad + wgrad, direct-conv FLOPs
  print('%-26s bwd fused %8.1f us %6.1f TF | separate wgrad+dgrad %8.1f us %6.1f TF' % (
      name, tf, bflop / tf / 1e6, ts, bflop / ts / 1e6), flush=True)
# stage-1 head forward: conv + maxpool_fwd vs the pool fused into the
# Winograd epilogue (wino_conv_pool_kernel)
if not ONLY or ONLY in 'head conv2 pool deep':
  x = torch.randn(N, 36, 48, 16, device=dev)
  w = torch.randn(3, 3, 16, 32, device=dev) * 0.1
  b = torch.randn(32, device=dev)
  tc = timeit(lambda: C.cf32_maxpool_fwd(C.cf32_conv_fwd(x, w, b, 1, 1, 1, 36, 48), 0, 0))
  tfp = timeit(lambda: C.cf32_wino_conv_pool_fwd(x, w, b))
  flop = 2.0 * N * 36 * 48 * 9 * 16 * 32
  print('%-26s fwd+pool: conv + maxpool %8.1f us | fused %8.1f us %6.1f TF' % (
      'head conv2 16->32 36x48', tc, tfp, flop / tfp / 1e6), flush=True)
if ONLY:
  sys.exit(0)
xp = torch.randn(N, 72, 96, 16, device=dev)
tp = timeit(lambda: C.cf32_maxpool_fwd(xp, 0, 0))
y, arg = C.cf32_maxpool_fwd(xp, 0, 0)
tb = timeit(lambda: C.cf32_maxpool_bwd(y, arg, 72, 96, 0, 0))
print('maxpool 72x96x16 fwd %.1f us bwd %.1f us' % (tp, tb))
