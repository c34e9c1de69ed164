#!/usr/bin/env python3
"""Winograd fp32 conv (csrc/kernels/conv_wino.hip) vs a float64 oracle at
learner-like batch sizes, every deep-torso 3x3/1 shape, forward (+ReLU-in,
residual, ReLU-out) and data gradient (+mask, skip add).  Prints the max
error relative to the output scale.  Usage: python tools/wino_check.py [N]"""
import sys
import torch

sys.path.insert(0, '.')
from scalable_agent_amd import ops  # noqa: E402
from scalable_agent_amd.models import layers  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 37
C = ops.ext()
dev = torch.device('cuda')
g = torch.Generator().manual_seed(0)
worst = 0.0
for (H, W, Ci, Co) in [(36, 48, 16, 16), (36, 48, 16, 32), (18, 24, 32, 32),
                       (9, 12, 32, 32), (11, 11, 32, 32), (36, 48, 32, 16)]:
  x = torch.randn(N, H, W, Ci, generator=g)
  w = torch.randn(3, 3, Ci, Co, generator=g) / (9 * Ci) ** 0.5
  b = torch.randn(Co, generator=g) * 0.1
  add = torch.randn(N, H, W, Co, generator=g)
  ref = layers.conv2d_same_nhwc(x.double().clamp(min=0), w.double(), b.double(), 1)
  ref = (ref + add.double()).clamp(min=0)
  y = C.cf32_conv_fwd(x.to(dev), w.to(dev), b.to(dev), 1, 1, 1, H, W,
                      relu_in=True, add=add.to(dev), relu_out=True)
  e1 = ((y.double().cpu() - ref).abs().max() / ref.abs().max()).item()
  dy = torch.randn(N, H, W, Co, generator=g)
  mask = torch.randn(N, H, W, Ci, generator=g)
  sk = torch.randn(N, H, W, Ci, generator=g)
  x64 = x.double().requires_grad_(True)
  yy = layers.conv2d_same_nhwc(x64, w.double(), None, 1)
  (dref,) = torch.autograd.grad(yy, x64, dy.double())
  dref = torch.where(mask.double() > 0, dref, torch.zeros_like(dref)) + sk.double()
  dx = C.cf32_conv_dgrad(dy.to(dev), w.to(dev), 1, 1, 1, H, W, mask=mask.to(dev),
                         add=sk.to(dev))
  e2 = ((dx.double().cpu() - dref).abs().max() / dref.abs().max()).item()
  # weight + bias gradient (ReLU on the input), accumulated into non-zero dW
  xin = x.double().clamp(min=0).requires_grad_(True)
  wd = w.double().requires_grad_(True)
  bd = b.double().requires_grad_(True)
  yy = layers.conv2d_same_nhwc(xin, wd, bd, 1)
  gw, gb = torch.autograd.grad(yy, (wd, bd), dy.double())
  if (Ci, Co) == (32, 16):  # only a data-gradient shape (no forward layer)
    worst = max(worst, e1, e2)
    print('%2dx%2d %2d->%2d  fwd rel %.2e  dgrad rel %.2e' % (H, W, Ci, Co, e1, e2))
    continue
  dw0 = torch.randn(3, 3, Ci, Co, generator=g)
  db0 = torch.randn(Co, generator=g)
  dw, db = dw0.to(dev), db0.to(dev)
  C.cf32_conv_wgrad(x.to(dev), dy.to(dev), 1, 1, 1, True, dw, db)
  e3 = ((dw.double().cpu() - dw0.double() - gw).abs().max() / gw.abs().max()).item()
  e4 = ((db.double().cpu() - db0.double() - gb).abs().max() / gb.abs().max()).item()
  worst = max(worst, e1, e2, e3, e4)
  print('%2dx%2d %2d->%2d  fwd rel %.2e  dgrad rel %.2e  wgrad rel %.2e  bgrad rel %.2e'
        % (H, W, Ci, Co, e1, e2, e3, e4), flush=True)
print('worst %.2e %s' % (worst, 'OK' if worst <= 1e-5 else 'FAIL'))
if worst > 1e-5:
  sys.exit(1)


def check_fused_bwd(N=37):
  """cf32_conv_bwd_fused == the float64 data + weight gradients."""
  worst = 0.0
  for (H, W, Cc) in [(36, 48, 16), (11, 11, 16), (9, 12, 32), (18, 24, 32)]:
    x = torch.randn(N, H, W, Cc, generator=g)
    w = torch.randn(3, 3, Cc, Cc, generator=g) / (9 * Cc) ** 0.5
    dy = torch.randn(N, H, W, Cc, generator=g)
    add = torch.randn(N, H, W, Cc, generator=g)
    for relu_x, use_add in ((False, False), (True, True)):
      x64 = x.double().requires_grad_(True)
      xin = x64.clamp(min=0) if relu_x else x64
      w64 = w.double().requires_grad_(True)
      b64 = torch.zeros(Cc, dtype=torch.float64, requires_grad=True)
      y = layers.conv2d_same_nhwc(xin, w64, b64, 1)
      gx, gw, gb = torch.autograd.grad(y, (x64, w64, b64), dy.double())
      # dX of the raw conv (x -> conv), masked by x > 0, + add
      x2 = x.double().requires_grad_(True)
      (gx2,) = torch.autograd.grad(layers.conv2d_same_nhwc(x2, w.double(), None, 1), x2,
                                   dy.double())
      ref = torch.where(x.double() > 0, gx2, torch.zeros_like(gx2))
      if use_add:
        ref = ref + add.double()
      dw = torch.zeros(3, 3, Cc, Cc, device=dev)
      db = torch.zeros(Cc, device=dev)
      dx = C.cf32_conv_bwd_fused(dy.to(dev), w.to(dev), x.to(dev), relu_x, dw, db,
                                 add=add.to(dev) if use_add else None)
      e = [((dx.double().cpu() - ref).abs().max() / ref.abs().max()).item(),
           ((dw.double().cpu() - gw).abs().max() / gw.abs().max()).item(),
           ((db.double().cpu() - gb).abs().max() / gb.abs().max()).item()]
      worst = max(worst, *e)
      print('fused bwd %2dx%2d C=%2d relu_x=%d add=%d: dx %.2e dw %.2e db %.2e' %
            (H, W, Cc, relu_x, use_add, *e), flush=True)
  return worst


if __name__ == '__main__':
  wf = check_fused_bwd()
  print('fused worst %.2e %s' % (wf, 'OK' if wf <= 1e-5 else 'FAIL'))
  sys.exit(0 if wf <= 1e-5 else 1)
