#!/usr/bin/env python3
"""Per-shape timing of the exact-fp32 learner GEMMs (kernels/gemm_f32.hip).

The seven products of one fp32 learner step (ops/core.py _CoreLSTMF32) at
B=32, T=100 (N = 3232 rows), 9 actions, with their epilogues; achieved TFLOP/s
against the 157 TF fp32 MFMA peak.  Knobs (SA_GEMM_WG_TARGET, SA_GEMM_RM,
SA_GEMM_BL) are read once per process.
usage: python tools/gemm_f32_bench.py [reps]
"""
import sys

import torch

sys.path.insert(0, '.')
from scalable_agent_amd import ops  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
C = ops.ext()
dev = torch.device('cuda')
N, F, H, G, K = 3232, 3456, 256, 1024, 272  # rows, feats, core, gates, aug
g = torch.Generator(device='cpu').manual_seed(0)


def r(*s):
  return torch.randn(*s, generator=g).to(dev)


feats, w_fc, b_fc = r(N, F), r(F, H) * 0.02, r(H)
h_aug, kx, bias = r(N, K), r(K + H, G) * 0.05, r(G)
dg, dh, hpm = r(N, G), r(N, H), r(N, H)
rew = r(N)
act = torch.randint(0, 9, (N,), device=dev)
out_aug = torch.empty(N, K, device=dev)
xw = torch.empty(N, G, device=dev)
dh_o = torch.empty(N, H, device=dev)
dfeats = torch.empty(N, F, device=dev)
gk = torch.zeros(K + H, G, device=dev)
gb = torch.zeros(G, device=dev)
gwfc = torch.zeros(F, H, device=dev)
gbfc = torch.zeros(H, device=dev)

CASES = [
    ('fc fwd  [N,F]x[F,256] +bias relu aug', 2 * N * F * H,
     lambda: C.gemm_f32(feats, w_fc, False, False, out_aug, bias=b_fc, relu=True,
                        aug_reward=rew, aug_action=act)),
    ('xproj   [N,272]x[272,1024] +bias', 2 * N * K * G,
     lambda: C.gemm_f32(h_aug, kx[:K], False, False, xw, bias=bias)),
    ('dh      [N,1024]x[256,1024]^T mask', 2 * N * G * H,
     lambda: C.gemm_f32(dg, kx[:H], False, True, dh_o, mask=h_aug[:, :H])),
    ('dfeats  [N,256]x[3456,256]^T mask', 2 * N * H * F,
     lambda: C.gemm_f32(dh, w_fc, False, True, dfeats, mask=feats)),
    ('dW_h    [N,256]^Tx[N,1024] acc', 2 * N * H * G,
     lambda: C.gemm_f32(hpm, dg, True, False, gk[K:], accumulate=True)),
    ('dW_x    [N,272]^Tx[N,1024] acc colsum', 2 * N * K * G,
     lambda: C.gemm_f32(h_aug, dg, True, False, gk[:K], accumulate=True, colsum=gb)),
    ('dW_fc   [N,3456]^Tx[N,256] acc colsum', 2 * N * F * H,
     lambda: C.gemm_f32(feats, dh, True, False, gwfc, accumulate=True, colsum=gbfc)),
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
  return s.elapsed_time(e) * 1e3 / REPS


tot_us = tot_fl = 0.0
for name, flops, fn in CASES:
  us = timeit(fn)
  tot_us += us
  tot_fl += flops
  print('%-40s %8.1f us  %6.1f TF' % (name, us, flops / us / 1e6))
print('%-40s %8.1f us  %6.1f TF' % ('total', tot_us, tot_fl / tot_us / 1e6))
