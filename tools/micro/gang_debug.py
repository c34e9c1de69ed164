"""Repeatability / accuracy probe of the gang LSTM kernels over (T, B)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
from scalable_agent_amd import ops  # noqa: E402
from scalable_agent_amd.ops import lstm as lstm_ops  # noqa: E402

NAMES = ['hs', 'cs', 'acts', 'hpm', 'dg', 'dc0', 'dg16']


def run(C, args):
  hs, cs, acts, hpm, wt = C.lstm_fwd(*args[:5])
  dg, dc0, dg16 = C.lstm_bwd(args[5], args[1], wt, acts, cs, args[2], args[6], True)
  return [hs, cs, acts, hpm, dg, dc0, dg16.float()]


def main():
  C = ops.load()
  d = torch.device('cuda')
  H = 256
  ws = int(sys.argv[1]) if len(sys.argv) > 1 else 1
  C.lstm_gang_ws(ws)
  for T, B in [(37, 7), (37, 8), (37, 32), (101, 7), (101, 32), (4, 7), (2, 1)]:
    torch.manual_seed(11)
    xw = torch.randn(T, B, 4 * H, device=d)
    done = (torch.rand(T, B, device=d) < 0.1).to(torch.uint8)
    c0 = torch.randn(B, H, device=d) * 0.5
    h0 = torch.randn(B, H, device=d) * 0.5
    w_h = torch.randn(H, 4 * H, device=d) * 0.05
    dh = torch.randn(T, B, H, device=d)
    dcl = torch.randn(B, H, device=d)
    args = (xw, done, c0, h0, w_h, dh, dcl)
    lstm_ops.set_gang(False)
    ref = run(C, args)
    lstm_ops.set_gang(True)
    runs = [run(C, args) for _ in range(3)]
    torch.cuda.synchronize()
    for i, n in enumerate(NAMES):
      bad = [(runs[0][i] != r[i]) for r in runs[1:]]
      nb = sum(int(b.sum()) for b in bad)
      msg = ''
      if nb:
        idx = bad[0].nonzero()
        msg = 'first diffs %s' % idx[:4].tolist()
        if idx.shape[1] == 3:
          msg += ' t-range %d..%d cols %s' % (int(idx[:, 0].min()), int(idx[:, 0].max()),
                                             sorted(set((idx[:, 2] % 256).tolist()))[:8])
      rel = float((runs[0][i] - ref[i]).norm() / ref[i].norm().clamp_min(1e-12))
      print('T=%3d B=%2d %-5s nondet=%6d rel_vs_fp32=%.2e %s' % (T, B, n, nb, rel, msg),
            flush=True)
  print('error word', lstm_ops.persistent_error(d))


if __name__ == '__main__':
  main()
