"""Per-(T,B) error-word probe of the gang LSTM kernels (word reset per case)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
from scalable_agent_amd import ops  # noqa: E402
from scalable_agent_amd.ops import lstm as lstm_ops  # noqa: E402


def main():
  C = ops.load()
  d = torch.device('cuda')
  H = 256
  errw = C.lstm_error_word(torch.empty(0, device=d))
  for T, B in [(2, 32), (2, 31), (2, 16), (2, 8), (2, 1), (2, 32), (37, 7)]:
    for zero_done in (True, False):
      torch.manual_seed(11)
      xw = torch.randn(T, B, 4 * H, device=d)
      done = (torch.rand(T, B, device=d) < 0.1).to(torch.uint8)
      if zero_done:
        done.zero_()
      c0 = torch.randn(B, H, device=d) * 0.5
      h0 = torch.randn(B, H, device=d) * 0.5
      w_h = torch.randn(H, 4 * H, device=d) * 0.05
      dh = torch.randn(T, B, H, device=d)
      lstm_ops.set_gang(False)
      hs, cs, acts, hpm, wt = C.lstm_fwd(xw, done, c0, h0, w_h)
      ref, rdc0, _ = C.lstm_bwd(dh, done, wt, acts, cs, c0, None, True)
      lstm_ops.set_gang(True)
      errw.zero_()
      hs, cs, acts, hpm, wt = C.lstm_fwd(xw, done, c0, h0, w_h)
      torch.cuda.synchronize()
      e1 = int(errw[0])
      dg, dc0, _ = C.lstm_bwd(dh, done, wt, acts, cs, c0, None, True)
      torch.cuda.synchronize()
      e2 = int(errw[0])
      rel = float((dg - ref).norm() / ref.norm())
      bad_units = ((dg - ref).abs() > 0.05 * ref.abs().max()).any(0).any(0).nonzero().flatten()
      print('T=%3d B=%2d zero_done=%d err fwd %d bwd %d rel %.2e bad cols %d %s' % (
          T, B, zero_done, e1, e2, rel, bad_units.numel(),
          sorted(set((bad_units % 256 // 32).tolist()))), flush=True)


if __name__ == '__main__':
  main()
