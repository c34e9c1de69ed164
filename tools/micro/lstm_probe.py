"""Times the LSTM recurrence kernels (per-step, persistent fp32, 8-workgroup
bf16 gang) in a hipGraph."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
from scalable_agent_amd import ops  # noqa: E402
from scalable_agent_amd.ops import lstm as lstm_ops  # noqa: E402


def t_us(fn, reps=20):
  s0 = torch.cuda.Stream()
  s0.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(s0):
    for _ in range(2):
      fn()
  torch.cuda.current_stream().wait_stream(s0)
  torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(reps):
      fn()
  g.replay()
  torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record()
  g.replay()
  e.record()
  torch.cuda.synchronize()
  return s.elapsed_time(e) / reps * 1e3


def main():
  C = ops.load()
  d = torch.device('cuda')
  T, B, H = 101, 32, 256
  xw = torch.randn(T, B, 4 * H, device=d)
  done = (torch.rand(T, B, device=d) < 0.02).to(torch.uint8)
  c0 = torch.randn(B, H, device=d) * 0.5
  h0 = torch.randn(B, H, device=d) * 0.5
  w_h = torch.randn(H, 4 * H, device=d) * 0.05
  dh = torch.randn(T, B, H, device=d)
  modes = [('step', 4, 1), ('persistent', 1, 1), ('gang_ws', 1, 1)]
  modes += [('gang', 1, nap) for nap in (0, 1, 2, 4, 8, 16, 1, 0)]
  for mode, xp, nap in modes:
    lstm_ops.set_persistent(mode == 'persistent')
    lstm_ops.set_gang(mode.startswith('gang'))
    C.lstm_gang_ws(1 if mode == 'gang_ws' else 0)
    C.lstm_gang_nap(nap)
    C.lstm_xpack(xp)
    m = C.lstm_mode(H, B, T, False)
    hs, cs, acts, hpm, wt = C.lstm_fwd(xw, done, c0, h0, w_h, m)
    f = lambda: C.lstm_fwd(xw, done, c0, h0, w_h, m)
    b = lambda: C.lstm_bwd(dh, done, wt, acts, cs, c0, None, True, m)
    print('%-10s xpack=%d nap=%2d fwd %8.1f us  bwd %8.1f us' % (mode, xp, nap, t_us(f), t_us(b)),
          flush=True)
  print('error word', lstm_ops.persistent_error(d))


if __name__ == '__main__':
  main()
