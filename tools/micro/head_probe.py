"""Times the fused learner-head kernels standalone over B and T."""
import sys
import torch
sys.path.insert(0, '.')
from scalable_agent_amd import ops  # noqa: E402


def t_us(fn, reps=50):
  """GPU time per call, from a hipGraph of `reps` calls (no host overhead)."""
  s0 = torch.cuda.Stream()
  s0.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(s0):
    for _ in range(3):
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
  A = 9
  for B, T in [(32, 100), (1, 100), (8, 100), (32, 10), (32, 1), (64, 100)]:
    T1 = T + 1
    core = torch.randn(T1, B, 256, device=d)
    wp = torch.randn(256, A, device=d)
    bp = torch.randn(A, device=d)
    wb = torch.randn(256, device=d)
    bb = torch.randn(1, device=d)
    beh = torch.randn(T1, B, A, device=d)
    act = torch.randint(0, A, (T1, B), device=d)
    rew = torch.randn(T1, B, device=d)
    done = torch.zeros(T1, B, dtype=torch.bool, device=d)
    tk = torch.zeros(1, dtype=torch.int32, device=d)
    f = lambda: C.learner_head_fwd(core, wp, bp, wb, bb, beh, act, rew, done,
                                   tk, 0.99, 0, 1.0, 1.0, 0.5, 0.01)
    loss, dl, dv = f()
    g = torch.ones(1, device=d)
    gw = [torch.zeros_like(wp), torch.zeros_like(bp), torch.zeros_like(wb),
          torch.zeros_like(bb)]
    fb = lambda: C.learner_head_bwd(g, core, dl, dv, wp, wb, *gw)
    print('B=%3d T=%3d fwd %7.1f us  bwd %7.1f us' % (B, T, t_us(f), t_us(fb)))


if __name__ == '__main__':
  main()
