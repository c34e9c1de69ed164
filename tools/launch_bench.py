#!/usr/bin/env python3
"""Calibrates the per-launch cost of dependent kernels in a hipGraph on this
GPU (noop kernels of several geometries) and times the LSTM step kernels."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from scalable_agent_amd import ops

C = ops.ext()
dev = torch.device('cuda', 0)
cnt = torch.zeros(1, dtype=torch.int32, device=dev)


def graph_time(fn, reps=20):
  s = torch.cuda.Stream()
  s.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(s):
    fn()
  torch.cuda.current_stream().wait_stream(s)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    fn()
  g.replay()
  torch.cuda.synchronize()
  t = time.perf_counter()
  for _ in range(reps):
    g.replay()
  torch.cuda.synchronize()
  return (time.perf_counter() - t) / reps


N = 200
for blocks, threads in [(1, 64), (64, 256), (64, 1024), (256, 256), (1024, 256)]:
  t = graph_time(lambda: [C.noop(blocks, threads, cnt) for _ in range(N)])
  print('noop grid=%5d x %4d : %.2f us/launch (graph)' % (blocks, threads, 1e6 * t / N))

T, B, H = 101, 32, 256
xw = torch.randn(T, B, 4 * H, device=dev)
done = (torch.rand(T, B, device=dev) < 0.01).to(torch.uint8)
c0 = torch.zeros(B, H, device=dev)
h0 = torch.zeros(B, H, device=dev)
wh = torch.randn(H, 4 * H, device=dev) * 0.05
t = graph_time(lambda: C.lstm_fwd(xw, done, c0, h0, wh))
print('lstm_fwd T=101: %.1f us total, %.2f us/step' % (1e6 * t, 1e6 * t / T))
hs, cs, acts = C.lstm_fwd(xw, done, c0, h0, wh)
dh = torch.randn_like(hs)
t = graph_time(lambda: C.lstm_bwd(dh, done, wh, acts, cs, c0))
print('lstm_bwd T=101: %.1f us total, %.2f us/step' % (1e6 * t, 1e6 * t / T))
