"""H2D bandwidth from pinned host memory: one 67 MB copy (the learner batch's
frames) on a side stream, alone and concurrently with compute."""
import time
import torch

n = 101 * 32 * 72 * 96 * 3
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device='cuda')
s = torch.cuda.Stream()
for rep in range(3):
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  with torch.cuda.stream(s):
    d.copy_(h, non_blocking=True)
  s.synchronize()
  dt = time.perf_counter() - t0
  print('pinned H2D %.1f MB: %.3f ms = %.1f GB/s' % (n / 1e6, dt * 1e3, n / dt / 1e9))
# 8 MB chunks
torch.cuda.synchronize()
t0 = time.perf_counter()
with torch.cuda.stream(s):
  for i in range(0, n, 8 << 20):
    d[i:i + (8 << 20)].copy_(h[i:i + (8 << 20)], non_blocking=True)
s.synchronize()
dt = time.perf_counter() - t0
print('chunked 8MB: %.3f ms = %.1f GB/s' % (dt * 1e3, n / dt / 1e9))
