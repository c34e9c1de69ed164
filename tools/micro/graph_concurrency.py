"""Does a captured hipGraph run independent branches concurrently on MI355X?

Two branches: A = a chain of small dependent kernels (latency-bound, like the
LSTM steps), B = a few big matmuls (throughput-bound, like the conv torso).
Times each alone, both serialized on one stream, and both forked onto two
streams, eager and graph-captured.  If the forked graph time is close to
max(A, B) the replay overlaps branches.
"""
import time

import torch


def main():
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(dev)
  a = torch.randn(32, 256, device=dev)
  w = torch.randn(256, 256, device=dev) * 0.05
  x = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
  y = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
  out = torch.empty_like(x)
  s_main = torch.cuda.current_stream()
  s2 = torch.cuda.Stream()

  def chain():
    h = a
    for _ in range(200):
      h = torch.tanh(h @ w)
    return h

  def big():
    for _ in range(6):
      torch.matmul(x, y, out=out)

  def forked():
    s2.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s2):
      chain()
    big()
    torch.cuda.current_stream().wait_stream(s2)

  def serial():
    chain()
    big()

  def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
      fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3

  res = {}
  for name, fn in [('chain', chain), ('big', big), ('serial', serial),
                   ('forked', forked)]:
    res['eager_' + name] = timeit(fn)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
      fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
      fn()
    res['graph_' + name] = timeit(g.replay)
  for k, v in res.items():
    print('%-16s %8.3f ms' % (k, v))


if __name__ == '__main__':
  main()
