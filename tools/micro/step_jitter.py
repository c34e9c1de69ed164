#!/usr/bin/env python3
"""Per-step time distribution of the graph-replayed learner step (no H2D
prefetch, no profiler): K steps each bracketed by events, percentiles and
the slowest steps.  usage: python tools/micro/step_jitter.py [fp32|bf16] [K] [one|two|h2d|h2d_thp|h2d_mid|h2d_chunk|d2d|ev|w_done|rec|hw_ready|hw_both|side|w_pending|x_wait|x_wait_k|dp0|dpA|dpB|dpC]"""
import os
import sys

import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
from scalable_agent_amd import flags as flags_lib  # noqa: E402
from scalable_agent_amd.envs.synthetic import make_synthetic_batch  # noqa: E402
from scalable_agent_amd.learner import FlatStaging, Learner  # noqa: E402
from scalable_agent_amd.models import Agent  # noqa: E402

dtype = sys.argv[1] if len(sys.argv) > 1 else 'bf16'
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
dev = torch.device('cuda')
copy_stream = torch.cuda.Stream()  # the process's first stream, as bench.py
flags = flags_lib.default_flags(batch_size=32, unroll_length=100, torso='deep', dtype=dtype)
agent = Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=1, backend='hip',
              compute_dtype=torch.bfloat16 if dtype == 'bf16' else torch.float32)
learner = Learner(agent, flags, dev)
hb = make_synthetic_batch(32, 100, (72, 96, 3), 9, seed=3, pin_memory=False)
mode = sys.argv[3] if len(sys.argv) > 3 else 'one'
graphs, dev_flat = [], []
host_flat = FlatStaging(hb, 'cpu', pin=True).load(hb)
if mode == 'h2d_thp':
  # the same bytes in a 2 MiB-aligned transparent-huge-page mapping,
  # registered with the HIP runtime torch loaded (fewer host translations)
  import ctypes
  import mmap
  import numpy as np
  A = 2 << 20
  size = (host_flat.nbytes + A - 1) // A * A
  mm = mmap.mmap(-1, size + A, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
  base = ctypes.addressof(ctypes.c_char.from_buffer(mm))
  off = (-base) % A
  mm.madvise(mmap.MADV_HUGEPAGE, off, size)
  arr = np.frombuffer(mm, dtype=np.uint8, count=size, offset=off)
  arr[:host_flat.nbytes] = host_flat.flat[:host_flat.nbytes].numpy()
  lib = [l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l][0]
  hip = ctypes.CDLL(lib)
  rc = hip.hipHostRegister(ctypes.c_void_p(base + off), ctypes.c_size_t(size),
                           ctypes.c_uint(0))
  print('thp:', open('/sys/kernel/mm/transparent_hugepage/enabled').read().strip(),
        'register rc', rc, [l.strip() for l in open('/proc/self/smaps_rollup')
                            if 'AnonHuge' in l])
  host_flat.flat = torch.from_numpy(arr)
  print('pinned:', host_flat.flat.is_pinned())
mid_ev = torch.cuda.Event()
side_buf = torch.zeros(1024, device=dev)
src_dev = host_flat.flat[:host_flat.nbytes].to(dev) if mode == 'd2d' else None
nxt = [0]


def prefetch(after):
  k = nxt[0]
  j = (k + 1) % len(graphs)
  with torch.cuda.stream(copy_stream):
    copy_stream.wait_event(after)
    c = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    c[0].record(copy_stream)
    if mode == 'ev':  # the event protocol alone, no copy
      pass
    elif mode == 'd2d':  # same bytes device -> device (no PCIe, no host)
      dev_flat[j].flat.copy_(src_dev, non_blocking=True)
    elif mode == 'h2d_chunk':  # 16 copies of 1/16 each
      n = host_flat.nbytes
      for c0 in range(0, n, (n + 15) // 16):
        c1 = min(n, c0 + (n + 15) // 16)
        dev_flat[j].flat[c0:c1].copy_(host_flat.flat[c0:c1], non_blocking=True)
    else:
      dev_flat[j].copy_from(host_flat)
    c[1].record(copy_stream)
    cev.append(c)
    slot_ready[j].record(copy_stream)


def mid_hook():
  mid_ev.record(comp)
  prefetch(mid_ev)


if mode.startswith('dp'):
  # data-parallel stream pattern on one GPU: split graphs (forward + late
  # backward, then the conv-torso backward), a stand-in for each all-reduce
  # bucket on a side stream (10 passes over the bucket, ~ a collective's time)
  learner._split = True
  split = learner._torso_offset()
  side = torch.cuda.Stream()
  ev0, ev1 = torch.cuda.Event(), torch.cuda.Event()
for _ in range(1 if mode in ('one', 'w_done', 'rec', 'side', 'w_pending', 'x_wait', 'x_wait_k') else 2):
  dev_flat.append(FlatStaging(hb, dev).load(hb))
  learner.capture(dev_flat[-1].views, clone=False)
  graphs.append((learner._graph, learner._static_in, learner._static_loss,
                 getattr(learner, '_graph_keep', None)))


slot_free = [torch.cuda.Event(), torch.cuda.Event()]
slot_ready = [torch.cuda.Event(), torch.cuda.Event()]
for e in slot_ready + slot_free:
  e.record()
slot_ready[0].record(copy_stream)
comp = torch.cuda.current_stream()


host_t = []  # host seconds per graph_step() call
cev = []  # (start, end) of each prefetch copy
wev = []  # compute-stream events around the wait for the slot


def dp_bucket(lo, hi):
  g = learner.flat.grads[lo:hi]
  for _ in range(10):
    g.mul_(1.0)


dp_t = [0.0, 0.0, 0.0, 0]  # host seconds in g0 / g1 replay / _apply, steps


def dp_step(m):
  g0, g1 = learner._graph
  n = learner.flat.grads.numel()
  t0 = time.perf_counter()
  g0.replay()
  dp_t[0] += time.perf_counter() - t0
  dp_t[3] += 1
  if m == 'dpA':  # device-side waits (torch.distributed's pattern)
    side.wait_stream(comp)
    with torch.cuda.stream(side):
      dp_bucket(0, split)
    g1.replay()
  elif m in ('dpB', 'dpC'):  # early bucket enqueued once the host saw g0 end
    ev0.record(comp)
    g1.replay()
    ev0.synchronize()
    with torch.cuda.stream(side):
      dp_bucket(0, split)
  else:
    t0 = time.perf_counter()
    g1.replay()
    dp_t[1] += time.perf_counter() - t0
  if m in ('dpA', 'dpB'):
    side.wait_stream(comp)
  elif m == 'dpC':
    ev1.record(comp)
    ev1.synchronize()
  if m != 'dp0':
    with torch.cuda.stream(side):
      dp_bucket(split, n)
    comp.wait_stream(side)
  t0 = time.perf_counter()
  learner._apply()
  dp_t[2] += time.perf_counter() - t0


def step(k):
  # 'h2d': bench.py's loop (prefetch of the next batch on a copy stream)
  i, j = k % len(graphs), (k + 1) % len(graphs)
  nxt[0] = k
  if mode == 'side':  # the DP all-reduce's stream pattern, a tiny kernel
    comp.wait_event(slot_ready[0])
  if mode == 'w_pending':  # wait on a copy-stream record enqueued just now
    slot_ready[0].record(copy_stream)
    comp.wait_event(slot_ready[0])
  if mode == 'x_wait_k':  # the same after one tiny kernel behind the graph
    side_buf.add_(1.0)
  if mode in ('x_wait', 'x_wait_k'):  # another stream waits on the compute stream
    slot_free[0].record(comp)
    copy_stream.wait_event(slot_free[0])
    slot_ready[0].record(copy_stream)
  if mode == 'w_done':  # wait on a copy-stream event completed long ago
    comp.wait_event(slot_ready[0])
  if mode == 'rec':  # record a (non-timing) event on the compute stream only
    slot_free[i].record(comp)
  if mode in ('hw_ready', 'hw_both'):
    slot_ready[i].synchronize()  # complete at enqueue: no device-side wait
  if mode.startswith('h2d') or mode in ('d2d', 'ev'):
    w = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    w[0].record(comp)
    comp.wait_event(slot_ready[i])
    w[1].record(comp)
    wev.append(w)
  (learner._graph, learner._static_in, learner._static_loss,
   learner._graph_keep) = graphs[i]
  t = time.perf_counter()
  if mode.startswith('dp'):
    dp_step(mode)
  else:
    learner.graph_step()
  host_t.append(time.perf_counter() - t)
  if (mode.startswith('h2d') or mode in ('d2d', 'ev')) and mode != 'h2d_mid':
    slot_free[i].record(comp)
    prefetch(slot_free[j])
  if mode == 'side':
    slot_free[0].record(comp)
    with torch.cuda.stream(copy_stream):
      copy_stream.wait_event(slot_free[0])
      side_buf.add_(1.0)
      slot_ready[0].record(copy_stream)
  if mode == 'hw_ready':  # device-side wait for the copy's start only
    slot_free[i].record(comp)
    with torch.cuda.stream(copy_stream):
      copy_stream.wait_event(slot_free[j])
      dev_flat[j].copy_from(host_flat)
      slot_ready[j].record(copy_stream)
  if mode == 'hw_both':  # host waits for slot j's previous step, then copies
    slot_free[i].record(comp)
    slot_free[j].synchronize()
    with torch.cuda.stream(copy_stream):
      dev_flat[j].copy_from(host_flat)
      slot_ready[j].record(copy_stream)


for k in range(5):
  step(k)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
ev[0].record()
for k in range(K):
  step(k)
  ev[k + 1].record()
torch.cuda.synchronize()
raw = [ev[k].elapsed_time(ev[k + 1]) for k in range(K)]
print('per 25-step block means:', ' '.join(
    '%.3f' % (sum(raw[b:b + 25]) / len(raw[b:b + 25])) for b in range(0, K, 25)))
ts = sorted(raw)
if cev:
  cd = sorted(a.elapsed_time(b) for a, b in cev[-K:])
  wd = sorted(a.elapsed_time(b) for a, b in wev[-K:])
  print('copy ms: p50 %.3f p90 %.3f max %.3f; slot wait ms: p50 %.3f p90 %.3f max %.3f' % (
      cd[len(cd) // 2], cd[int(len(cd) * .9)], cd[-1], wd[len(wd) // 2],
      wd[int(len(wd) * .9)], wd[-1]))
mean = sum(ts) / K
print('%s/%s: %d steps, mean %.3f ms, p50 %.3f, p90 %.3f, p99 %.3f, max %.3f' % (
    dtype, mode, K, mean, ts[K // 2], ts[int(K * .9)], ts[int(K * .99)], ts[-1]))
ht = sorted(host_t[-K:])
print('host graph_step ms: p50 %.3f p90 %.3f max %.3f' % (
    1e3 * ht[K // 2], 1e3 * ht[int(K * .9)], 1e3 * ht[-1]))
if dp_t[3]:
  print('dp host ms per step: g0 %.3f g1 %.3f apply %.3f' % tuple(
      1e3 * x / dp_t[3] for x in dp_t[:3]))
print('slowest:', ['%.3f' % t for t in ts[-8:]])
print('mean without the 2 %% slowest: %.3f ms' % (sum(ts[:int(K * .98)]) / int(K * .98)))
