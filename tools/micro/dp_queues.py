"""Which hardware queue each stream of the data-parallel learner path runs on
(parallel/streams.py).

Run under rocprofv3 on ONE GPU with a world-size-1 RCCL group (with
GPU_MAX_HW_QUEUES=4, HIP's default, to check the first-use order alone; with
8, as bench.py sets it - on the rocprofv3 command line either way):

  GPU_MAX_HW_QUEUES=4 rocprofv3 --kernel-trace --memory-copy-trace -d OUT -o run -- \
      python3 tools/micro/dp_queues.py
  python3 tools/micro/dp_queues.py --parse OUT/<host>/<pid>/run_results.db

The probe brings the process up exactly as bench.py does (the stream plan,
created and first used; the RCCL group with device_id; the warm-up
collective), captures a small HIP learner step (warm-up
on the plan's capture stream) and replays it on the default stream, and
issues the early all-reduce from the plan's early stream after a host wait
(Learner.graph_step itself, with the synchronizer told world 2).  Each stream also runs one marker kernel: a
fill of its own dtype, so the trace names the stream:
  default (compute) bool | copy int16 | capture float64 | early int8.
The copy stream also runs the H2D batch copy.  --parse prints the queue and
stream ids of the markers, of the learner step's kernels, of RCCL's kernels
and of the copies."""

import collections
import os
import sqlite3
import sys

MARKERS = {'bool': 'default (compute)', 'short': 'copy',
           'double': 'capture', 'signed char': 'early'}


def probe():
  root = os.path.dirname(os.path.dirname(os.path.dirname(
      os.path.abspath(__file__))))
  sys.path.insert(0, root)
  import datetime
  import torch
  import torch.distributed as dist
  from scalable_agent_amd import flags as flags_lib
  from scalable_agent_amd import ops, parallel
  from scalable_agent_amd.envs.synthetic import make_synthetic_batch
  from scalable_agent_amd.learner import Learner, batch_to_device
  from scalable_agent_amd.models import Agent

  os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
  os.environ.setdefault('MASTER_PORT', '29533')
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(dev)
  # as bench.py: the stream plan (created and first used) before RCCL's
  # init, then the group as parallel.init_distributed makes it (device_id:
  # eager communicator), then the warm-up collective
  plan = parallel.stream_plan(dev)
  dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev,
                          timeout=datetime.timedelta(seconds=120))
  parallel.warmup_collective(dev)
  ops.load()

  def mark(stream, dtype):
    with torch.cuda.stream(stream):
      torch.empty(1 << 16, dtype=dtype, device=dev).fill_(1)

  # the headline learner shape: the early bucket's all-reduce is issued while
  # the ~5 ms torso-backward graph runs, so the trace shows whether they overlap
  B, T = 32, 100
  f = flags_lib.default_flags(batch_size=B, unroll_length=T, torso='deep')
  agent = Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=1,
                backend='hip', compute_dtype=torch.float32)
  # the data-parallel learner (split backward graphs, early all-reduce from
  # the plan's early stream); the one-rank group reports world 1, so the
  # synchronizer is told 2 and reduces with AVG, which makes RCCL launch a
  # kernel (oneRankReduce) the trace can place on a queue
  lrn = Learner(agent, f, dev, world_size=2)
  lrn.grad_sync.world = 2
  lrn.grad_sync.op = dist.ReduceOp.AVG
  assert lrn._split
  batch = batch_to_device(make_synthetic_batch(B, T, (72, 96, 3), 9), dev)
  lrn.capture(batch)
  host = torch.empty(8 << 20, dtype=torch.uint8).pin_memory()
  slab = torch.empty(8 << 20, dtype=torch.uint8, device=dev)
  for _ in range(3):
    mark(torch.cuda.current_stream(dev), torch.bool)
    mark(plan.capture, torch.float64)
    with torch.cuda.stream(plan.copy):
      slab.copy_(host, non_blocking=True)
    mark(plan.copy, torch.int16)
    mark(plan.early, torch.int8)
    lrn.graph_step()  # graph 0, host wait, early bucket, graph 1, late bucket
    torch.cuda.synchronize()
  print('probe done', flush=True)
  dist.destroy_process_group()


def parse(path):
  c = sqlite3.connect(path)
  rows = list(c.execute('select name, queue_id, stream_id from kernels'))
  q_of = collections.defaultdict(collections.Counter)
  learner = collections.Counter()
  rccl = collections.Counter()
  for name, q, s in rows:
    if 'FillFunctor' in name:
      for key, who in MARKERS.items():
        if 'FillFunctor<%s>' % key in name:
          q_of[who][(q, s)] += 1
    elif name.startswith('void sa::') or name.startswith('sa::'):
      learner[(q, s)] += 1
    elif ('nccl' in name.lower() or 'rccl' in name.lower() or
          'oneRank' in name):
      rccl[(q, s, name[:70])] += 1
  print('stream marker            (queue_id, stream_id): kernels')
  for who in MARKERS.values():
    print('  %-22s %s' % (who, dict(q_of[who])))
  print('learner step kernels (sa::*)  %s' % dict(learner))
  print('RCCL kernels:')
  for (q, s, n), k in sorted(rccl.items()):
    print('  queue %s stream %s x%d  %s' % (q, s, k, n))
  # does each RCCL kernel run while a learner kernel on another queue runs?
  full = list(c.execute('select name, queue_id, start, end from kernels '
                        'order by start'))
  lk = [r for r in full if r[0].startswith(('void sa::', 'sa::'))]
  for name, q, t0, t1 in full:
    if 'nccl' not in name.lower() and 'rccl' not in name.lower() and \
        'oneRank' not in name:
      continue
    beside = [r for r in lk if r[1] != q and r[2] < t1 and r[3] > t0]
    print('  %s on queue %s: %.1f us, beside %d learner kernel(s) on '
          'queues %s' % (name[:50], q, (t1 - t0) / 1e3,
                         len(beside), sorted({r[1] for r in beside})))
  try:
    cp = collections.Counter(c.execute(
        'select queue_id, stream_id from memory_copies'))
    print('memory copies (queue_id, stream_id): %s' % dict(cp))
  except sqlite3.Error as e:
    print('memory copies: %s' % e)


if __name__ == '__main__':
  if len(sys.argv) > 2 and sys.argv[1] == '--parse':
    parse(sys.argv[2])
  else:
    probe()
