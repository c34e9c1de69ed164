"""Process-group setup and gradient synchronisation for DP learners.

One process per GPU (`torchrun`-style env: RANK, LOCAL_RANK, WORLD_SIZE,
MASTER_ADDR, MASTER_PORT).  Backend "nccl" == RCCL on ROCm for GPUs, "gloo"
for the CPU tests.

xGMI note: each MI355X has 7 point-to-point links (~153 GB/s each); the
gradient of this ~2 M-parameter model is ~6.5-8 MB fp32, i.e. latency-bound,
so it is reduced as ONE (or a few large) flat bucket(s) instead of per-tensor
calls; RCCL picks its all-peer algorithm for that size.  Buckets are the tail
of the flat buffer first (the LSTM/FC/head grads are produced first by
backward), so an eager backward can overlap the reduction of finished buckets
with the conv backward (`overlap=True`).
"""

import datetime
import os

import torch
import torch.distributed as dist


def world_info():
  rank = int(os.environ.get('RANK', '0'))
  world = int(os.environ.get('WORLD_SIZE', '1'))
  local = int(os.environ.get('LOCAL_RANK', str(rank)))
  return rank, world, local


def init_distributed(backend=None, timeout_s=600):
  """Initialises the default process group if WORLD_SIZE > 1.

  Returns (rank, world_size, local_rank).
  """
  rank, world, local = world_info()
  if world <= 1:
    return 0, 1, 0
  if not dist.is_initialized():
    if backend is None:
      # SA_DIST_BACKEND=gloo: rehearse the multi-rank GPU path on one card
      backend = os.environ.get('SA_DIST_BACKEND') or (
          'nccl' if torch.cuda.is_available() else 'gloo')
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29500')
    kwargs = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
    if backend == 'nccl':
      # a collective that times out aborts the process (instead of hanging
      # the job); torchrun --max-restarts + checkpoint auto-restore resume it
      os.environ.setdefault('TORCH_NCCL_ASYNC_ERROR_HANDLING', '1')
      # more ranks than visible GPUs (a one-card rehearsal): share the cards
      local = local % max(1, torch.cuda.device_count())
      torch.cuda.set_device(local)
      kwargs['device_id'] = torch.device('cuda', local)
    dist.init_process_group(**kwargs)
  return rank, world, local


def backend_info():
  """{'world_size', 'backend', 'rccl_version'} of the default group (for
  logs and the bench JSON: proves how many ranks the collective saw)."""
  info = {'world_size': 1, 'backend': None, 'rccl_version': None}
  if dist.is_initialized():
    info['world_size'] = dist.get_world_size()
    info['backend'] = dist.get_backend()
  try:
    if torch.cuda.is_available():
      v = torch.cuda.nccl.version()
      info['rccl_version'] = '.'.join(str(x) for x in v) if isinstance(
          v, tuple) else str(v)
  except Exception:  # pragma: no cover - build without RCCL
    pass
  return info


def cleanup():
  if dist.is_initialized():
    dist.destroy_process_group()


def broadcast_params(flat_params, src=0, group=None):
  """Initial weight broadcast so every replica starts identical."""
  if dist.is_initialized() and dist.get_world_size(group) > 1:
    dist.broadcast(flat_params, src=src, group=group)


def param_checksum_consistent(flat_params, group=None, rtol=0.0):
  """Consistency probe: all ranks hold bit-identical weights?"""
  if not (dist.is_initialized() and dist.get_world_size(group) > 1):
    return True
  s = torch.stack([flat_params.double().sum(),
                   flat_params.double().abs().sum()])
  mx = s.clone()
  mn = s.clone()
  dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
  dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=group)
  return bool(torch.all((mx - mn).abs() <= rtol * mx.abs()))


class GradientSynchronizer:
  """Flat-bucket gradient all-reduce for FlatParams-based learners."""

  def __init__(self, flat, group=None, reduce='sum', bucket_bytes=4 << 20,
               overlap=False, op=None):
    self.flat = flat
    self.group = group
    self.reduce = reduce
    # the reduction op (SUM; tools/micro/dp_queues.py uses AVG, which makes a
    # one-rank RCCL group launch a kernel the trace can place on its queue)
    self.op = dist.ReduceOp.SUM if op is None else op
    self.world = dist.get_world_size(group) if dist.is_initialized() else 1
    n = flat.numel
    per = max(1, bucket_bytes // 4)
    # buckets from the END of the buffer (produced first by backward)
    bounds = []
    hi = n
    while hi > 0:
      lo = max(0, hi - per)
      bounds.append((lo, hi))
      hi = lo
    self.buckets = bounds
    self.overlap = overlap
    self.split = None  # set_split(): [0, split) reduced before the rest
    self._works = []
    self._events = None
    self.last_time_s = 0.0  # device time of the latest finished all-reduce

  def set_split(self, offset):
    """Two-phase reduction: the gradients in [0, offset) (heads, core, torso
    FC: ~85 % of the parameters, produced first by backward) are all-reduced
    by begin_early() while the conv-torso backward still runs; all_reduce()
    then reduces [offset, n) and waits for both."""
    self.split = int(offset) if 0 < offset < self.flat.numel else None
    # the step guard's NaN sentinel (Learner._apply writes it AFTER the early
    # bucket went out) must travel with the late bucket
    sentinel = getattr(self.flat, 'sentinel', None)
    if self.split is not None and sentinel is not None:
      assert sentinel >= self.split, (sentinel, self.split)

  def _mark_start(self):
    g = self.flat.grads
    if not g.is_cuda:
      return
    if self._events is None:
      self._events = (torch.cuda.Event(enable_timing=True),
                      torch.cuda.Event(enable_timing=True))
    elif self._events[1].query():
      # previous step's collective has finished: harvest its duration
      self.last_time_s = self._events[0].elapsed_time(self._events[1]) / 1e3
    self._events[0].record()

  def _stream_ordered(self):
    """RCCL collectives on GPU tensors are issued stream-ordered
    (async_op=False): ProcessGroupNCCL runs them on the CURRENT stream, so
    the caller's stream - the stream plan's early stream with its own
    hardware queue, or the compute stream - decides where they run
    (parallel/streams.py).  gloo keeps async work handles."""
    g = self.flat.grads
    return g.is_cuda and dist.get_backend(self.group) == 'nccl'

  def begin_early(self):
    """Launches the all-reduce of the early bucket, ordered after the work
    already enqueued on the current stream (Learner: the stream plan's early
    stream, so it runs beside the conv-torso backward)."""
    if self.world <= 1 or self.split is None or self._works:
      return
    self._mark_start()
    g = self.flat.grads[:self.split]
    if self._stream_ordered():
      dist.all_reduce(g, op=self.op, group=self.group)
      done = torch.cuda.Event()
      done.record()
      self._works = [done]
    else:
      self._works = [dist.all_reduce(g, op=self.op, group=self.group,
                                     async_op=True)]

  def all_reduce(self):
    """Reduces what begin_early did not and leaves the current stream
    ordered after every reduction."""
    if self.world <= 1:
      return
    g = self.flat.grads
    timed = g.is_cuda
    if self.split is not None:
      if not self._works:  # no early phase this step: reduce both now
        self.begin_early()
      works = self._works
      self._works = []
      for w in works:
        if isinstance(w, torch.cuda.Event):
          torch.cuda.current_stream(g.device).wait_event(w)
      late = g[self.split:]
      if self._stream_ordered():
        dist.all_reduce(late, op=self.op, group=self.group)
      else:
        works = works + [dist.all_reduce(late, op=self.op, group=self.group,
                                         async_op=True)]
      for w in works:
        if not isinstance(w, torch.cuda.Event):
          w.wait()
      if self.reduce == 'mean':
        g.div_(self.world)
      if timed:
        self._events[1].record()
      return
    if timed:
      self._mark_start()
    if len(self.buckets) == 1 or self._stream_ordered():
      for lo, hi in (self.buckets if len(self.buckets) > 1 else [(0, None)]):
        dist.all_reduce(g[lo:hi], op=self.op, group=self.group)
    else:
      works = [dist.all_reduce(g[lo:hi], op=self.op, group=self.group,
                               async_op=True)
               for lo, hi in self.buckets]
      for w in works:
        w.wait()
    if self.reduce == 'mean':
      g.div_(self.world)
    if timed:
      self._events[1].record()
