"""The learner process's HIP streams, created once, in a fixed order.

HIP backs streams with GPU_MAX_HW_QUEUES (4 by default) hardware queues
per device.  Two streams on one queue are serialised by the queue's barrier
packets:

  * the 67 MB H2D batch prefetch on the compute stream's queue costs its
    full 1.2 ms per step (bench.py; profiles/experiments.md round 3);
  * the data-parallel early all-reduce on the compute queue would wait for
    the whole conv-torso backward instead of running beside it.

Measured (tools/micro/queue_map.py and dp_queues.py under rocprofv3 on one
MI355X, profiles/r6_dp_queues.txt): a stream takes its queue at its FIRST
USE, not at its creation.  With 4 queues the first four streams used get
queues of their own and the next ones share (the 5th shares the 4th's
queue, the 6th the 3rd's, ...); high-priority streams get queues of their
own.  RCCL's init uses internal streams, so a stream first used after
`init_process_group` was measured on the compute stream's queue.  Hence:

  * the plan's streams are created AND first used (one tiny kernel each,
    the default stream first) before RCCL's init, in ORDER: the default
    (compute) stream, `copy`, `early`, `capture` take the four queues;
  * entry points also raise GPU_MAX_HW_QUEUES to 8 (`reserve_hw_queues`,
    before the first HIP call), so RCCL's internal streams need not share
    either - measured: with 8 queues every stream of queue_map.py got its
    own.  (Under rocprofv3 the variable must be set on the command line:
    the profiler initialises the runtime before the program runs.)
  * a CU-masked stream also gets a queue of its own, but measured, its work
    did not run beside the compute queue's (the bench's H2D copy on one
    cost the whole 1.2 ms again), so none is used.

  * `copy`: the H2D batch prefetch (bench.py, the training feeder);
  * `early`: the early all-reduce.  GradientSynchronizer issues RCCL
    collectives stream-ordered (async_op=False), and ProcessGroupNCCL then
    runs them on the CURRENT stream rather than on its internal stream, so
    the early bucket runs on this stream's queue, the late bucket on the
    compute stream behind the torso backward it must follow anyway;
  * `capture`: the warm-up / capture stream of every `Learner.capture` (one
    stream for every capture: a new stream per capture would shift which
    queue every later stream gets).

`warmup_collective` then runs one collective at a known point, before the
first learner step.  Reference: /root/reference/experiment.py:497-512 (the
cluster setup this data-parallel path replaces); SURVEY.md §5.8.
"""

import collections
import os
import threading

ORDER = ('copy', 'early', 'capture')

StreamPlan = collections.namedtuple('StreamPlan', ORDER)

_PLANS = {}
_LOCK = threading.Lock()


# hardware queues per process (HIP's default is 4)
HW_QUEUES = 8


def reserve_hw_queues(environ=None):
  """GPU_MAX_HW_QUEUES=HW_QUEUES unless already set.  Must run before the
  process's first HIP call (the runtime reads it once).  With 4 queues the
  compute stream, the H2D copy stream, the early all-reduce stream and
  RCCL's internal streams cannot all have queues of their own: a stream
  takes its queue at its first use, and the early stream, first used by the
  warm-up collective after RCCL's init, measured on the compute stream's
  queue (profiles/r6_dp_queues.txt)."""
  env = os.environ if environ is None else environ
  env.setdefault('GPU_MAX_HW_QUEUES', str(HW_QUEUES))


def stream_plan(device, factory=None):
  """The device's StreamPlan, created on first use in ORDER.  `factory`
  (tests) replaces torch.cuda.Stream; it is called with the device."""
  import torch
  device = torch.device(device)
  with _LOCK:
    plan = _PLANS.get(device)
    if plan is None:
      make = factory or torch.cuda.Stream
      plan = StreamPlan(*[make(device) for _ in ORDER])
      if factory is None and device.type == 'cuda':
        # a stream takes its hardware queue at its FIRST use: use the
        # default stream, then the plan's streams, in order, now
        _touch(torch.cuda.current_stream(device), device)
        for s in plan:
          _touch(s, device)
        torch.cuda.synchronize(device)
      _PLANS[device] = plan
    return plan


def _touch(stream, device):
  import torch
  with torch.cuda.stream(stream):
    torch.zeros(1, device=device)


def reset_stream_plans():
  """Forget every plan (tests)."""
  with _LOCK:
    _PLANS.clear()


def warmup_collective(device, group=None):
  """One all-reduce of a one-element tensor, issued from the plan's early
  stream and waited for: the communicator exists (and works) before the
  first learner step.  No-op without a process group."""
  import torch
  import torch.distributed as dist
  if not dist.is_initialized():
    return
  device = torch.device(device)
  if device.type != 'cuda':
    t = torch.ones(1)
    dist.all_reduce(t, group=group)
    return
  plan = stream_plan(device)
  with torch.cuda.stream(plan.early):
    t = torch.ones(1, device=device)
    dist.all_reduce(t, group=group)
  plan.early.synchronize()
  torch.cuda.synchronize(device)
