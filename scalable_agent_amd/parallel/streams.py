"""The learner process's HIP streams, created once, in a fixed order.

HIP backs streams with GPU_MAX_HW_QUEUES (4) hardware queues per device
and hands a new stream the least-used queue, so WHICH queue a stream lands
on depends on how many streams exist when it is created.  Two streams on one
hardware queue are serialised by the queue's barrier packets: the 67 MB H2D
batch prefetch on the compute stream's queue costs its full 1.2 ms per step
(bench.py, profiles/experiments.md round 3), and a collective behind the
compute queue would not overlap the torso backward at all.
Every stream of the learner path therefore comes from this plan:

  * RCCL's communicator stream: `init_distributed` passes `device_id`, so
    ProcessGroupNCCL builds the communicator and takes its stream at init,
    before any stream below (`warmup_collective` then runs one collective at
    that known point and checks it returns);
  * `copy`: the H2D batch prefetch (bench.py, the training feeder), on a
    hardware queue of its own;
  * `capture`: the warm-up / capture stream of every `Learner.capture`
    (one stream reused by every capture, not a new one each time);
  * `early`: the data-parallel early all-reduce, on a hardware queue of its
    own.  GradientSynchronizer issues RCCL collectives stream-ordered
    (async_op=False), and ProcessGroupNCCL then runs them on the CURRENT
    stream rather than on its internal pool stream, so the early bucket's
    kernels run on this queue (the trace shows it) and the late bucket's on
    the compute stream, behind the torso backward they must follow anyway.

A plain new stream gets the least-used of HIP's queues; measured on one
MI355X (profiles/r6_dp_queues.txt) the third pool stream of the plan landed
on the compute stream's queue, where the early all-reduce would have waited
for the whole torso backward.  `_C.own_queue_stream` creates its stream with
a full CU mask, which always makes a new queue.

The compute stream is the device's default stream (graphs replay there).
The queue each of them runs on is measured with
`tools/micro/dp_queues.py` under rocprofv3 (profiles/r6_dp_queues.txt).
Reference: /root/reference/experiment.py:497-512 (the cluster setup this
data-parallel path replaces); SURVEY.md §5.8.
"""

import collections
import threading

ORDER = ('copy', 'capture', 'early')

StreamPlan = collections.namedtuple('StreamPlan', ORDER)

_PLANS = {}
_LOCK = threading.Lock()


# streams that get a hardware queue of their own (the rest share HIP's pool)
OWN_QUEUE = ('copy', 'early')


def _own_queue_stream(device):
  """A stream on a new hardware queue (_C.own_queue_stream: a full CU mask
  makes HIP create a queue instead of sharing the least-used one).  Falls
  back to a pool stream when the extension is not built (CPU tooling)."""
  import torch
  try:
    from ..ops import _ext
    C = _ext.load()
  except Exception:  # pylint: disable=broad-except
    return torch.cuda.Stream(device)
  handle = C.own_queue_stream(device.index if device.index is not None
                              else torch.cuda.current_device())
  return torch.cuda.ExternalStream(handle, device=device)


def stream_plan(device, factory=None):
  """The device's StreamPlan, created on first use in ORDER.  `factory`
  (tests) replaces the stream constructors; it is called with the device."""
  import torch
  device = torch.device(device)
  with _LOCK:
    plan = _PLANS.get(device)
    if plan is None:
      made = []
      for name in ORDER:
        if factory is not None:
          made.append(factory(device))
        elif name in OWN_QUEUE:
          made.append(_own_queue_stream(device))
        else:
          made.append(torch.cuda.Stream(device))
      plan = StreamPlan(*made)
      _PLANS[device] = plan
    return plan


def reset_stream_plans():
  """Forget every plan (tests)."""
  with _LOCK:
    _PLANS.clear()


def warmup_collective(device, group=None):
  """One all-reduce of a one-element tensor, issued from the plan's early
  stream and waited for: the communicator and its stream exist (and work)
  before the first learner step.  No-op without a process group."""
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
