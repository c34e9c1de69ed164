#!/usr/bin/env python3
"""Data-parallel equivalence check on ONE card (tests/test_dp_gpu.py).

N ranks (torch.distributed.run, backend from SA_DIST_BACKEND, gloo on one
card) each take their B/N columns of the same synthetic batch, run one HIP
learner step (captured graph; --dtype bf16 uses the gang LSTM) with the
flat-gradient all-reduce (--grad_reduce=sum), and rank 0 writes the
parameters; with WORLD_SIZE=1 the same script runs the whole batch on one
learner.  Under the reference's sum losses both must give the same update.
usage: dp_check.py --out params.pt [--dtype fp32|bf16] [--batch 4]

--fault_rank R: rank R gets an injected hand-off timeout on the first step
only: --fault_kind conv (fp32: the fused Winograd backward) or lstm (bf16:
the gang LSTM).  Every rank writes `<out>.<rank>` with whether each of two
steps applied, the replicas' consistency after each, and its health
counters: the collective step guard must make every rank skip step 1 and
apply step 2.  With --graph 1 each step is captured (the injected fault is
part of the captured launches) and replayed through Learner.graph_step: the
split backward graphs, the early all-reduce after the host has seen the
first graph end, the sentinel poison before the late bucket.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from scalable_agent_amd import flags as flags_lib  # noqa: E402
from scalable_agent_amd import parallel  # noqa: E402
from scalable_agent_amd.envs.synthetic import make_synthetic_batch  # noqa
from scalable_agent_amd.learner import Learner, _map_tensors  # noqa: E402
from scalable_agent_amd.models import Agent  # noqa: E402


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--out', required=True)
  ap.add_argument('--dtype', default='fp32')
  ap.add_argument('--batch', type=int, default=4)
  ap.add_argument('--unroll', type=int, default=6)
  ap.add_argument('--graph', type=int, default=1)
  ap.add_argument('--fault_rank', type=int, default=-1)
  ap.add_argument('--fault_kind', default='conv', choices=('conv', 'lstm'))
  args = ap.parse_args()
  rank, world, local = parallel.init_distributed()
  device = torch.device('cuda', local % torch.cuda.device_count())
  torch.cuda.set_device(device)
  B = args.batch // world
  flags = flags_lib.default_flags(batch_size=B, unroll_length=args.unroll,
                                  torso='deep', dtype=args.dtype,
                                  grad_reduce='sum')
  cdt = torch.bfloat16 if args.dtype == 'bf16' else torch.float32
  agent = Agent(9, torso='deep', seed=11, backend='hip', compute_dtype=cdt)
  learner = Learner(agent, flags, device, world_size=world)
  parallel.broadcast_params(learner.flat.params)
  full = make_synthetic_batch(args.batch, args.unroll, (72, 96, 3), 9, seed=5)

  def cols(t):
    if t.dim() >= 2 and t.shape[0] == args.unroll + 1:  # time-major [T+1, B]
      return t[:, rank * B:(rank + 1) * B].contiguous()
    return t[rank * B:(rank + 1) * B].contiguous()  # [B, ...] (agent state)

  mine = _map_tensors(full, lambda t: cols(t).to(device))
  if args.fault_rank >= 0:
    from scalable_agent_amd.ops import _ext
    C = _ext.ext()
    fault = C.cf32_wino_fault if args.fault_kind == 'conv' else C.lstm_gang_fault
    rec = {'world': world, 'rank': rank, 'split': learner._split}
    for step in (1, 2):
      p0 = learner.flat.params.clone()
      prev = fault(1 if (step == 1 and rank == args.fault_rank) else 0)
      try:
        if args.graph:
          learner.capture(mine)
          learner.graph_step()
        else:
          learner.step(mine)
        torch.cuda.synchronize()
      finally:
        fault(prev)
      rec['applied%d' % step] = not torch.equal(learner.flat.params, p0)
      rec['consistent%d' % step] = parallel.param_checksum_consistent(
          learner.flat.params)
      rec['health%d' % step] = learner.health()
    torch.save(rec, '%s.%d' % (args.out, rank))
    parallel.cleanup()
    return
  if args.graph:
    learner.capture(mine)
    learner.graph_step()
  else:
    learner.step(mine)
  torch.cuda.synchronize()
  if rank == 0:
    torch.save({'params': learner.flat.params.cpu(),
                'grads': learner.flat.grads.cpu(), 'world': world,
                'health': learner.health()}, args.out)
  parallel.cleanup()


if __name__ == '__main__':
  main()
