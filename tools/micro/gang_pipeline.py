#!/usr/bin/env python3
"""The bf16 gang LSTM beside the conv torso.

The time-chunked learner (`--pipeline_chunks`, models/agent.py
_pipelined_core) runs chunk k's fused core (torso-FC / x-projection GEMMs
and the recurrence) on a side stream while the torso of chunk k+1 runs on
the main stream.  With SA_PIPELINE_GANG=1 (SA_MEASURE_KNOBS=1) the chunk's
recurrence is the resident 8-workgroup gang kernel (one launch per
direction and chunk) instead of per-step kernels, and the persistent conv
grids leave R CUs per XCD free (cf32_cu_reserve, bf16 and fp32 torso).

  python3 tools/micro/gang_pipeline.py [steps]

prints ms per captured bf16 learner step (B=32, T=100, 72x96) for:
the unchunked step (gang), and 2 chunks in the proportions 4:1 (a short last
chunk keeps the exposed recurrence short) with the gang or the per-step
kernels, at R = 0, 1, 2 (GANG_SPLIT overrides the proportions).  Run
under rocprofv3 --kernel-trace with GANG_ONLY=chunks,gang|step,R for one
variant's timeline.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
os.environ['SA_MEASURE_KNOBS'] = '1'

from scalable_agent_amd import flags as flags_lib  # noqa: E402
from scalable_agent_amd import ops  # noqa: E402
from scalable_agent_amd.envs.synthetic import make_synthetic_batch  # noqa
from scalable_agent_amd.learner import Learner, batch_to_device  # noqa: E402
from scalable_agent_amd.models import Agent  # noqa: E402


def run(chunks, gang, reserve, steps, batch, dev):
  C = ops.ext()
  os.environ['SA_PIPELINE_GANG'] = '1' if gang else '0'
  os.environ['SA_PIPELINE_SPLIT'] = os.environ.get('GANG_SPLIT', '4,1')
  prev = C.cf32_cu_reserve(reserve)
  try:
    f = flags_lib.default_flags(batch_size=32, unroll_length=100,
                                torso='deep', dtype='bf16')
    agent = Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=1,
                  backend='hip', compute_dtype=torch.bfloat16,
                  pipeline_chunks=chunks)
    lrn = Learner(agent, f, dev)
    lrn.capture(batch)
    for _ in range(3):
      lrn.graph_step()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(steps):
      lrn.graph_step()
    torch.cuda.synchronize()
    ms = 1e3 * (time.time() - t0) / steps
    health = lrn.health()
    del lrn, agent
    torch.cuda.empty_cache()
    return ms, health
  finally:
    C.cf32_cu_reserve(prev)


def main():
  steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(dev)
  ops.load()
  batch = batch_to_device(make_synthetic_batch(32, 100, (72, 96, 3), 9,
                                               seed=3), dev)
  variants = [(1, True, 0)] + [(2, g, r) for r in (0, 1, 2)
                               for g in (True, False)]
  only = os.environ.get('GANG_ONLY')
  if only:
    c, g, r = only.split(',')
    variants = [(int(c), g == 'gang', int(r))]
  for chunks, gang, reserve in variants:
    ms, health = run(chunks, gang, reserve, steps, batch, dev)
    print('chunks %d  %-8s  reserve %d/XCD  %.3f ms/step  %s' % (
        chunks, 'gang' if gang else 'per-step', reserve, ms, health),
          flush=True)


if __name__ == '__main__':
  main()
