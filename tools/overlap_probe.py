#!/usr/bin/env python3
"""Does side-stream work overlap the persistent-grid conv-torso backward?

With world > 1 the learner replays its step as two graphs (learner.py
graph_step): forward + the backward down to the torso features, then the
conv-torso backward; the early gradient all-reduce (parallel/dist.py
GradientSynchronizer.begin_early) is launched between the
two replays on RCCL's own stream.  Whether that collective really runs UNDER
the torso backward depends on whether the persistent conv grids leave it any
CU slots.  This probe measures it on one GPU with stand-ins for the RCCL
kernel: device copies (6 MB, 24 MB, 384 MB), one 1.5M-element elementwise
kernel and a chain of 50 of them (a collective is many dependent kernels),
launched on a side stream between the replays.

For each job it reports, from device events:
  alone_ms    the job on an idle GPU
  lat_ms      launch -> completion when launched next to the torso backward
  g1_ms       the forward + late-backward replay before the job's launch
  g2_ms       the torso-backward replay with / without the job
  step_ms     the whole step (graphs + optimizer) with / without the job
A job that overlaps finishes after ~alone_ms; a starved one only when the
torso backward ends (lat_ms ~ g2_ms).

  python tools/overlap_probe.py [--steps 20] [--out file.jsonl]
(SA_PROBE_HIGH_PRIO=1 adds a high-priority side stream.)
"""
import argparse
import json
import os
import sys

ap = argparse.ArgumentParser()
ap.add_argument('--steps', type=int, default=20)
ap.add_argument('--out', default='')
args = ap.parse_args()

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scalable_agent_amd import flags as flags_lib  # noqa: E402
from scalable_agent_amd.envs.synthetic import make_synthetic_batch  # noqa: E402
from scalable_agent_amd.learner import Learner  # noqa: E402
from scalable_agent_amd.models import Agent  # noqa: E402


def main():
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(dev)
  fl = flags_lib.default_flags(batch_size=32, unroll_length=100, torso='deep',
                               dtype='fp32', height=72, width=96)
  agent = Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=fl.seed,
                backend='hip', compute_dtype=torch.float32)
  learner = Learner(agent, fl, dev, world_size=1)
  if learner._torso_offset() is None:
    raise SystemExit('torso parameters are not the flat buffer tail')
  learner._split = True  # two graphs, as with world > 1
  hb = make_synthetic_batch(32, 100, (72, 96, 3), 9, seed=5, pin_memory=False)
  learner.capture(hb)
  g1, g2 = learner._graph
  main_s = torch.cuda.current_stream(dev)

  n = 6 * (1 << 20) // 4
  src6, dst6 = torch.randn(n, device=dev), torch.empty(n, device=dev)
  src24, dst24 = torch.randn(4 * n, device=dev), torch.empty(4 * n, device=dev)
  x = torch.randn(n, device=dev)
  big_s = torch.randn(64 * n, device=dev)
  big_d = torch.empty_like(big_s)

  def chain():
    for _ in range(50):
      x.mul_(0.999)

  # a long collective is many dependent kernels (RCCL: one per bucket /
  # ring phase); `chain_50` needs a CU slot 50 times over the backward
  jobs = {
      'copy_6MB': lambda: dst6.copy_(src6),
      'copy_24MB': lambda: dst24.copy_(src24),
      'copy_384MB': lambda: big_d.copy_(big_s),
      'elementwise_1.5M': lambda: x.mul_(0.999),
      'chain_50_elementwise': chain,
  }
  streams = {'normal': torch.cuda.Stream(dev)}
  if os.environ.get('SA_PROBE_HIGH_PRIO') == '1':
    # measured: a high-priority side stream slows the whole step by ~9 ms
    streams['high_prio'] = torch.cuda.Stream(dev, priority=-1)

  def ev():
    return torch.cuda.Event(enable_timing=True)

  def step(job=None, side=None):
    e = [ev() for _ in range(6)]
    e[0].record(main_s)
    g1.replay()
    if job is not None:
      side.wait_stream(main_s)
      with torch.cuda.stream(side):
        e[4].record(side)
        job()
        e[5].record(side)
    e[1].record(main_s)
    g2.replay()
    e[2].record(main_s)
    if job is not None:
      main_s.wait_stream(side)
    learner._apply()
    e[3].record(main_s)
    return e

  def run(job=None, side=None):
    for _ in range(3):
      step(job, side)
    torch.cuda.synchronize()
    evs = [step(job, side) for _ in range(args.steps)]
    torch.cuda.synchronize()
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    r = {'step_ms': med([a[0].elapsed_time(a[3]) for a in evs]),
         'g1_ms': med([a[0].elapsed_time(a[1]) for a in evs]),
         'g2_ms': med([a[1].elapsed_time(a[2]) for a in evs])}
    if job is not None:
      r['lat_ms'] = med([a[4].elapsed_time(a[5]) for a in evs])
      # completion relative to the torso-backward start
      r['done_after_g2_start_ms'] = med([a[1].elapsed_time(a[5]) for a in evs])
    return r

  out = {'base': run()}
  for name, job in jobs.items():
    s = streams['normal']
    for _ in range(3):
      with torch.cuda.stream(s):
        job()
    torch.cuda.synchronize()
    a0, a1 = ev(), ev()
    with torch.cuda.stream(s):
      a0.record(s)
      for _ in range(10):
        job()
      a1.record(s)
    torch.cuda.synchronize()
    res = {'alone_ms': a0.elapsed_time(a1) / 10}
    for sn, st in streams.items():
      res[sn] = run(job, st)
    out[name] = res
    print(name, json.dumps(res), flush=True)
  print(json.dumps(out), flush=True)
  if args.out:
    with open(args.out, 'a') as f:
      f.write(json.dumps(out) + '\n')


if __name__ == '__main__':
  main()
