#!/usr/bin/env python3
"""Actor-inference throughput: N actor threads issuing batch-1 agent steps
through the dynamic batcher (reference experiment.py:534-546), with the
pinned-slab staged server (inference.StagedBatchedInfer) vs the generic
batch_fn runner (per-array H2D/D2H copies, torch heads + multinomial).

usage: python tools/inference_bench.py [--actors 64] [--calls 200]
           [--torso deep] [--mode all|graph,staged,generic] [--switch S]
Prints one JSON line per mode: agent steps/s, mean batch, latency p50/p99.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scalable_agent_amd import inference  # noqa: E402
from scalable_agent_amd.models import Agent  # noqa: E402


def run(mode, args):
  torch.manual_seed(0)
  agent = Agent(9, torso=args.torso, backend='hip',
                compute_dtype=torch.bfloat16)
  model = inference.InferenceModel(agent, 'cuda', True, seed=1)
  if mode == 'generic':
    from scalable_agent_amd.ops.heads import PhiloxStream
    if isinstance(model._gen, PhiloxStream):  # torch sampler path
      model._gen = torch.Generator(device='cuda').manual_seed(1)
  srv = inference.make_batched_infer(model, 1, args.max_batch, args.timeout_ms,
                                     staged=(mode != 'generic'),
                                     graphs=(mode == 'graph'))
  lat = [[] for _ in range(args.actors)]
  start = threading.Barrier(args.actors + 1)
  warm = threading.Barrier(args.actors + 1)

  def actor(i):
    rng = np.random.RandomState(i)
    frame = rng.randint(0, 255, (1, 72, 96, 3)).astype(np.uint8)
    c = np.zeros((1, 256), np.float32)
    h = np.zeros((1, 256), np.float32)
    a = np.zeros(1, np.int64)
    for k in range(args.warmup):  # bucket graphs captured here, untimed
      srv(a, np.zeros(1, np.float32), np.array([False]), frame,
          np.zeros((1, 16), np.int64), np.zeros(1, np.int64), c, h)
    warm.wait()
    start.wait()
    for k in range(args.calls):
      t0 = time.perf_counter()
      out = srv(a, np.zeros(1, np.float32), np.array([k == 0]), frame,
                np.zeros((1, 16), np.int64), np.zeros(1, np.int64), c, h)
      lat[i].append(time.perf_counter() - t0)
      a, c, h = out[0].astype(np.int64), out[3], out[4]

  ts = [threading.Thread(target=actor, args=(i,)) for i in range(args.actors)]
  for t in ts:
    t.start()
  warm.wait()
  st0 = srv.stats()
  start.wait()
  t0 = time.perf_counter()
  for t in ts:
    t.join()
  dt = time.perf_counter() - t0
  st = srv.stats()
  srv.close()
  srv.join(10)
  lats = np.concatenate([np.asarray(x) for x in lat]) * 1e3
  return {'mode': mode, 'actors': args.actors, 'calls': args.calls,
          'torso': args.torso,
          'agent_steps_per_s': round(args.actors * args.calls / dt, 1),
          'mean_batch': round((st['requests'] - st0['requests']) /
                              max(1, st['batches'] - st0['batches']), 2),
          'switch_interval_s': sys.getswitchinterval(),
          'server_busy_frac': round((st.get('busy_s', 0) - st0.get('busy_s', 0))
                                    / dt, 3),
          'latency_ms_p50': round(float(np.percentile(lats, 50)), 3),
          'latency_ms_p99': round(float(np.percentile(lats, 99)), 3)}


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--actors', type=int, default=64)
  ap.add_argument('--calls', type=int, default=200)
  ap.add_argument('--torso', default='deep')
  ap.add_argument('--max_batch', type=int, default=1024)
  ap.add_argument('--timeout_ms', type=int, default=100)
  ap.add_argument('--mode', default='all')
  ap.add_argument('--warmup', type=int, default=20)
  ap.add_argument('--switch', type=float, default=0.0,
                  help='sys.setswitchinterval (0 = keep the default)')
  args = ap.parse_args()
  if args.switch > 0:
    sys.setswitchinterval(args.switch)
  modes = (['graph', 'staged', 'generic'] if args.mode == 'all' else
           args.mode.split(','))
  for m in modes:
    print(json.dumps(run(m, args)), flush=True)


if __name__ == '__main__':
  main()
