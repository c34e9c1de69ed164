#!/usr/bin/env python3
"""Learning evidence on the learnable synthetic levels (envs/synthetic.py).

Runs `experiment.train` in-process on 'synthetic_cue' (reactive: act with the
index of the bright band in the current frame) or 'synthetic_memory' (the
band is shown only on the first frame of an episode) and reports the mean
episode return per window of episodes, against the random-policy return
(episode_length / num_actions).  Usage:
  python tools/learning_curve.py [--level synthetic_cue] [--backend hip|torch]
      [--frames 400000] [--dtype fp32|bf16] [--out file.json]
"""
import argparse
import json
import logging
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from scalable_agent_amd import experiment  # noqa: E402
from scalable_agent_amd import flags as flags_lib  # noqa: E402


def run(level, backend, frames, dtype, torso='shallow', episode_length=20,
        num_actors=16, batch_size=8, unroll_length=20, height=36, width=48,
        learning_rate=0.0006, seed=1, logdir=None, log_every_frames=10 ** 9,
        entropy_cost=0.003, grad_scale=1.0):
  logdir = logdir or tempfile.mkdtemp(prefix='sa_learn_')
  fl = flags_lib.default_flags(
      level_name=level, env='synthetic', backend=backend, dtype=dtype,
      torso=torso, total_environment_frames=frames, num_actors=num_actors,
      batch_size=batch_size, unroll_length=unroll_length, height=height,
      width=width, synthetic_episode_length=episode_length,
      num_action_repeats=1, learning_rate=learning_rate, seed=seed,
      entropy_cost=entropy_cost, grad_scale=grad_scale, logdir=logdir,
      save_summaries_secs=0,
      save_checkpoint_secs=1e9, log_every_frames=log_every_frames)
  t0 = time.time()
  experiment.train(fl)
  wall = time.time() - t0
  returns = []
  with open(os.path.join(logdir, 'summaries.jsonl')) as f:
    for line in f:
      rec = json.loads(line)
      for k, v in rec.get('values', rec).items():
        if k.endswith('/episode_return'):
          returns.append((rec['step'], v))
  returns.sort()
  n = len(returns)
  win = max(1, n // 10)
  curve = [(returns[min(n - 1, i + win - 1)][0],
            sum(r for _, r in returns[i:i + win]) / len(returns[i:i + win]))
           for i in range(0, n, win)]
  return {'level': level, 'backend': backend, 'dtype': dtype, 'torso': torso,
          'frames': frames, 'episodes': n, 'wall_s': round(wall, 1),
          'random_return': episode_length / 9.0,
          'perfect_return': float(episode_length),
          'first_window_mean': curve[0][1] if curve else None,
          'last_window_mean': curve[-1][1] if curve else None,
          'curve': curve}


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--level', default='synthetic_cue')
  ap.add_argument('--backend', default='hip')
  ap.add_argument('--frames', type=int, default=400000)
  ap.add_argument('--dtype', default='fp32')
  ap.add_argument('--torso', default='shallow')
  ap.add_argument('--out', default='')
  # the headline configuration: --height 72 --width 96 --batch_size 32
  # --unroll_length 100 --num_actors 48 (README.md:37-41 of the reference)
  ap.add_argument('--height', type=int, default=36)
  ap.add_argument('--width', type=int, default=48)
  ap.add_argument('--batch_size', type=int, default=8)
  ap.add_argument('--unroll_length', type=int, default=20)
  ap.add_argument('--num_actors', type=int, default=16)
  ap.add_argument('--episode_length', type=int, default=20)
  ap.add_argument('--learning_rate', type=float, default=0.0006)
  ap.add_argument('--log_every_frames', type=int, default=10 ** 9)
  ap.add_argument('--entropy_cost', type=float, default=0.003)
  # data-parallel semantics on one GPU: batch N*B with grad_scale 1 (N
  # learners, --grad_reduce=sum) or 1/N (--grad_reduce=mean)
  ap.add_argument('--grad_scale', type=float, default=1.0)
  args = ap.parse_args()
  logging.basicConfig(level=logging.INFO, stream=sys.stdout)
  res = run(args.level, args.backend, args.frames, args.dtype, torso=args.torso,
            episode_length=args.episode_length, num_actors=args.num_actors,
            batch_size=args.batch_size, unroll_length=args.unroll_length,
            height=args.height, width=args.width,
            learning_rate=args.learning_rate,
            log_every_frames=args.log_every_frames,
            entropy_cost=args.entropy_cost, grad_scale=args.grad_scale)
  res.update(learning_rate=args.learning_rate, entropy_cost=args.entropy_cost,
             grad_scale=args.grad_scale,
             height=args.height, width=args.width, batch_size=args.batch_size,
             unroll_length=args.unroll_length, num_actors=args.num_actors)
  line = json.dumps(res)
  print(line, flush=True)
  if args.out:
    with open(args.out, 'a') as f:
      f.write(line + '\n')


if __name__ == '__main__':
  main()
