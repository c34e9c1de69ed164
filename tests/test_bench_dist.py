"""bench.py's multi-rank contract on CPU: torch.distributed.run with 2 gloo
ranks at 127.0.0.1, one JSON line from rank 0 with the whole-job value."""

import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
  s = socket.socket()
  s.bind(('127.0.0.1', 0))
  p = s.getsockname()[1]
  s.close()
  return p


def test_bench_two_ranks_cpu():
  cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
         '--nproc-per-node', '2', '--master-addr', '127.0.0.1',
         '--master-port', str(_port()), os.path.join(ROOT, 'bench.py'),
         '--gpus', '2', '--steps', '2', '--warmup', '1', '--device', 'cpu',
         '--batch_size', '2', '--unroll_length', '4', '--torso', 'shallow',
         '--height', '24', '--width', '32', '--dtype', 'fp32']
  r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                     env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS='2'))
  assert r.returncode == 0, r.stderr[-3000:]
  lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
  assert len(lines) == 1, r.stdout
  out = json.loads(lines[0])
  assert out['steps'] == 2 and out['warmup'] == 1
  assert out['config']['parallelism'] == 'dp2'
  assert out['config']['global_batch'] == 4
  assert out['value'] > 0 and out['higher_is_better'] is True
  frames_per_step = 2 * 2 * 4 * 4  # world x B x T x repeats
  assert abs(out['value'] - frames_per_step / (out['ms_per_step'] / 1e3)) \
      <= 0.02 * out['value']


def _self_launch_cmd(*extra):
  return [sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2',
          '--steps', '2', '--warmup', '1', '--device', 'cpu',
          '--batch_size', '2', '--unroll_length', '4', '--torso', 'shallow',
          '--height', '24', '--width', '32', '--dtype', 'fp32'] + list(extra)


def test_bench_self_launch_two_ranks_cpu():
  """`python bench.py --gpus 2` without torchrun: the launcher process starts
  the two ranks itself and relays exactly one JSON line (the driver's plain
  command form)."""
  env = {k: v for k, v in os.environ.items()
         if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_PORT')}
  env.update(PYTHONPATH=ROOT, OMP_NUM_THREADS='2')
  r = subprocess.run(_self_launch_cmd(), capture_output=True, text=True,
                     timeout=300, env=env)
  assert r.returncode == 0, r.stderr[-3000:]
  lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
  assert len(lines) == 1, r.stdout
  out = json.loads(lines[0])
  assert out['config']['parallelism'] == 'dp2'
  assert out['config']['dist']['world_size'] == 2
  assert out['config']['dist']['backend'] == 'gloo'
  assert len(out['config']['dist']['per_rank_ms_per_step']) == 2
  assert 'allreduce_ms_standalone' in out['config']['dist']


def test_bench_self_launch_propagates_rank_failure():
  env = {k: v for k, v in os.environ.items()
         if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_PORT')}
  env.update(PYTHONPATH=ROOT, OMP_NUM_THREADS='2')
  r = subprocess.run(_self_launch_cmd('--backend', 'no-such-backend'),
                     capture_output=True, text=True, timeout=300, env=env)
  assert r.returncode != 0
  assert not [l for l in r.stdout.splitlines() if l.startswith('{')]
