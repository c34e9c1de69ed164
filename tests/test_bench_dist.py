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


def _launcher_env():
  env = {k: v for k, v in os.environ.items()
         if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_PORT',
                      'SA_DIST_BACKEND')}
  env.update(PYTHONPATH=ROOT, OMP_NUM_THREADS='1')
  return env


def test_bench_self_launch_eight_ranks_cpu():
  """The driver's largest shape (8 ranks) through the self-launcher, on gloo:
  one JSON line, every rank's step time reported."""
  cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '8',
         '--steps', '2', '--warmup', '1', '--device', 'cpu',
         '--batch_size', '1', '--unroll_length', '3', '--torso', 'shallow',
         '--height', '16', '--width', '16', '--dtype', 'fp32']
  r = subprocess.run(cmd, capture_output=True, text=True, timeout=600,
                     env=_launcher_env())
  assert r.returncode == 0, r.stderr[-3000:]
  lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
  assert len(lines) == 1, r.stdout
  out = json.loads(lines[0])
  assert out['config']['parallelism'] == 'dp8'
  assert out['config']['global_batch'] == 8
  assert out['config']['dist']['world_size'] == 8
  assert len(out['config']['dist']['per_rank_ms_per_step']) == 8


def test_bench_launcher_sigterm_leaves_no_rank():
  """SIGTERM to the launcher (a driver timeout) kills every rank: none
  outlives it."""
  import signal
  import time
  import psutil
  cmd = _self_launch_cmd('--steps', '100000')
  p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       env=_launcher_env())
  try:
    me = psutil.Process(p.pid)
    deadline = time.time() + 120
    kids = []
    while time.time() < deadline:
      kids = [c for c in me.children(recursive=True)
              if 'bench.py' in ' '.join(c.cmdline())]
      if len(kids) >= 2:
        break
      time.sleep(0.2)
    assert len(kids) >= 2, 'ranks never started'
    time.sleep(3)  # let them get into torch / gloo setup
    p.send_signal(signal.SIGTERM)
    p.wait(timeout=60)
    assert p.returncode != 0
    gone, alive = psutil.wait_procs(kids, timeout=30)
    assert not alive, [a.pid for a in alive]
  finally:
    if p.poll() is None:
      p.kill()
      p.wait()


def test_bench_launcher_rejects_more_ranks_than_gpus(tmp_path):
  """--gpus 4 on a one-GPU node (fake KFD topology) fails at once with a
  clear message, before any rank starts."""
  import time
  topo = tmp_path / 'class/kfd/kfd/topology/nodes'
  (topo / '0').mkdir(parents=True)
  (topo / '0' / 'properties').write_text('simd_count 0\n')
  (topo / '1').mkdir()
  (topo / '1' / 'properties').write_text('simd_count 1024\nlocation_id 256\n')
  env = _launcher_env()
  env['SA_SYSFS_ROOT'] = str(tmp_path)
  for k in ('HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES',
            'ROCR_VISIBLE_DEVICES'):
    env.pop(k, None)
  t0 = time.time()
  r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'),
                      '--gpus', '4', '--steps', '2'],
                     capture_output=True, text=True, timeout=60, env=env)
  assert r.returncode == 2
  assert 'only 1 GPU(s) are visible' in r.stderr
  assert not r.stdout.strip()
  assert time.time() - t0 < 20
