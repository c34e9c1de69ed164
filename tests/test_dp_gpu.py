"""Data-parallel HIP learner on one card: 2 ranks (gloo over the GPU tensors,
the one-card stand-in for RCCL) x B/2 columns each must equal one learner
with the whole batch (reference losses are sums, --grad_reduce=sum), for the
exact-fp32 path and the bf16 path (captured graph + gang LSTM)."""

import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
  s = socket.socket()
  s.bind(('127.0.0.1', 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _run(cmd, env):
  r = subprocess.run(cmd, capture_output=True, text=True, timeout=240,
                     env=dict(os.environ, PYTHONPATH=ROOT, **env))
  assert r.returncode == 0, r.stderr[-4000:]


@pytest.mark.parametrize('dtype,tol,atol', [('fp32', 2e-5, 1e-6), ('bf16', 2e-2, 5e-4)])
def test_two_ranks_match_one_rank_with_the_whole_batch(cuda, tmp_path, dtype, tol,
                                                       atol):
  script = os.path.join(ROOT, 'tools', 'dp_check.py')
  one, two = str(tmp_path / 'one.pt'), str(tmp_path / 'two.pt')
  env1 = {k: v for k, v in os.environ.items()
          if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
  r = subprocess.run([sys.executable, script, '--out', one, '--dtype', dtype],
                     capture_output=True, text=True, timeout=240,
                     env=dict(env1, PYTHONPATH=ROOT))
  assert r.returncode == 0, r.stderr[-4000:]
  _run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
        '--nproc-per-node', '2', '--master-addr', '127.0.0.1',
        '--master-port', str(_port()), script, '--out', two, '--dtype', dtype],
       {'SA_DIST_BACKEND': 'gloo', 'OMP_NUM_THREADS': '2'})
  a, b = torch.load(one, weights_only=True), torch.load(two, weights_only=True)
  assert a['world'] == 1 and b['world'] == 2
  g1, g2 = a['grads'].double(), b['grads'].double()
  assert ((g2 - g1).norm() / g1.norm()).item() <= tol
  assert b['health'] == {'skipped_updates': 0, 'lstm_timeouts': 0,
                                'conv_timeouts': 0}
  # the RMSProp update built from them agrees too
  assert torch.allclose(a['params'], b['params'], rtol=0, atol=atol)


@pytest.mark.parametrize('kind,dtype,graph', [('conv', 'fp32', 0),
                                              ('conv', 'fp32', 1),
                                              ('lstm', 'bf16', 1)])
def test_one_rank_fault_skips_the_step_on_every_rank(cuda, tmp_path, kind,
                                                     dtype, graph):
  """DP step guard: rank 1's fused Winograd backward (conv) or gang LSTM
  (lstm) times out (injected) on step 1 only.  Its error words poison the
  reduced gradient, so BOTH ranks skip step 1 (replicas stay identical,
  skipped_updates == 1 on each, the timeout counted on rank 1 only) and
  both apply step 2 - eager, and through the captured split-backward graphs
  with the host-ordered early all-reduce (Learner.graph_step)."""
  script = os.path.join(ROOT, 'tools', 'dp_check.py')
  out = str(tmp_path / 'fault.pt')
  _run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
        '--nproc-per-node', '2', '--master-addr', '127.0.0.1',
        '--master-port', str(_port()), script, '--out', out, '--dtype', dtype,
        '--graph', str(graph), '--fault_rank', '1', '--fault_kind', kind,
        '--unroll', '8'],
       {'SA_DIST_BACKEND': 'gloo', 'OMP_NUM_THREADS': '2'})
  recs = [torch.load('%s.%d' % (out, r), weights_only=True) for r in (0, 1)]
  for r, rec in enumerate(recs):
    assert rec['world'] == 2 and rec['rank'] == r
    assert rec['split'] is True  # the two-phase (split) backward ran
    assert rec['applied1'] is False, 'rank %d applied the poisoned step' % r
    assert rec['consistent1'] and rec['consistent2']
    assert rec['applied2'] is True
    assert rec['health1']['skipped_updates'] == 1
    assert rec['health2']['skipped_updates'] == 1
    mine = 1 if r == 1 else 0
    assert rec['health2']['conv_timeouts'] == (mine if kind == 'conv' else 0)
    assert rec['health2']['lstm_timeouts'] == (mine if kind == 'lstm' else 0)


@pytest.mark.gpu
def test_bench_two_ranks_one_card(cuda):
  """bench.py's multi-rank path on the GPU (the driver's N>1 launch shape,
  here two ranks sharing one card over gloo): captured split-backward graphs,
  the early all-reduce between their replays, fp32 and bf16 learners, one
  JSON line from rank 0 reporting both ranks."""
  import json
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  s = socket.socket()
  s.bind(('127.0.0.1', 0))
  port = s.getsockname()[1]
  s.close()
  cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
         '--nproc-per-node', '2', '--master-addr', '127.0.0.1',
         '--master-port', str(port), os.path.join(root, 'bench.py'),
         '--gpus', '2', '--steps', '3', '--warmup', '2', '--batch_size', '4',
         '--unroll_length', '10']
  env = dict(os.environ, PYTHONPATH=root, SA_DIST_BACKEND='gloo',
             OMP_NUM_THREADS='2')
  r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
  assert r.returncode == 0, r.stderr[-3000:]
  lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
  assert len(lines) == 1, r.stdout
  out = json.loads(lines[0])
  cfg = out['config']
  assert out['n_gpus'] == 2 and cfg['parallelism'] == 'dp2'
  assert cfg['dist']['world_size'] == 2 and cfg['dist']['backend'] == 'gloo'
  assert cfg['global_batch'] == 8 and cfg['hip_graph'] and cfg['loss_finite']
  assert cfg['torso_kernels'] == 'fp32' and cfg['bf16']['loss_finite']
  assert cfg['learner_health']['skipped_updates'] == 0
