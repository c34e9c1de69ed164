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
  assert b['health'] == {'skipped_updates': 0, 'lstm_timeouts': 0}
  # the RMSProp update built from them agrees too
  assert torch.allclose(a['params'], b['params'], rtol=0, atol=atol)
