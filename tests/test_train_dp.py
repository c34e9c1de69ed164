"""Data-parallel `experiment.train` end to end on CPU: two learner processes
under `torch.distributed.run` (gloo), each with its own actors and its own
trajectory queue, gradients summed by an all-reduce every step (SURVEY §2.4
C10; the reference has one learner, experiment.py:497-512).

Checks: both ranks finish; the frame counter advances by
world * B * T * repeats per step; rank 0 alone writes checkpoints; the
replica-consistency probe passes every step; the ranks trained on
different data (their own actors: different first-step losses); a restart
resumes every rank from rank 0's checkpoint.
"""

import os
import re
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ['--level_name=synthetic', '--unroll_length=5', '--device=cpu',
        '--dtype=fp32', '--torso=shallow', '--synthetic_episode_length=6',
        '--height=24', '--width=32', '--num_actors=2', '--batch_size=2',
        '--num_learners=2', '--consistency_check_steps=1',
        '--save_summaries_secs=0']
LINE = re.compile(r'rank (\d)/2: (\d+) learner steps, (\d+) env frames \(all ranks\), '
                  r'(\d+) episodes .*?, (\d+) replica-consistency checks passed, '
                  r'first loss (\S+)')


def _port():
  s = socket.socket()
  s.bind(('127.0.0.1', 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _torchrun(logdir, frames, timeout=300):
  env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS='1')
  env.pop('WORLD_SIZE', None)
  cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
         '--nproc-per-node=2', '--master-addr=127.0.0.1',
         '--master-port=%d' % _port(), os.path.join(ROOT, 'experiment.py')]
  cmd += ARGS + ['--logdir=' + logdir, '--total_environment_frames=%d' % frames]
  return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout,
                        env=env)


def test_train_two_learners_gloo(tmp_path):
  logdir = str(tmp_path / 'dp')
  per_step = 2 * 2 * 5 * 4  # world * B * T * repeats
  r = _torchrun(logdir, 6 * per_step)
  out = r.stdout + r.stderr
  assert r.returncode == 0, out[-4000:]
  ranks = {int(m.group(1)): m.groups()[1:] for m in LINE.finditer(out)}
  assert sorted(ranks) == [0, 1], out[-4000:]
  for rk, (steps, frames, episodes, checks, loss) in ranks.items():
    steps, frames, checks = int(steps), int(frames), int(checks)
    assert steps == 6 and frames == steps * per_step, (rk, steps, frames)
    assert checks == steps, (rk, checks)
    assert int(episodes) > 0, rk  # this rank's own actors produced episodes
  assert ranks[0][4] != ranks[1][4], 'ranks trained on the same data'
  # rank 0 checkpoints into logdir; other ranks never write checkpoints
  assert os.path.exists(os.path.join(logdir, 'checkpoint'))
  assert not os.path.exists(os.path.join(logdir, 'rank1', 'checkpoint'))
  # restart: every rank restores rank 0's checkpoint and continues
  r = _torchrun(logdir, 8 * per_step)
  out = r.stdout + r.stderr
  assert r.returncode == 0, out[-4000:]
  assert out.count('Restored checkpoint at %d frames' % (6 * per_step)) == 2
  ranks = {int(m.group(1)): m.groups()[1:] for m in LINE.finditer(out)}
  assert all(int(v[0]) == 2 and int(v[1]) == 8 * per_step
             for v in ranks.values()), ranks


import pytest  # noqa: E402


@pytest.mark.gpu
def test_train_two_learners_one_card_gloo(tmp_path):
  """The same on the GPU box: two learner ranks share the one card
  (SA_DIST_BACKEND=gloo rehearses the collective path; RCCL needs one GPU
  per rank), each with its actor-group process, trajectory queue, H2D
  feeder and captured learner graphs (HIP backend, exact-fp32 kernels)."""
  logdir = str(tmp_path / 'dpgpu')
  per_step = 2 * 2 * 5 * 4
  env_extra = {'SA_DIST_BACKEND': 'gloo'}
  os.environ.update(env_extra)
  try:
    global ARGS
    saved = ARGS
    ARGS = [a.replace('--device=cpu', '--device=cuda') for a in ARGS] + [
        '--backend=hip', '--torso=deep', '--height=72', '--width=96']
    r = _torchrun(logdir, 4 * per_step, timeout=600)
  finally:
    ARGS = saved
    for k in env_extra:
      os.environ.pop(k, None)
  out = r.stdout + r.stderr
  assert r.returncode == 0, out[-4000:]
  ranks = {int(m.group(1)): m.groups()[1:] for m in LINE.finditer(out)}
  assert sorted(ranks) == [0, 1], out[-4000:]
  for rk, (steps, frames, episodes, checks, loss) in ranks.items():
    assert int(steps) == 4 and int(frames) == 4 * per_step, (rk, steps, frames)
    assert int(checks) == 4, (rk, checks)
  assert ranks[0][4] != ranks[1][4]
  assert os.path.exists(os.path.join(logdir, 'checkpoint'))
