"""End-to-end CPU runs of the experiment driver with the synthetic env (the
reference's Dockerfile smoke: short train + `--mode=test`), plus the
multi-process distributed mode (learner + actor processes on one node)."""

import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ['--level_name=synthetic', '--unroll_length=5', '--device=cpu',
          '--dtype=fp32', '--torso=shallow', '--synthetic_episode_length=6',
          '--height=24', '--width=32']


def _run(args, timeout=240):
  env = dict(os.environ, PYTHONPATH=ROOT)
  return subprocess.run([sys.executable, os.path.join(ROOT, 'experiment.py')]
                        + COMMON + args, capture_output=True, text=True,
                        timeout=timeout, env=env)


def test_train_then_test(tmp_path):
  logdir = str(tmp_path / 'run')
  r = _run(['--logdir=' + logdir, '--num_actors=3', '--batch_size=2',
            '--total_environment_frames=480', '--save_summaries_secs=0'])
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'Episode return' in r.stderr
  assert os.path.exists(os.path.join(logdir, 'checkpoint'))
  assert glob.glob(os.path.join(logdir, 'events.out.tfevents*'))
  # resume continues from the checkpoint's frame counter
  r = _run(['--logdir=' + logdir, '--num_actors=2', '--batch_size=2',
            '--total_environment_frames=560'])
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'Restored checkpoint at 480 frames' in r.stderr
  r = _run(['--logdir=' + logdir, '--mode=test', '--test_num_episodes=2'])
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'Mean episode return' in r.stderr


def test_distributed_actor_processes(tmp_path):
  logdir = str(tmp_path / 'dist')
  env = dict(os.environ, PYTHONPATH=ROOT)
  base = [sys.executable, os.path.join(ROOT, 'experiment.py')] + COMMON + [
      '--logdir=' + logdir, '--num_actors=2', '--batch_size=2']
  learner = subprocess.Popen(base + ['--job_name=learner', '--task=0',
                                     '--max_learner_steps=3'],
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                             text=True, env=env)
  actors = [subprocess.Popen(base + ['--job_name=actor', '--task=%d' % i],
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                             text=True, env=env) for i in range(2)]
  try:
    out, err = learner.communicate(timeout=240)
    assert learner.returncode == 0, err[-3000:]
    for a in actors:
      a.wait(timeout=60)
  finally:
    for p in [learner] + actors:
      if p.poll() is None:
        p.kill()
  assert os.path.exists(os.path.join(logdir, 'checkpoint'))


def test_train_doom_benchmark_sim(tmp_path):
  """`--level_name=doom_benchmark` through the IMPALA Doom adaptor (128x72
  frames, 9 actions) on the in-tree ViZDoom simulator backend."""
  env = dict(os.environ, PYTHONPATH=ROOT, SA_DOOM_BACKEND='sim')
  r = subprocess.run(
      [sys.executable, os.path.join(ROOT, 'experiment.py'),
       '--level_name=doom_benchmark', '--unroll_length=5', '--device=cpu',
       '--dtype=fp32', '--torso=shallow', '--num_actors=2', '--batch_size=2',
       '--total_environment_frames=400', '--logdir=' + str(tmp_path / 'd')],
      capture_output=True, text=True, timeout=240, env=env)
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'Level: doom_benchmark Episode return' in r.stderr or \
      os.path.exists(str(tmp_path / 'd' / 'checkpoint'))


def test_train_popart(tmp_path):
  logdir = str(tmp_path / 'popart')
  r = _run(['--logdir=' + logdir, '--num_actors=2', '--batch_size=2',
            '--total_environment_frames=240', '--popart=true',
            '--popart_beta=0.1'])
  assert r.returncode == 0, r.stderr[-3000:]
  import torch
  from scalable_agent_amd import checkpoint as ckpt
  sd = ckpt.load_state(ckpt.latest_checkpoint(logdir))
  assert 'popart' in sd and sd['popart']['mu'].shape == (1,)
  assert float(sd['popart']['mu'].abs().sum()) > 0


def test_tf_checkpoint_format_train_resume_test(tmp_path):
  """--checkpoint_format=tf writes the reference layout (model.ckpt-N
  .index/.data + a TF `checkpoint` index); training resumes from it and
  --mode=test evaluates it (reference experiment.py:608-616, 675-708)."""
  from scalable_agent_amd import tf_checkpoint
  logdir = str(tmp_path / 'tfrun')
  r = _run(['--logdir=' + logdir, '--num_actors=2', '--batch_size=2',
            '--total_environment_frames=240', '--checkpoint_format=tf',
            '--popart=true'])
  assert r.returncode == 0, r.stderr[-3000:]
  prefix = os.path.join(logdir, 'model.ckpt-240')
  assert os.path.exists(prefix + '.index')
  assert os.path.exists(prefix + '.data-00000-of-00001')
  assert not glob.glob(os.path.join(logdir, '*.pt'))
  text = open(os.path.join(logdir, 'checkpoint')).read()
  assert 'model_checkpoint_path: "model.ckpt-240"' in text
  t = tf_checkpoint.read_checkpoint(prefix)
  assert int(t['num_environment_frames']) == 240
  assert 'agent/baseline/linear/w/RMSProp' in t or any(
      k.endswith('/RMSProp') for k in t)
  assert 'popart/mu' in t
  r = _run(['--logdir=' + logdir, '--num_actors=2', '--batch_size=2',
            '--total_environment_frames=320', '--checkpoint_format=tf',
            '--popart=true'])
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'Restored checkpoint at 240 frames' in r.stderr
  assert os.path.exists(os.path.join(logdir, 'model.ckpt-320.index'))
  r = _run(['--logdir=' + logdir, '--mode=test', '--test_num_episodes=2'])
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'Mean episode return' in r.stderr


def test_tf_checkpoint_keeps_newest(tmp_path):
  import torch
  from scalable_agent_amd import checkpoint as ckpt
  from scalable_agent_amd import flags as flags_lib
  from scalable_agent_amd.learner import Learner
  from scalable_agent_amd.models import Agent
  flags = flags_lib.default_flags(batch_size=2, unroll_length=3)
  learner = Learner(Agent(9, torso='shallow', frame_shape=(24, 32, 3)), flags,
                    torch.device('cpu'))
  logdir = str(tmp_path)
  for f in (10, 20, 30):
    learner.frames.fill_(f)
    ckpt.save(logdir, learner, flags, keep=2, fmt='tf')
  assert [n for n, _ in __import__(
      'scalable_agent_amd.tf_checkpoint',
      fromlist=['x']).list_tf_checkpoints(logdir)] == [20, 30]
  assert ckpt.latest_checkpoint(logdir).endswith('model.ckpt-30')
  saved = {n: p.detach().clone() for n, p in learner.flat.named}
  with torch.no_grad():
    learner.flat.params.add_(1.0)
    learner.opt.ms.add_(1.0)
  state = ckpt.load_state(ckpt.latest_checkpoint(logdir))
  assert state['num_environment_frames'] == 30
  learner.frames.fill_(0)
  assert ckpt.restore(logdir, learner) == 30
  for n, p in learner.flat.named:  # (the flat buffer's padding is not saved)
    assert torch.equal(p, saved[n]), n
  assert int(learner.frames) == 30


@pytest.mark.parametrize('groups', [0, 1])
def test_train_with_grouped_env_workers(tmp_path, groups):
  """--envs_per_worker=3: the 5 envs run in two worker processes (3 + 2,
  py_process.start_group), with actor threads (groups=0) and with an actor
  group process stepping them split-phase (groups=1)."""
  logdir = str(tmp_path / ('grouped%d' % groups))
  r = _run(['--logdir=' + logdir, '--num_actors=5', '--batch_size=2',
            '--total_environment_frames=400', '--save_summaries_secs=0',
            '--envs_per_worker=3', '--actor_groups=%d' % groups])
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'Episode return' in r.stderr


def test_auto_board_layout_group_counts():
  """--actor_groups=-1 on a GPU: CPU groups of ~40 envs (>= 2) with the
  inference board from AUTO_BOARD_ACTORS actors on (profiles/r6_e2e.md)."""
  from scalable_agent_amd import experiment as ex
  assert ex.AUTO_BOARD_ACTORS == 32
  assert [ex.auto_board_groups(n) for n in (32, 48, 80, 81, 150, 200)] == \
      [2, 2, 2, 3, 4, 5]
