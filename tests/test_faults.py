"""Failure detection / recovery: supervised env workers
(crash respawn, hang watchdog, stale-reply protocol), the non-finite update
guard, --fault_inject parsing, and checkpoint-on-SIGTERM end to end."""

import os
import signal
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

from scalable_agent_amd import py_process
from scalable_agent_amd.actor import Actor
from scalable_agent_amd.environments import FlowEnvironment
from scalable_agent_amd.envs.synthetic import SyntheticEnv
from scalable_agent_amd.runtime.faults import FaultSpec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPE = (12, 16, 3)


def _env(**sup):
  return py_process.EnvProcess(SyntheticEnv, SHAPE, 'synthetic', {}, 4, 1,
                               frame_shape=SHAPE, episode_length=50, **sup)


def test_fault_spec():
  f = FaultSpec('env_crash:0.5,actor_stall:20,learner_nan:3')
  assert f.get('env_crash') == 0.5 and f.get('actor_stall') == 20
  assert f.env_spec() == 'env_crash:0.5'
  assert not FaultSpec('')
  with pytest.raises(ValueError, match='bad --fault_inject'):
    FaultSpec('disk_full:1')


def test_env_crash_respawn():
  env = _env(fault_inject='env_crash:0.2', fault_seed=3).start()
  try:
    env.initial()
    restarts = 0
    for _ in range(100):
      try:
        env.step(0)
      except py_process.EnvRestartedError:
        restarts += 1
        env.initial()  # a fresh episode on the replacement worker
    assert restarts >= 3
    assert env.restarts == restarts
    assert env.is_alive
  finally:
    env.close()
  assert not env.is_alive


def test_env_hang_watchdog():
  env = _env(fault_inject='env_hang:0.3', fault_seed=5, timeout=0.5).start()
  try:
    env.initial()
    t0 = time.time()
    hung = 0
    for _ in range(20):
      try:
        env.step(1)
      except py_process.EnvRestartedError:
        hung += 1
        env.initial()
    assert hung >= 1
    assert time.time() - t0 < 20 * 0.5 + 15
  finally:
    env.close()


def test_env_exception_is_reraised_not_respawned():
  class Broken(SyntheticEnv):
    def step(self, action):
      raise ValueError('broken env step')

  env = py_process.EnvProcess(Broken, SHAPE, 'synthetic', {}, 4, 1,
                              frame_shape=SHAPE).start()
  try:
    env.initial()
    with pytest.raises(ValueError, match='broken env step'):
      env.step(0)
  finally:
    env.close()


def test_actor_drops_unroll_on_restart():
  env = _env(fault_inject='env_crash:0.05', fault_seed=11).start()
  calls = []

  def infer(last_action, reward, done, frame, ids, n, c, h):
    calls.append(1)
    return (np.zeros(1, np.int64), np.zeros((1, 9), np.float32),
            np.zeros(1, np.float32), c, h)

  actor = Actor(FlowEnvironment(env), infer, 'synthetic', list(range(9)), 10,
                9, use_instruction=False)
  try:
    for _ in range(8):
      out = actor.unroll()
      assert out.env_outputs.reward.shape == (11,)
    assert actor.env_restarts >= 1
  finally:
    env.close()


def test_nonfinite_update_skipped():
  from scalable_agent_amd.optim import FlatParams, RMSProp
  m = torch.nn.Linear(4, 4)
  flat = FlatParams(m)
  opt = RMSProp(flat, 0.1, use_hip=False)
  before = flat.params.clone()
  flat.grads.fill_(1.0)
  flat.grads[3] = float('nan')
  opt.step(torch.zeros((), dtype=torch.int64))
  assert torch.equal(flat.params, before) and opt.skipped_steps == 1
  flat.grads.fill_(1.0)
  opt.step(torch.zeros((), dtype=torch.int64))
  assert not torch.equal(flat.params, before) and opt.skipped_steps == 1


COMMON = ['--level_name=synthetic', '--unroll_length=5', '--device=cpu',
          '--dtype=fp32', '--torso=shallow', '--synthetic_episode_length=6',
          '--height=24', '--width=32']


def test_train_survives_env_crashes_and_nan_batch(tmp_path):
  logdir = str(tmp_path / 'faulty')
  r = subprocess.run(
      [sys.executable, os.path.join(ROOT, 'experiment.py')] + COMMON + [
          '--logdir=' + logdir, '--num_actors=3', '--batch_size=2',
          '--total_environment_frames=800', '--save_summaries_secs=0',
          '--fault_inject=env_crash:0.02,learner_nan:2'],
      capture_output=True, text=True, timeout=300,
      env=dict(os.environ, PYTHONPATH=ROOT))
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'dropping the in-flight unroll' in r.stderr
  import json
  rows = [json.loads(l) for l in open(os.path.join(logdir,
                                                    'summaries.jsonl'))]
  skipped = [x['skipped_updates'] for x in rows if 'skipped_updates' in x]
  assert skipped and max(skipped) == 1


def test_sigterm_checkpoints(tmp_path):
  logdir = str(tmp_path / 'term')
  p = subprocess.Popen(
      [sys.executable, os.path.join(ROOT, 'experiment.py')] + COMMON + [
          '--logdir=' + logdir, '--num_actors=2', '--batch_size=2',
          '--total_environment_frames=100000000', '--save_checkpoint_secs=1e9',
          '--log_every_frames=1'],
      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
      env=dict(os.environ, PYTHONPATH=ROOT))
  try:
    deadline = time.time() + 180
    # wait until training is underway (the first throughput log line)
    while time.time() < deadline:
      line = p.stderr.readline()
      if 'frames/s' in line:
        break
    p.send_signal(signal.SIGTERM)
    _, err = p.communicate(timeout=120)
  finally:
    if p.poll() is None:
      p.kill()
  assert p.returncode == 0, err[-3000:]
  assert 'SIGTERM: stopping and checkpointing' in err
  assert os.path.exists(os.path.join(logdir, 'checkpoint'))
