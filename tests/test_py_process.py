"""Port of the reference py_process_test.py (py_process_test.py:31-221):
fake env backends are in-test classes hosted in real subprocesses."""

import os
import tempfile
import threading
import time

import numpy as np
import pytest

from scalable_agent_amd import py_process


class _Small(object):

  def __init__(self, a):
    self._a = a

  def inc(self):
    self._a += 1

  def compute(self, b):
    return np.array(self._a + b, dtype=np.int32)


def test_small():
  p = py_process.PyProcess(_Small, 1)
  py_process.start_all([p])
  try:
    assert p.proxy.inc() is None
    assert p.proxy.compute(2) == 4
  finally:
    py_process.close_all([p])


class _Wait(object):

  def wait(self):
    time.sleep(.2)


def test_threading():
  p = py_process.PyProcess(_Wait).start()
  errors = []

  def run():
    try:
      p.proxy.wait()
    except py_process.OutOfRangeError as e:
      errors.append(e)

  t = threading.Thread(target=run)
  t.start()
  time.sleep(.1)
  p.close()
  t.join()
  assert len(errors) == 1


class _Args(object):

  def __init__(self, dim0):
    self._dim0 = dim0

  def compute(self, dim1):
    return np.zeros([self._dim0, dim1], dtype=np.int32)


def test_args():
  p = py_process.PyProcess(_Args, 1).start()
  try:
    r = p.proxy.compute(2)
    assert r.shape == (1, 2)
    np.testing.assert_array_equal([[0, 0]], r)
  finally:
    p.close()


class _BadCtor(object):

  def __init__(self):
    raise ValueError('foo')


def test_error_handling_constructor():
  p = py_process.PyProcess(_BadCtor)
  with pytest.raises(Exception, match='foo'):
    py_process.start_all([p])


class _BadMethod(object):

  def something(self):
    raise ValueError('foo')


def test_error_handling_method():
  p = py_process.PyProcess(_BadMethod).start()
  try:
    with pytest.raises(Exception, match='foo'):
      p.proxy.something()
  finally:
    p.close()


class _Closer(object):

  def __init__(self, filename):
    self._filename = filename

  def something(self):
    raise ValueError('foo')

  def close(self):
    with open(self._filename, 'w') as f:
      f.write('was_closed')


def test_close():
  with tempfile.TemporaryDirectory() as d:
    fn = os.path.join(d, 'c')
    p = py_process.PyProcess(_Closer, fn)
    py_process.start_all([p])
    py_process.close_all([p])
    assert open(fn).read() == 'was_closed'


def test_close_on_error():
  with tempfile.TemporaryDirectory() as d:
    fn = os.path.join(d, 'c')
    p = py_process.PyProcess(_Closer, fn).start()
    with pytest.raises(Exception, match='foo'):
      p.proxy.something()
    p.close()
    assert open(fn).read() == 'was_closed'


def test_many_processes_dmlab_shaped_frames():
  """Benchmark-shaped smoke (py_process_test.py:224-270): 16 processes
  returning uint8[72,96,3] frames through shared memory."""
  from scalable_agent_amd.envs.synthetic import SyntheticEnv
  ps = [py_process.EnvProcess(SyntheticEnv, (72, 96, 3), 'synthetic', {}, 4, i)
        for i in range(16)]
  py_process.start_all(ps)
  try:
    for p in ps:
      frame, instr = p.initial()
      assert frame.shape == (72, 96, 3) and frame.dtype == np.uint8
      r, d, (frame2, _) = p.step(0)
      assert frame2.shape == (72, 96, 3)
  finally:
    py_process.close_all(ps)


class _Boom(object):
  """An env whose step(7) raises (the others answer normally)."""

  def __init__(self, seed):
    self._s = seed

  def initial(self):
    return [np.full((4, 4, 1), self._s, np.uint8), None]

  def step(self, action):
    if int(action) == 7:
      raise ValueError('boom %d' % self._s)
    return (np.float32(self._s), np.bool_(False),
            [np.full((4, 4, 1), self._s + int(action), np.uint8), None])

  def close(self):
    pass


def test_grouped_envs_match_separate_ones():
  """start_all(per_worker=k): k envs in one worker process (one doorbell,
  one wake per batch) give the same frames / rewards / dones as one env per
  process, through the split-phase calls an actor group uses."""
  from scalable_agent_amd.envs.synthetic import SyntheticEnv

  def make():
    return [py_process.EnvProcess(SyntheticEnv, (72, 96, 3), 'synthetic', {},
                                  4, i) for i in range(5)]
  sep, grp = make(), make()
  py_process.start_all(sep)
  py_process.start_all(grp, per_worker=3)  # groups of 3 and 2
  try:
    assert len({p._process.pid for p in grp}) == 2
    assert grp[0]._process is grp[2]._process is not grp[3]._process
    for a, b in zip(sep, grp):
      a.initial_nocopy()
      b.initial_nocopy()
      assert np.array_equal(a.frame_view, b.frame_view)
    for t in range(20):
      ta = [p.step_send(t % 9) for p in sep]
      tb = [p.step_send(t % 9) for p in grp]
      for p, q, sa, sb in zip(sep, grp, ta, tb):
        assert p.step_recv(sa) == q.step_recv(sb)
        assert np.array_equal(p.frame_view, q.frame_view)
  finally:
    py_process.close_all(sep)
    py_process.close_all(grp)
  assert not any(p.is_alive for p in grp)


def test_grouped_env_error_stays_with_its_env():
  ps = [py_process.EnvProcess(_Boom, (4, 4, 1), i) for i in range(3)]
  py_process.start_all(ps, per_worker=3)
  try:
    for p in ps:
      p.initial()
    with pytest.raises(ValueError, match='boom 1'):
      ps[1].step(7)
    # the other envs of the worker are unaffected, and so is env 1
    for i, p in enumerate(ps):
      r, d, (f, _) = p.step(2)
      assert float(r) == i and int(f[0, 0, 0]) == i + 2
  finally:
    py_process.close_all(ps)


def test_grouped_env_crash_restarts_the_group():
  """A crashed group worker (env_crash fault) is respawned by the group's
  supervisor: every member's caller sees EnvRestartedError once, then the
  envs step again."""
  from scalable_agent_amd.envs.synthetic import SyntheticEnv
  ps = [py_process.EnvProcess(SyntheticEnv, (8, 8, 3), 'synthetic', {}, 4, i,
                              frame_shape=(8, 8, 3),
                              fault_inject='env_crash:0.01', fault_seed=5)
        for i in range(3)]
  py_process.start_all(ps, per_worker=3)
  seen = [0] * 3

  def initial(p):
    while True:  # a restart notice may arrive on the initial() itself
      try:
        return p.initial()
      except py_process.EnvRestartedError:
        pass
  try:
    for p in ps:
      initial(p)
    for _ in range(200):
      for i, p in enumerate(ps):
        try:
          p.step(0)
        except py_process.EnvRestartedError:
          seen[i] += 1
          initial(p)
    assert ps[0].restarts >= 1
    assert all(n >= 1 for n in seen), seen
  finally:
    py_process.close_all(ps)
