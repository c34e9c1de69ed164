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
