"""Native shared-memory env channel (csrc/envpool/env_channel.cc) and the
EnvProcess hot path over it: request/response across a fork, action and
instruction encodings, a replacement worker ignoring its predecessor's
unanswered request, and errors surfacing through the pipe."""

import multiprocessing as mp
import os

import numpy as np
import pytest

from scalable_agent_amd import py_process
from scalable_agent_amd.runtime import native


def _serve(chan, n):
  for _ in range(n):
    while True:
      seq, method, kind, vals = chan.wait_request(1000)
      if seq >= 0:
        break
    act = py_process._decode_action(kind, vals)
    reward = float(np.sum(act)) + method
    instr = py_process._encode_instr('step %d' % seq if method else None)
    chan.respond(seq, 0, reward, bool(method), instr)
  os._exit(0)


def test_round_trip_across_fork():
  chan = native.EnvChannel()
  p = mp.get_context('fork').Process(target=_serve, args=(chan, 3))
  p.start()
  try:
    for method, action in ((1, 3), (1, (0, 0, -20, 1, 0, 0, 0)),
                           (0, None)):
      kind, vals = (py_process._encode_action(action) if action is not None
                    else (0, [0.0]))
      seq = chan.request(method, kind, vals)
      assert chan.wait_response(seq, 5000) == 1
      want = float(np.sum(action if action is not None else 0)) + method
      assert chan.reward == pytest.approx(want)
      assert chan.done == bool(method)
      instr = py_process._decode_instr(chan.instr)
      assert instr == ('step %d' % seq if method else None)
  finally:
    p.join(10)
  assert p.exitcode == 0


def test_action_encoding():
  assert py_process._encode_action(4) == (0, [4.0])
  assert py_process._decode_action(0, [4.0]) == 4
  k, v = py_process._encode_action((20, 0, 0, 1, 0, 0, 0))
  a = py_process._decode_action(k, v)
  assert a.dtype == np.int64 and a.tolist() == [20, 0, 0, 1, 0, 0, 0]
  k, v = py_process._encode_action(np.array([0.5, -1.0]))
  assert py_process._decode_action(k, v).tolist() == [0.5, -1.0]
  assert py_process._encode_action(np.zeros((2, 2))) is None  # -> pipe
  assert py_process._encode_action(list(range(17))) is None
  assert py_process._decode_instr(py_process._encode_instr(b'\x00raw')) == \
      b'\x00raw'


def test_replacement_worker_skips_the_unanswered_request():
  chan = native.EnvChannel()
  seq = chan.request(1, 0, [1.0])  # the "dead" worker never answers
  chan.discard_pending()           # what a replacement worker does first
  assert chan.wait_request(20)[0] == -1
  assert chan.wait_response(seq, 20) == 0  # and the caller is not answered
  seq2 = chan.request(1, 0, [2.0])
  got = chan.wait_request(100)
  assert got[0] == seq2 and got[3] == [2.0]


class _Boom(object):
  def __init__(self, *a, **k):
    self.n = 0

  def initial(self):
    return [np.zeros((2, 2, 1), np.uint8), 'hi']

  def step(self, action):
    self.n += 1
    if action == 7:
      raise ValueError('bad action 7')
    return np.float32(action), np.bool_(False), [
        np.full((2, 2, 1), self.n, np.uint8), 'x']

  def close(self):
    pass


def test_env_process_channel_path_and_errors():
  env = py_process.EnvProcess(_Boom, (2, 2, 1)).start()
  try:
    assert env._chan is not None
    frame, instr = env.initial()
    assert instr == 'hi' and frame.shape == (2, 2, 1)
    r, d, (frame, instr) = env.step(3)
    assert r == 3.0 and not d and instr == 'x' and frame[0, 0, 0] == 1
    with pytest.raises(ValueError, match='bad action 7'):
      env.step(7)
    r, _, (frame, _) = env.step(2)  # the worker survives an env exception
    assert r == 2.0 and frame[0, 0, 0] == 3
  finally:
    env.close()
  assert not env.is_alive
