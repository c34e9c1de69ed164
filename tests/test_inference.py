"""Batched actor inference: the packed-staging server (native GetInputsPacked
+ one-slab copies) against the per-call path, and the packed batcher API."""

import threading

import numpy as np
import pytest
import torch

from scalable_agent_amd import dynamic_batching
from scalable_agent_amd import inference
from scalable_agent_amd.models.agent import Agent


def _args(rng, k):
  return (np.array([k % 9], np.int64), np.array([0.5 * k], np.float32),
          np.array([k == 2]),
          rng.randint(0, 255, (1, 72, 96, 3)).astype(np.uint8),
          np.zeros((1, 16), np.int64), np.zeros(1, np.int64),
          rng.rand(1, 256).astype(np.float32),
          rng.rand(1, 256).astype(np.float32))


def test_get_inputs_packed_layout():
  b = dynamic_batching.Batcher(3, 3, None)
  outs = {}

  def client(i):
    x = np.full((1, 5), i, np.float32)
    y = np.full((1, 2, 3), i, np.int64)
    z = np.array([i % 2 == 0])
    outs[i] = b.compute([x, y, z])

  ts = [threading.Thread(target=client, args=(i,)) for i in range(3)]
  for t in ts:
    t.start()
  slab = np.zeros(4096, np.uint8)
  n, cid, used, rows, metas = b.get_inputs_packed(slab.ctypes.data,
                                                  slab.nbytes, 256)
  assert n == 3 and rows == 3
  assert [m[2] for m in metas] == [0, 256, 512]
  assert used == 512 + 3
  x = slab[0:60].view(np.float32).reshape(3, 5)
  y = slab[256:256 + 144].view(np.int64).reshape(3, 2, 3)
  z = slab[512:515].view(np.bool_)
  assert sorted(x[:, 0].tolist()) == [0, 1, 2]
  assert (x[:, :1] == x).all() and (y[:, 0, 0] == x[:, 0]).all()
  assert (z == (x[:, 0] % 2 == 0)).all()
  b.set_outputs([x * 2], cid)
  for t in ts:
    t.join()
  for i in range(3):
    assert np.all(outs[i][0] == 2 * i)
  # too small a slab is an InvalidArgument that closes the batcher
  ts = [threading.Thread(target=lambda: pytest.raises(
      dynamic_batching.CancelledError, b.compute,
      [np.zeros((1, 5), np.float32)])) for _ in range(3)]
  for t in ts:
    t.start()
  with pytest.raises(dynamic_batching.InvalidArgumentError):
    b.get_inputs_packed(slab.ctypes.data, 16, 256)
  for t in ts:
    t.join()
  assert b.closed


def test_staged_server_matches_direct_inference():
  torch.manual_seed(0)
  agent = Agent(9, torso='shallow', frame_shape=(72, 96, 3))
  model = inference.InferenceModel(agent, 'cpu', True, seed=3)
  ref = inference.InferenceModel(
      Agent(9, torso='shallow', frame_shape=(72, 96, 3)), 'cpu', True, seed=3)
  ref.flat.params.copy_(model.flat.params)
  srv = inference.make_batched_infer(model, 1, 8, 20, staged=True)
  assert isinstance(srv, inference.StagedBatchedInfer)
  errors = []

  def actor(i):
    rng = np.random.RandomState(i)
    try:
      for k in range(4):
        a = _args(rng, k)
        o = srv(*a)
        r = ref.infer(*a)
        for got, want in zip(o[1:], r[1:]):
          np.testing.assert_allclose(got, want, atol=1e-5, rtol=1e-5)
        assert o[0].shape == (1,) and 0 <= int(o[0][0]) < 9
    except Exception as e:  # pylint: disable=broad-except
      errors.append(e)

  ts = [threading.Thread(target=actor, args=(i,)) for i in range(6)]
  for t in ts:
    t.start()
  for t in ts:
    t.join()
  st = srv.stats()
  srv.close()
  srv.join()
  assert not errors, errors[0]
  assert st['requests'] == 24 and 1 <= st['batches'] <= 24


def test_get_inputs_packed_pow2_layout():
  b = dynamic_batching.Batcher(3, 8, None)
  outs = {}

  def client(i):
    outs[i] = b.compute([np.full((1, 5), i, np.float32),
                         np.full((1, 6), i, np.int64)])

  ts = [threading.Thread(target=client, args=(i,)) for i in range(3)]
  for t in ts:
    t.start()
  slab = np.zeros(4096, np.uint8)
  n, cid, used, rows, metas = b.get_inputs_packed(
      slab.ctypes.data, slab.nbytes, 256, True)
  assert (n, rows) == (3, 4)
  assert [m[2] for m in metas] == [0, 256] and used == 256 + 4 * 48
  assert metas[0][1] == [3, 5]
  x = slab[0:60].view(np.float32).reshape(3, 5)
  b.set_outputs([x + 1], cid)
  for t in ts:
    t.join()
  for i in range(3):
    assert np.all(outs[i][0] == i + 1)
