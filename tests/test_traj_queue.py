"""Native time-major trajectory queue (csrc/envpool/traj_queue.cc) and the
actor -> slab path: producers claim columns and write [t, b] in place, the
B-th commit publishes a slab, the consumer sees complete batches in fill
order; the same from forked processes over a named shm object."""

import multiprocessing as mp
import os
import threading

import numpy as np
import pytest

from scalable_agent_amd.runtime import native
from scalable_agent_amd.runtime.traj_queue import BatchLayout, TrajectoryQueue


def _fill(v, col, token, T1):
  v['level'][col] = token
  v['c'][col] = token
  for t in range(T1):
    v['reward'][t, col] = token * 1000 + t
    v['frame'][t, col] = token % 251
    v['action'][t, col] = t


def _check(v, T1, B):
  tokens = []
  for col in range(B):
    tok = int(v['level'][col])
    tokens.append(tok)
    assert np.all(v['c'][col] == tok)
    assert np.array_equal(v['reward'][:, col], tok * 1000 + np.arange(T1))
    assert np.all(v['frame'][:, col] == tok % 251)
    assert np.array_equal(v['action'][:, col], np.arange(T1))
  return tokens


def test_threads_fill_columns_in_place():
  T1, B, P, per = 6, 4, 7, 20
  layout = BatchLayout(T1, B, (8, 10, 3), 5)
  tq = TrajectoryQueue(layout, num_slabs=4)
  counter = iter(range(10 ** 6))
  lock = threading.Lock()

  def producer():
    for _ in range(per):
      s, col, v = tq.claim(timeout_ms=5000)
      assert s >= 0
      with lock:
        tok = next(counter)
      _fill(v, col, tok, T1)
      tq.commit(s)

  threads = [threading.Thread(target=producer) for _ in range(P)]
  for t in threads:
    t.start()
  seen = []
  for _ in range(P * per // B):
    s = tq.acquire(timeout_ms=5000)
    assert s >= 0
    seen += _check(tq.host_views(s), T1, B)
    tq.release(s)
  for t in threads:
    t.join()
  assert sorted(seen) == list(range(P * per))  # every unroll exactly once
  assert tq.acquire(timeout_ms=10) == -1
  tq.close()
  assert tq.acquire(timeout_ms=10) == -2
  assert tq.claim(timeout_ms=10)[0] == -2


def test_claim_blocks_until_a_slab_is_released():
  layout = BatchLayout(2, 1, (2, 2, 1), 3)
  tq = TrajectoryQueue(layout, num_slabs=2)
  for _ in range(2):
    s, col, v = tq.claim(timeout_ms=100)
    tq.commit(s)
  assert tq.claim(timeout_ms=50)[0] == -1  # both slabs READY, none free
  s = tq.acquire(timeout_ms=100)
  tq.release(s)
  assert tq.claim(timeout_ms=100)[0] == s


def _proc_producer(name, T1, B, start, n):
  q = native.TrajQueue(name)
  layout = BatchLayout(T1, B, (8, 10, 3), 5)
  views = [layout.numpy_views(q.slab_view(s)) for s in range(q.num_slabs)]
  for k in range(n):
    s, col = q.claim(5000)
    _fill(views[s], col, start + k, T1)
    q.commit(s)


@pytest.mark.skipif(not os.path.isdir('/dev/shm'), reason='needs POSIX shm')
def test_named_queue_across_processes():
  T1, B = 5, 3
  name = '/sa_tq_test_%d' % os.getpid()
  layout = BatchLayout(T1, B, (8, 10, 3), 5)
  tq = TrajectoryQueue(layout, num_slabs=3, name=name)
  ctx = mp.get_context('fork')
  procs = [ctx.Process(target=_proc_producer, args=(name, T1, B, 100 * i, 6))
           for i in range(2)]
  for p in procs:
    p.start()
  seen = []
  for _ in range(12 // B):
    s = tq.acquire(timeout_ms=10000)
    assert s >= 0
    seen += _check(tq.host_views(s), T1, B)
    tq.release(s)
  for p in procs:
    p.join(timeout=10)
    assert p.exitcode == 0
  assert sorted(seen) == sorted(list(range(6)) + list(range(100, 106)))
  tq.close()


def test_claim_n_is_all_or_nothing():
  layout = BatchLayout(2, 4, (2, 2, 1), 3)
  tq = TrajectoryQueue(layout, num_slabs=2)
  got = tq.claim_n(3, timeout_ms=0)
  assert [(s, c) for s, c, _ in got] == [(got[0][0], 0), (got[0][0], 1),
                                         (got[0][0], 2)]
  got2 = tq.claim_n(5, timeout_ms=0)  # 1 left in slab A + 4 in slab B
  assert len(got2) == 5 and got2[0][0] == got[0][0]
  assert tq.claim_n(1, timeout_ms=20) == -1  # full: nothing handed out
  for s, _, _ in got + got2:
    tq.commit(s)
  a = tq.acquire(timeout_ms=100)
  tq.release(a)
  assert len(tq.claim_n(4, timeout_ms=100)) == 4
  tq.close()
  assert tq.claim_n(1, timeout_ms=10) == -2


def test_dead_producer_is_fail_stop():
  """A producer that dies after claiming a column never publishes that slab
  (no half-written unroll reaches the learner): the consumer's acquire times
  out instead, which train() turns into a 'learner starved' stop."""
  T1, B = 3, 2
  layout = BatchLayout(T1, B, (4, 4, 3), 3)
  tq = TrajectoryQueue(layout, num_slabs=3)
  s, col, v = tq.claim(timeout_ms=1000)
  _fill(v, col, 7, T1)
  tq.commit(s)
  # the second column of the same slab is claimed by a thread that then
  # "dies" (never commits)
  s2, col2, _ = tq.claim(timeout_ms=1000)
  assert s2 == s and col2 != col
  assert tq.acquire(timeout_ms=300) < 0
  assert tq.num_ready == 0
  tq.close()
