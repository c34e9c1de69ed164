"""Port of the reference dynamic_batching_test.py (15 cases) onto the native
C++ batcher.  The reference's session/QueueRunner plumbing maps to: runner
thread start = `f.start()` (start_queue_runners), runner errors surface from
`f.join()` (Coordinator.join), session close = `f.cancel()`,
coord.request_stop = `f.close()`."""

import datetime
import threading
import time
from multiprocessing import pool

import numpy as np
import pytest

from scalable_agent_amd import dynamic_batching as db

_SLEEP_TIME = 1.0


def _bs_fn(a, b):
  batch_size = a.shape[0]
  return a + b, np.full([batch_size], batch_size, dtype=np.int32)


def test_one():
  f = db.batch_fn(_bs_fn)
  result, batch_size = f(np.array([[1, 3]]), np.array([2]))
  np.testing.assert_array_equal([[3, 5]], result)
  np.testing.assert_array_equal([1], batch_size)
  f.close()
  f.join()


def test_two():
  f = db.batch_fn_with_options(autostart=False)(_bs_fn)
  tp = pool.ThreadPool(2)
  f0 = tp.apply_async(f, [np.array([1]), np.array([2])])
  f1 = tp.apply_async(f, [np.array([2]), np.array([3])])
  time.sleep(_SLEEP_TIME)  # both inputs queued before the runner starts
  f.start()
  result0, batch_size0 = f0.get()
  result1, batch_size1 = f1.get()
  np.testing.assert_array_equal([3], result0)
  np.testing.assert_array_equal([2], batch_size0)
  np.testing.assert_array_equal([5], result1)
  np.testing.assert_array_equal([2], batch_size1)
  f.close()


def test_many_small():
  f = db.batch_fn(lambda a, b: a + b)
  tp = pool.ThreadPool(10)
  futures = [tp.apply_async(f, [np.full([1, 5], i), np.full([1, 5], i)])
             for i in range(200)]
  for i, fut in enumerate(futures):
    np.testing.assert_array_equal([[i * 2] * 5], fut.get())
  f.close()


def test_input_batch_size_should_be_one():
  f = db.batch_fn(lambda a: a)
  with pytest.raises(db.CancelledError):
    f(np.array([1, 2]))
  with pytest.raises(db.InvalidArgumentError, match='requires batch size 1'):
    f.join()


def test_run_after_error_should_be_cancelled():
  f = db.batch_fn(lambda a: a)
  with pytest.raises(db.CancelledError):
    f(np.array([1, 2]))
  with pytest.raises(db.CancelledError):
    f(np.array([1, 2]))


def test_input_shapes_should_be_equal():
  f = db.batch_fn_with_options(autostart=False)(lambda a, b: a + b)
  tp = pool.ThreadPool(2)
  f0 = tp.apply_async(f, [np.array([1]), np.array([2])])
  f1 = tp.apply_async(f, [np.array([[2]]), np.array([3])])
  time.sleep(_SLEEP_TIME)
  f.start()
  with pytest.raises(db.CancelledError):
    f0.get()
    f1.get()
  with pytest.raises(db.InvalidArgumentError,
                     match='Shapes of inputs much be equal'):
    f.join()


def test_output_must_have_batch_dimension():
  f = db.batch_fn(lambda _: np.array(1))
  with pytest.raises(db.CancelledError):
    f(np.array([1]))
  with pytest.raises(db.InvalidArgumentError,
                     match='Output shape must have a batch dimension'):
    f.join()


def test_output_must_have_same_batch_dimension_size_as_input():
  f = db.batch_fn(lambda _: np.array([1, 2, 3, 4]))
  with pytest.raises(db.CancelledError):
    f(np.array([1]))
  with pytest.raises(
      db.InvalidArgumentError,
      match='Output shape must have the same batch dimension as the input '
            'batch size. Expected: 1 Observed: 4'):
    f.join()


def test_get_inputs_cancelled():
  f = db.batch_fn_with_options(autostart=False)(lambda a: a)
  f.start()
  time.sleep(_SLEEP_TIME)  # runner blocked in get_inputs
  f.cancel()                # session close
  with pytest.raises(db.CancelledError,
                     match='GetInputs operation was cancelled'):
    f.join()


def test_batcher_closed():
  f = db.batch_fn_with_options(autostart=False)(lambda a: a)
  f.start()
  time.sleep(_SLEEP_TIME)
  f.close()  # coord.request_stop(): clean shutdown
  f.join()


def test_minimum_batch_size():
  f = db.batch_fn_with_options(minimum_batch_size=2, timeout_ms=1000)(_bs_fn)
  start = datetime.datetime.now()
  f(np.array([[1, 3]]), np.array([2]))
  duration = (datetime.datetime.now() - start).total_seconds()
  # only one sample and minimum 2: returns after the 1 s timeout
  assert .9 <= duration <= 1.5
  tp = pool.ThreadPool(2)
  start = datetime.datetime.now()
  futs = [tp.apply_async(f, [np.array([[1, 3]]), np.array([2])])
          for _ in range(2)]
  (_, batch_size), _ = [x.get() for x in futs]
  duration = (datetime.datetime.now() - start).total_seconds()
  assert duration <= .5
  assert batch_size[0] == 2
  f.close()


def test_maximum_batch_size():
  f = db.batch_fn_with_options(maximum_batch_size=2)(_bs_fn)
  tp = pool.ThreadPool(5)
  futs = [tp.apply_async(f, [np.array([1]), np.array([2])]) for _ in range(5)]
  for fut in futs:
    value, batch_size = fut.get()
    assert value[0] == 3
    assert batch_size[0] <= 2
  f.close()


def test_static_shape():
  """Eager analogue of the TF static-shape test: with min == max and no
  timeout the function always sees exactly that batch size; otherwise any
  size up to the maximum."""
  seen0, seen2 = [], []
  f0 = db.batch_fn_with_options(minimum_batch_size=1, maximum_batch_size=2)(
      lambda a: (seen0.append(a.shape[0]), a)[1])
  f2 = db.batch_fn_with_options(minimum_batch_size=2, maximum_batch_size=2,
                                timeout_ms=None)(
      lambda a: (seen2.append(a.shape[0]), a)[1])
  tp = pool.ThreadPool(4)
  futs = [tp.apply_async(f, [np.array([1])]) for f in (f0, f0, f2, f2)]
  for fut in futs:
    fut.get()
  assert all(1 <= s <= 2 for s in seen0)
  assert seen2 == [2]
  f0.close()
  f2.close()


def _run_out_of_order(reverse):
  batcher = db.Batcher(minimum_batch_size=1, maximum_batch_size=1,
                       timeout_ms=None)
  tp = pool.ThreadPool(10)
  r0 = tp.apply_async(batcher.compute, [[np.array([1])]])
  (input0,), cid0 = batcher.get_inputs()
  r1 = tp.apply_async(batcher.compute, [[np.array([2])]])
  (input1,), cid1 = batcher.get_inputs()
  np.testing.assert_array_equal([1], input0)
  np.testing.assert_array_equal([2], input1)
  order = [(input0, cid0), (input1, cid1)]
  if reverse:
    order = order[::-1]
  for inp, cid in order:
    batcher.set_outputs([inp + 42], cid)
  np.testing.assert_array_equal([43], r0.get()[0])
  np.testing.assert_array_equal([44], r1.get()[0])
  batcher.close()


def test_out_of_order_execution1():
  _run_out_of_order(False)


def test_out_of_order_execution2():
  _run_out_of_order(True)


def test_invalid_computation_id():
  batcher = db.Batcher(minimum_batch_size=1, maximum_batch_size=1,
                       timeout_ms=None)
  tp = pool.ThreadPool(10)
  tp.apply_async(batcher.compute, [[np.array([1])]])
  (input0,), _ = batcher.get_inputs()
  np.testing.assert_array_equal([1], input0)
  with pytest.raises(db.InvalidArgumentError, match='Invalid computation id'):
    batcher.set_outputs([input0], 42)


def test_op_shape():
  batcher = db.Batcher(minimum_batch_size=1, maximum_batch_size=1,
                       timeout_ms=None)
  errors = []

  def call():
    try:
      batcher.compute([np.array([1])])
    except db.CancelledError as e:  # close() cancels the pending call
      errors.append(e)

  t = threading.Thread(target=call)
  t.start()
  _, computation_id = batcher.get_inputs()
  assert isinstance(computation_id, int) and np.ndim(computation_id) == 0
  batcher.close()
  t.join()
  assert len(errors) == 1


# ---- beyond the reference -------------------------------------------------

def test_get_inputs_into_caller_buffer():
  batcher = db.Batcher(2, 4, None)
  tp = pool.ThreadPool(2)
  futs = [tp.apply_async(batcher.compute,
                         [[np.full([1, 3], i, np.float32)]]) for i in (1, 2)]
  buf = np.zeros((4, 3), np.float32)
  n, cid, metas = batcher.get_inputs_into([(buf.ctypes.data, buf.nbytes)])
  assert n == 2 and metas[0][1] == [2, 3]
  assert sorted(buf[:2, 0].tolist()) == [1.0, 2.0]
  batcher.set_outputs([buf[:2] * 10], cid)
  vals = sorted(float(f.get()[0][0, 0]) for f in futs)
  assert vals == [10.0, 20.0]
  batcher.close()


def test_close_cancels_pending_and_later_calls():
  batcher = db.Batcher(5, 5, None)
  tp = pool.ThreadPool(2)
  fut = tp.apply_async(batcher.compute, [[np.array([1])]])
  time.sleep(0.2)
  batcher.close()
  with pytest.raises(db.CancelledError, match='Compute was cancelled'):
    fut.get()
  with pytest.raises(db.CancelledError, match='Batcher is closed'):
    batcher.compute([np.array([1])])


def test_stress_many_threads_many_batches():
  f = db.batch_fn_with_options(maximum_batch_size=64, timeout_ms=5)(
      lambda a: a * 2)
  tp = pool.ThreadPool(32)
  futs = [tp.apply_async(f, [np.array([[i, -i]])]) for i in range(2000)]
  for i, fut in enumerate(futs):
    np.testing.assert_array_equal([[2 * i, -2 * i]], fut.get())
  f.close()
