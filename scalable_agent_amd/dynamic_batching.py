"""Dynamic batching of per-actor calls (reference dynamic_batching.py:30-162).

The C++17 batcher (csrc/batcher/, `runtime._native.Batcher`) replaces the
reference's TF custom op (batcher.cc).  Semantics kept:

  * `batch_fn` / `batch_fn_with_options(minimum_batch_size=1,
    maximum_batch_size=1024, timeout_ms=100)` decorate a function whose inputs
    are nests of arrays with leading dimension 1; concurrent callers are
    coalesced into one batched call of `f` executed by a runner thread, and
    each caller receives its own row of the result;
  * min/max batch size, timeout (None = wait for the minimum), out-of-order
    `set_outputs` across computation ids, cancellation/close, and the same
    error messages (CancelledError / InvalidArgumentError).

Beyond the reference, `Batcher.get_inputs_into()` gathers the request rows
straight into caller-provided (pinned host) buffers so a GPU inference server
can issue one hipMemcpyAsync per batch.
"""

import functools
import threading

import numpy as np

from .runtime import native as _native_loader
from .utils import nest

_N = _native_loader.load()
CancelledError = _N.CancelledError
InvalidArgumentError = _N.InvalidArgumentError


class Batcher(object):
  """Thin Python layer over the native batcher (mirrors `_Batcher`)."""

  def __init__(self, minimum_batch_size, maximum_batch_size, timeout_ms):
    self._impl = _N.Batcher(int(minimum_batch_size), int(maximum_batch_size),
                            -1 if timeout_ms is None else int(timeout_ms))

  @property
  def name(self):
    return 'batcher'

  def compute(self, flat_args):
    return self._impl.compute([np.asarray(a) for a in flat_args])

  def get_inputs(self):
    """Returns (list of batched arrays, computation_id)."""
    return self._impl.get_inputs()

  def get_inputs_into(self, buffers):
    """buffers: list of (address, nbytes). Returns (batch, id, metas)."""
    return self._impl.get_inputs_into(list(buffers))

  def get_inputs_packed(self, address, capacity, align=256,
                        layout_pow2=False):
    """Gathers the batch into ONE slab at `address` (capacity bytes), input
    k at an `align`-aligned offset (segments sized for `layout_rows` rows:
    the batch, or with layout_pow2 the batch rounded up to a power of two).
    Returns (batch, id, used_bytes, layout_rows, [(dtype, shape, offset)])."""
    return self._impl.get_inputs_packed(int(address), int(capacity),
                                        int(align), bool(layout_pow2))

  def set_outputs(self, flat_result, computation_id):
    self._impl.set_outputs([np.require(r, requirements='C') for r in flat_result],
                           int(computation_id))

  def close(self, cancel_pending_enqueues=False):
    del cancel_pending_enqueues
    self._impl.close()

  def cancel(self):
    self._impl.cancel()

  @property
  def closed(self):
    return self._impl.closed

  @property
  def num_batches(self):
    return self._impl.num_batches

  @property
  def num_requests(self):
    return self._impl.num_requests


class Runner(object):
  """Runner thread: get_inputs -> f -> set_outputs until the batcher closes.

  Plays the role of the reference's QueueRunner; errors other than the
  close-induced CancelledError are recorded and re-raised by `join()` (the
  tf.train.Coordinator behaviour the reference tests rely on).
  """

  def __init__(self, batcher, fn, in_structure_fn, name='batcher-runner'):
    self._batcher = batcher
    self._fn = fn
    self._in_structure_fn = in_structure_fn
    self.out_structure = None
    self._structure_ready = threading.Event()
    self._error = None
    self._stop_requested = False
    self._thread = threading.Thread(target=self._run, name=name, daemon=True)

  def start(self):
    self._thread.start()
    return self

  def _run(self):
    try:
      while True:
        inputs, cid = self._batcher.get_inputs()
        args = nest.pack_sequence_as(self._in_structure_fn(), inputs)
        result = self._fn(*args)
        if self.out_structure is None:
          self.out_structure = result
          self._structure_ready.set()
        self._batcher.set_outputs(
            [np.asarray(r) for r in nest.flatten(result)], cid)
    except CancelledError as e:
      if not self._stop_requested and 'Batcher is closed' not in str(e):
        self._error = e
    except BaseException as e:  # pylint: disable=broad-except
      self._error = e
      try:
        self._batcher.cancel()
      except Exception:  # pragma: no cover
        pass
    finally:
      self._structure_ready.set()

  def request_stop(self):
    self._stop_requested = True
    self._batcher.close()

  def join(self, timeout=None):
    """Waits for the thread; re-raises its error (Coordinator.join)."""
    self._thread.join(timeout)
    if self._error is not None:
      raise self._error

  @property
  def error(self):
    return self._error

  def is_alive(self):
    return self._thread.is_alive()


def batch_fn(f):
  """See `batch_fn_with_options` for details."""
  return batch_fn_with_options()(f)


def batch_fn_with_options(minimum_batch_size=1, maximum_batch_size=1024,
                          timeout_ms=100, autostart=True):
  """Decorator that automatically batches concurrent calls of `f`.

  Every input leaf must have a leading dimension of size 1.  The first call
  lazily creates the batcher; the runner thread starts then (autostart) or on
  `wrapper.start()` (the reference's `tf.train.start_queue_runners()`).  The
  decorated function exposes `.start()`, `.close()`, `.cancel()`, `.join()`.
  """

  def decorator(f):
    state = {'batcher': None, 'runner': None, 'in_structure': None,
             'started': False}
    lock = threading.Lock()

    def _create():
      if state['batcher'] is None:
        state['batcher'] = Batcher(minimum_batch_size, maximum_batch_size,
                                   timeout_ms)
        state['runner'] = Runner(state['batcher'], f,
                                 lambda: state['in_structure'])

    def _start_locked():
      if not state['started']:
        state['started'] = True
        state['runner'].start()

    def _ensure(args):
      with lock:
        if state['in_structure'] is None:
          state['in_structure'] = args
        _create()
        if autostart:
          _start_locked()
      return state['batcher'], state['runner']

    def start():
      with lock:
        _create()
        _start_locked()

    @functools.wraps(f)
    def wrapper(*args):
      batcher, runner = _ensure(args)
      flat = [np.asarray(a) for a in nest.flatten(args)]
      flat_result = batcher.compute(flat)
      runner._structure_ready.wait()
      if runner.out_structure is None:
        return flat_result
      return nest.pack_sequence_as(runner.out_structure, flat_result)

    def close():
      if state['runner'] is not None:
        state['runner'].request_stop()

    def cancel():
      if state['batcher'] is not None:
        state['batcher'].cancel()

    def join(timeout=None):
      if state['runner'] is not None and state['started']:
        state['runner'].join(timeout)

    def stats():
      """{'batches', 'requests'} served so far (mean batch = ratio)."""
      b = state['batcher']
      impl = getattr(b, '_impl', None)
      if impl is None:
        return {'batches': 0, 'requests': 0}
      return {'batches': int(impl.num_batches),
              'requests': int(impl.num_requests)}

    wrapper.start = start
    wrapper.stats = stats
    wrapper.close = close
    wrapper.cancel = cancel
    wrapper.join = join
    wrapper.state = state
    return wrapper

  return decorator
