"""Hosts Python objects (environments) in separate processes.

Behaviour parity with the reference py_process.py:62-222:
  * `PyProcess(type_, *args, **kwargs)` constructs `type_(*args, **kwargs)` in
    a child process; `p.proxy.<method>(*args)` forwards the call over a pipe
    and returns the (flattened) result;
  * a constructor exception is re-raised by `start()`, a method exception is
    re-raised in the caller and the object's `close()` is still attempted;
  * `close()` sends the stop message, calls the object's `close()` in the
    child and joins; a call blocked while the process is being closed raises
    `OutOfRangeError` (the reference's IOError -> StopIteration -> OutOfRange
    clean-stop path);
  * `start_all` / `close_all` start/stop many processes in parallel (the
    reference's PyProcessHook).

MI355X-era additions: processes are forked BEFORE the learner touches the GPU
(never exec after HIP init), and `EnvProcess` moves observation frames through
a per-process shared-memory slot instead of pickling them.
"""

import multiprocessing
import multiprocessing.pool
import threading
import traceback

import numpy as np

_CTX = multiprocessing.get_context('fork')


class OutOfRangeError(Exception):
  """Raised by a call whose process was closed (clean stop)."""


class _RemoteError(Exception):
  pass


def _worker(type_, args, kwargs, conn):
  obj = None
  try:
    obj = type_(*args, **kwargs)
    conn.send(('ready', None))
    while True:
      msg = conn.recv()
      if msg is None:
        if hasattr(obj, 'close'):
          obj.close()
        conn.close()
        return
      name, margs = msg
      result = getattr(obj, name)(*margs)
      conn.send(('ok', result))
  except (EOFError, KeyboardInterrupt):
    pass
  except Exception as e:  # pylint: disable=broad-except
    if obj is not None and hasattr(obj, 'close'):
      try:
        obj.close()
      except Exception:  # pylint: disable=broad-except
        pass
    try:
      e.remote_traceback = traceback.format_exc()
      conn.send(('error', e))
    except Exception:  # pylint: disable=broad-except
      conn.send(('error', _RemoteError(repr(e))))


class _Proxy(object):

  def __init__(self, process):
    self._p = process

  def __getattr__(self, name):
    def call(*args):
      return self._p._call(name, args)
    return call


class PyProcess(object):
  """See module docstring."""

  def __init__(self, type_, *constructor_args, **constructor_kwargs):
    self._type = type_
    self._args = constructor_args
    self._kwargs = constructor_kwargs
    self._conn = None
    self._process = None
    self._lock = threading.Lock()
    self._closed = False
    self._proxy = _Proxy(self)

  @property
  def proxy(self):
    return self._proxy

  @property
  def constructor_kwargs(self):
    return self._kwargs

  def start(self):
    self._conn, child = _CTX.Pipe()
    self._process = _CTX.Process(target=_worker,
                                 args=(self._type, self._args, self._kwargs,
                                       child), daemon=True)
    self._process.start()
    child.close()
    status, payload = self._conn.recv()
    if status == 'error':
      self._process.join()
      raise payload
    return self

  def _call(self, name, args):
    if self._closed:
      raise OutOfRangeError('process closed')
    with self._lock:
      try:
        self._conn.send((name, args))
        status, payload = self._conn.recv()
      except (EOFError, OSError, BrokenPipeError):
        raise OutOfRangeError('process closed')
      if self._closed:
        raise OutOfRangeError('process closed')
      if status == 'error':
        raise payload
      return payload

  def close(self):
    """Stops the child (calls its object's close()) and joins it."""
    if self._process is None or self._closed:
      self._closed = True
      return
    self._closed = True
    try:
      self._conn.send(None)
    except (OSError, BrokenPipeError):
      pass
    self._process.join(timeout=30)
    if self._process.is_alive():
      self._process.terminate()
      self._process.join()
    try:
      self._conn.close()
    except OSError:
      pass

  @property
  def is_alive(self):
    return self._process is not None and self._process.is_alive()


def start_all(processes):
  """Starts processes in parallel (PyProcessHook.begin)."""
  processes = list(processes)
  if not processes:
    return
  tp = multiprocessing.pool.ThreadPool(min(32, len(processes)))
  try:
    tp.map(lambda p: p.start(), processes)
  finally:
    tp.close()
    tp.join()


def close_all(processes):
  """Closes processes in parallel (PyProcessHook.end)."""
  processes = list(processes)
  if not processes:
    return
  tp = multiprocessing.pool.ThreadPool(min(32, len(processes)))
  try:
    tp.map(lambda p: p.close(), processes)
  finally:
    tp.close()
    tp.join()


# --------------------------------------------------------------------------
# Environment worker with shared-memory observation frames.

def _env_worker(env_ctor, args, kwargs, conn, frame_buf, frame_shape):
  env = None
  frames = np.frombuffer(frame_buf, dtype=np.uint8).reshape(frame_shape)
  try:
    env = env_ctor(*args, **kwargs)
    conn.send(('ready', None))
    while True:
      msg = conn.recv()
      if msg is None:
        env.close()
        conn.close()
        return
      name, margs = msg
      if name == 'initial':
        frame, instr = env.initial()
        frames[...] = frame
        conn.send(('ok', (instr,)))
      elif name == 'step':
        reward, done, (frame, instr) = env.step(*margs)
        frames[...] = frame
        conn.send(('ok', (float(reward), bool(done), instr)))
      else:
        conn.send(('ok', getattr(env, name)(*margs)))
  except (EOFError, KeyboardInterrupt):
    pass
  except Exception as e:  # pylint: disable=broad-except
    if env is not None:
      try:
        env.close()
      except Exception:  # pylint: disable=broad-except
        pass
    conn.send(('error', e))


class EnvProcess(object):
  """Env in a child process; frames cross via shared memory, not pickle.

  The env must follow the reference protocol: `initial() -> [frame, instr]`,
  `step(action) -> (reward, done, [frame, instr])`.
  """

  def __init__(self, env_ctor, obs_shape, *args, **kwargs):
    self._ctor = env_ctor
    self._shape = tuple(obs_shape)
    self._args = args
    self._kwargs = kwargs
    self._buf = _CTX.RawArray('B', int(np.prod(self._shape)))
    self._frames = np.frombuffer(self._buf, dtype=np.uint8).reshape(self._shape)
    self._conn = None
    self._process = None
    self._closed = False

  def start(self):
    self._conn, child = _CTX.Pipe()
    self._process = _CTX.Process(
        target=_env_worker,
        args=(self._ctor, self._args, self._kwargs, child, self._buf,
              self._shape), daemon=True)
    self._process.start()
    child.close()
    status, payload = self._conn.recv()
    if status == 'error':
      self._process.join()
      raise payload
    return self

  def _rpc(self, name, *args):
    if self._closed:
      raise OutOfRangeError('env process closed')
    try:
      self._conn.send((name, args))
      status, payload = self._conn.recv()
    except (EOFError, OSError):
      raise OutOfRangeError('env process closed')
    if status == 'error':
      raise payload
    return payload

  def initial(self):
    (instr,) = self._rpc('initial')
    return [self._frames.copy(), instr]

  def step(self, action):
    reward, done, instr = self._rpc('step', action)
    return np.float32(reward), np.bool_(done), [self._frames.copy(), instr]

  def close(self):
    if self._closed or self._process is None:
      self._closed = True
      return
    self._closed = True
    try:
      self._conn.send(None)
    except (OSError, BrokenPipeError):
      pass
    self._process.join(timeout=30)
    if self._process.is_alive():
      self._process.terminate()
      self._process.join()

  @property
  def is_alive(self):
    return self._process is not None and self._process.is_alive()
