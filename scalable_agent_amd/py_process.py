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
import multiprocessing.connection
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


def start_all(processes, per_worker=1):
  """Starts processes in parallel (PyProcessHook.begin).  per_worker > 1:
  consecutive EnvProcesses are hosted k at a time by one worker process
  (start_group)."""
  processes = list(processes)
  if not processes:
    return
  units = [[p] for p in processes]
  if per_worker > 1 and all(isinstance(p, EnvProcess) for p in processes):
    units = [processes[i:i + per_worker]
             for i in range(0, len(processes), per_worker)]
  tp = multiprocessing.pool.ThreadPool(min(32, len(units)))
  try:
    tp.map(lambda u: u[0].start() if len(u) == 1 else start_group(u), units)
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
# Environment worker with shared-memory observation frames, supervised.
#
# EnvProcess forks a small single-threaded SUPERVISOR before the learner
# initialises the GPU; the supervisor forks the actual env worker and
# re-forks a fresh one whenever it dies abnormally (signal, os._exit, a
# segfault in a simulator, or a kill by the caller's hang watchdog).  The
# replacement announces itself with a 'restarted' message; the caller raises
# EnvRestartedError so the actor can drop its in-flight unroll and start a
# new episode (env-worker watchdog).  Requests carry sequence
# numbers so a reply that belongs to a request the dead worker never answered
# can never be mistaken for a later one.  Env exceptions are NOT restarts:
# they are re-raised in the caller (reference py_process.py:171-177).


class EnvRestartedError(Exception):
  """The env worker died or hung and was replaced; its episode is lost."""


class _Faults(object):
  """Env-side fault injection: `env_crash:p` hard-kills the worker with
  probability p per step (tests the supervisor/respawn path)."""

  def __init__(self, spec, seed):
    self.crash_p = 0.0
    self.hang_p = 0.0
    for part in filter(None, (spec or '').split(',')):
      k, _, v = part.partition(':')
      if k == 'env_crash':
        self.crash_p = float(v)
      elif k == 'env_hang':
        self.hang_p = float(v)
    self._rng = np.random.RandomState(seed % (2 ** 32))

  def on_step(self):
    import os
    import time
    if self.crash_p and self._rng.rand() < self.crash_p:
      os._exit(17)
    if self.hang_p and self._rng.rand() < self.hang_p:
      time.sleep(3600)


# Hot env calls over the native shared-memory channel (runtime/native
# EnvChannel, csrc/envpool/env_channel.cc): method codes and action encoding.
_M_INITIAL, _M_STEP, _M_CLOSE = 0, 1, 2


def _encode_action(action):
  """-> (kind, values) for the channel, or None (send over the pipe)."""
  if isinstance(action, (bool, np.bool_)):
    return None
  if isinstance(action, (int, np.integer)):
    return 0, [float(action)]
  a = np.asarray(action)
  if a.ndim == 1 and a.size <= 16 and a.dtype.kind in 'iu':
    return 1, a.astype(np.float64).tolist()
  if a.ndim == 1 and a.size <= 16 and a.dtype.kind == 'f':
    return 2, a.astype(np.float64).tolist()
  return None


def _decode_action(kind, values):
  if kind == 0:
    return int(values[0])
  if kind == 1:
    return np.asarray(values, dtype=np.int64)
  return np.asarray(values, dtype=np.float64)


def _encode_instr(instr):
  if instr is None:
    return None
  if isinstance(instr, bytes):
    return b'b' + instr
  return b's' + str(instr).encode('utf-8')


def _decode_instr(raw):
  if raw is None:
    return None
  return raw[1:] if raw[:1] == b'b' else raw[1:].decode('utf-8', 'replace')


def _serve_channel(env, chan, conn, frames, faults, timeout_ms=20):
  """One channel request, if any arrives within timeout_ms: True = served
  (or closed -> 'close'), False = none."""
  seq, method, kind, vals = chan.wait_request(timeout_ms)
  if seq < 0:
    return False
  if method == _M_CLOSE:
    chan.respond(seq, 0, 0.0, False, None)
    return 'close'
  try:
    if method == _M_INITIAL:
      frame, instr = env.initial()
      frames[...] = frame
      chan.respond(seq, 0, 0.0, False, _encode_instr(instr))
    else:
      faults.on_step()
      reward, done, (frame, instr) = env.step(_decode_action(kind, vals))
      frames[...] = frame
      chan.respond(seq, 0, float(reward), bool(done), _encode_instr(instr))
  except Exception as e:  # pylint: disable=broad-except
    try:
      e.remote_traceback = traceback.format_exc()
      conn.send(('error', -1, e))
    except Exception:  # pylint: disable=broad-except
      conn.send(('error', -1, _RemoteError(repr(e))))
    chan.respond(seq, 1, 0.0, False, None)
  return True


def _env_worker(env_ctor, args, kwargs, conn, frame_buf, frame_shape,
                restarted, faults, chan=None):
  env = None
  frames = np.frombuffer(frame_buf, dtype=np.uint8).reshape(frame_shape)
  try:
    env = env_ctor(*args, **kwargs)
    if chan is not None:
      chan.discard_pending()  # a request the dead predecessor never answered
    conn.send(('restarted' if restarted else 'ready', -1, None))
    while True:
      if chan is not None:
        served = _serve_channel(env, chan, conn, frames, faults)
        if served == 'close':
          env.close()
          conn.close()
          return
        if served or not conn.poll(0):
          continue
      msg = conn.recv()
      if msg is None:
        env.close()
        conn.close()
        return
      seq, name, margs = msg
      if name == 'initial':
        frame, instr = env.initial()
        frames[...] = frame
        conn.send(('ok', seq, (instr,)))
      elif name == 'step':
        faults.on_step()
        reward, done, (frame, instr) = env.step(*margs)
        frames[...] = frame
        conn.send(('ok', seq, (float(reward), bool(done), instr)))
      else:
        conn.send(('ok', seq, getattr(env, name)(*margs)))
  except (EOFError, KeyboardInterrupt, BrokenPipeError):
    pass
  except Exception as e:  # pylint: disable=broad-except
    if env is not None:
      try:
        env.close()
      except Exception:  # pylint: disable=broad-except
        pass
    try:
      conn.send(('error', -1, e))
    except Exception:  # pylint: disable=broad-except
      conn.send(('error', -1, _RemoteError(repr(e))))


def _supervisor(env_ctor, args, kwargs, conn, frame_buf, frame_shape, pid_box,
                restarts_box, fault_spec, seed, max_restarts, chan=None):
  import os
  import signal
  signal.signal(signal.SIGINT, signal.SIG_IGN)
  restarts = 0
  while True:
    pid = os.fork()
    if pid == 0:
      code = 0
      try:
        _env_worker(env_ctor, args, kwargs, conn, frame_buf, frame_shape,
                    restarts > 0, _Faults(fault_spec, seed * 7919 + restarts),
                    chan)
      except BaseException:  # pylint: disable=broad-except
        code = 1
      os._exit(code)
    pid_box.value = pid
    _, status = os.waitpid(pid, 0)
    if os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0:
      return  # closed (or the caller went away): done
    restarts += 1
    restarts_box.value = restarts
    if restarts > max_restarts:
      try:
        conn.send(('error', -1, RuntimeError(
            'env worker died %d times; giving up' % restarts)))
      except Exception:  # pylint: disable=broad-except
        pass
      return


def _serve_pipe(env, conn, frames, faults):
  """One pipe message of a grouped env: False when it closed the env."""
  msg = conn.recv()
  if msg is None:
    env.close()
    conn.close()
    return False
  seq, name, margs = msg
  try:
    if name == 'initial':
      frame, instr = env.initial()
      frames[...] = frame
      conn.send(('ok', seq, (instr,)))
    elif name == 'step':
      faults.on_step()
      reward, done, (frame, instr) = env.step(*margs)
      frames[...] = frame
      conn.send(('ok', seq, (float(reward), bool(done), instr)))
    else:
      conn.send(('ok', seq, getattr(env, name)(*margs)))
  except Exception as e:  # pylint: disable=broad-except
    # the other envs of the worker keep running; this one's caller re-raises
    try:
      e.remote_traceback = traceback.format_exc()
      conn.send(('error', seq, e))
    except Exception:  # pylint: disable=broad-except
      conn.send(('error', seq, _RemoteError(repr(e))))
  return True


def _group_worker(specs, conns, bufs, shapes, restarted, faults, chans, bell):
  """k envs in ONE process: every channel request pending at a doorbell
  wake is served in that wake (py_process.start_group)."""
  k = len(specs)
  envs = [None] * k
  frames = [np.frombuffer(b, dtype=np.uint8).reshape(sh)
            for b, sh in zip(bufs, shapes)]
  live = [True] * k
  try:
    for i, (ctor, args, kwargs) in enumerate(specs):
      envs[i] = ctor(*args, **kwargs)
    for ch in chans:
      if ch is not None:
        ch.discard_pending()  # requests the dead predecessor never answered
    for c in conns:
      c.send(('restarted' if restarted else 'ready', -1, None))
    while any(live):
      seen = bell.value if bell is not None else 0
      served = False
      for i in range(k):
        if not live[i]:
          continue
        if chans[i] is not None:
          r = _serve_channel(envs[i], chans[i], conns[i], frames[i], faults, 0)
          if r == 'close':
            envs[i].close()
            conns[i].close()
            live[i] = False
            continue
          served = served or bool(r)
        if conns[i].poll(0):
          served = True
          live[i] = _serve_pipe(envs[i], conns[i], frames[i], faults)
      if not served:
        if bell is not None:
          bell.wait(seen, 20)
        else:
          multiprocessing.connection.wait(
              [c for c, l in zip(conns, live) if l], 0.02)
  except (EOFError, KeyboardInterrupt, BrokenPipeError):
    pass
  except Exception as e:  # pylint: disable=broad-except  (a constructor)
    for i in range(k):
      if envs[i] is not None:
        try:
          envs[i].close()
        except Exception:  # pylint: disable=broad-except
          pass
    for i, c in enumerate(conns):
      if live[i]:
        try:
          c.send(('error', -1, e))
        except Exception:  # pylint: disable=broad-except
          pass


def _group_supervisor(specs, conns, bufs, shapes, pid_box, restarts_box,
                      fault_spec, seed, max_restarts, chans, bell):
  """_supervisor for a group: a worker that dies takes all its envs down;
  the replacement re-creates every one and each caller sees the restart."""
  import os
  import signal
  signal.signal(signal.SIGINT, signal.SIG_IGN)
  restarts = 0
  while True:
    pid = os.fork()
    if pid == 0:
      code = 0
      try:
        _group_worker(specs, conns, bufs, shapes, restarts > 0,
                      _Faults(fault_spec, seed * 7919 + restarts), chans, bell)
      except BaseException:  # pylint: disable=broad-except
        code = 1
      os._exit(code)
    pid_box.value = pid
    _, status = os.waitpid(pid, 0)
    if os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0:
      return
    restarts += 1
    restarts_box.value = restarts
    if restarts > max_restarts:
      for c in conns:
        try:
          c.send(('error', -1, RuntimeError(
              'env worker died %d times; giving up' % restarts)))
        except Exception:  # pylint: disable=broad-except
          pass
      return


def start_group(procs):
  """Starts ONE supervised worker process that hosts every EnvProcess in
  `procs` (unstarted).  Each keeps its own frame buffer, channel slot and
  pipe, so callers use them exactly as separately started ones; the
  channels share a doorbell, so the worker sleeps on one futex and serves
  every pending step per wake: with an actor group stepping all its envs
  at once, k envs cost one wake-up instead of k (the
  reference runs one env per process, /root/reference/py_process.py:123-132).
  A crash or a watchdog kill of the worker restarts all k envs; the
  supervision, hang watchdog and fault injection of the first member apply
  to the group."""
  procs = list(procs)
  head = procs[0]
  bell = None
  if all(p._chan is not None for p in procs):
    try:
      from .runtime import native
      bell = native.EnvDoorbell()
      for p in procs:
        p._chan.attach_doorbell(bell)
    except Exception:  # pylint: disable=broad-except  (no native module)
      bell = None
  pid, restarts = _CTX.RawValue('i', 0), _CTX.RawValue('i', 0)
  pipes = [_CTX.Pipe() for _ in procs]
  group = {'open': len(procs), 'lock': threading.Lock()}
  process = _CTX.Process(
      target=_group_supervisor,
      args=([(p._ctor, p._args, p._kwargs) for p in procs],
            [child for _, child in pipes], [p._buf for p in procs],
            [p._shape for p in procs], pid, restarts, head._fault_spec,
            head._fault_seed, head._max_restarts, [p._chan for p in procs],
            bell), daemon=True)
  process.start()
  for p, (conn, child) in zip(procs, pipes):
    child.close()
    p._conn, p._pid, p._restarts, p._process = conn, pid, restarts, process
    p._group, p._bell = group, bell
  err = None
  for p in procs:
    status, _, payload = p._conn.recv()
    if status == 'error' and err is None:
      err = payload
  if err is not None:
    process.join()
    raise err
  return procs


class EnvProcess(object):
  """Env in a supervised child process; frames cross via shared memory.

  The env must follow the reference protocol: `initial() -> [frame, instr]`,
  `step(action) -> (reward, done, [frame, instr])`.  `timeout` (seconds, 0 =
  none) bounds every call: a worker that does not answer in time is killed
  and replaced (EnvRestartedError).
  """

  def __init__(self, env_ctor, obs_shape, *args, **kwargs):
    self._timeout = float(kwargs.pop('timeout', 0) or 0)
    self._fault_spec = kwargs.pop('fault_inject', '')
    self._fault_seed = int(kwargs.pop('fault_seed', 0))
    self._max_restarts = int(kwargs.pop('max_restarts', 100))
    self._ctor = env_ctor
    self._shape = tuple(obs_shape)
    self._args = args
    self._kwargs = kwargs
    self._buf = _CTX.RawArray('B', int(np.prod(self._shape)))
    self._frames = np.frombuffer(self._buf, dtype=np.uint8).reshape(self._shape)
    self._pid = _CTX.RawValue('i', 0)
    self._restarts = _CTX.RawValue('i', 0)
    self._conn = None
    self._process = None
    self._closed = False
    self._seq = 0
    self._group = None  # start_group: {'open': members not closed, 'lock'}
    self._bell = None
    # initial/step over the native futex channel (created before the fork);
    # the pipe stays for other methods, errors and restart notices
    self._chan = None
    if kwargs.pop('channel', True):
      try:
        from .runtime import native
        self._chan = native.EnvChannel()
      except Exception:  # pylint: disable=broad-except  (no native module)
        self._chan = None

  @property
  def restarts(self):
    return self._restarts.value

  def start(self):
    self._conn, child = _CTX.Pipe()
    self._process = _CTX.Process(
        target=_supervisor,
        args=(self._ctor, self._args, self._kwargs, child, self._buf,
              self._shape, self._pid, self._restarts, self._fault_spec,
              self._fault_seed, self._max_restarts, self._chan), daemon=True)
    self._process.start()
    child.close()
    status, _, payload = self._conn.recv()
    if status == 'error':
      self._process.join()
      raise payload
    return self

  def _kill_worker(self):
    import os
    import signal
    pid = self._pid.value
    if pid > 0:
      try:
        os.kill(pid, signal.SIGKILL)
      except ProcessLookupError:
        pass

  def _rpc(self, name, *args):
    return self._recv(self._send(name, args))

  def _send(self, name, args):
    if self._closed:
      raise OutOfRangeError('env process closed')
    self._seq += 1
    try:
      self._conn.send((self._seq, name, args))
    except (EOFError, OSError):
      raise OutOfRangeError('env process closed')
    return self._seq

  def _recv(self, seq):
    try:
      while True:
        if self._timeout and not self._conn.poll(self._timeout):
          self._kill_worker()  # hung: the supervisor forks a replacement
        status, rseq, payload = self._conn.recv()
        if status == 'restarted':
          raise EnvRestartedError('env worker replaced (restart %d)' %
                                  self._restarts.value)
        if status == 'error':
          raise payload
        if rseq == seq:
          return payload
        # a stale reply to a request issued before a restart: drop it
    except (EOFError, OSError):
      raise OutOfRangeError('env process closed')

  # ---------------------------------------------------- channel calls
  def _chan_send(self, method, action=None):
    if self._closed:
      raise OutOfRangeError('env process closed')
    if method == _M_STEP:
      enc = _encode_action(action)
      if enc is None:
        return None
      kind, vals = enc
    else:
      kind, vals = 0, []
    return ('chan', self._chan.request(method, kind, vals))

  def _chan_recv(self, seq):
    """Waits for the channel response in 50 ms slices, watching the pipe
    for a restart notice / error and enforcing the hang watchdog."""
    import time
    start = time.time()
    try:
      while not self._chan.wait_response(seq, 50):
        if self._conn.poll(0):
          status, _, payload = self._conn.recv()
          if status == 'restarted':
            raise EnvRestartedError('env worker replaced (restart %d)' %
                                    self._restarts.value)
          if status == 'error':
            raise payload
        if self._closed:
          raise OutOfRangeError('env process closed')
        if self._timeout and time.time() - start > self._timeout:
          self._kill_worker()  # hung: the supervisor forks a replacement
          start = time.time()
      # a worker that died BETWEEN requests leaves its restart notice on the
      # pipe while the replacement answers this request on a fresh env that
      # never ran initial(): report the episode boundary here, not on some
      # later step
      while self._chan.status == 0 and self._conn.poll(0):
        status, _, payload = self._conn.recv()
        if status == 'restarted':
          raise EnvRestartedError('env worker replaced (restart %d)' %
                                  self._restarts.value)
        if status == 'error':
          raise payload
      if self._chan.status != 0:  # the exception follows on the pipe
        status, _, payload = self._conn.recv()
        if status == 'restarted':
          raise EnvRestartedError('env worker replaced (restart %d)' %
                                  self._restarts.value)
        raise payload
    except (EOFError, OSError):
      raise OutOfRangeError('env process closed')
    return (self._chan.reward, self._chan.done,
            _decode_instr(self._chan.instr))

  def initial(self):
    return [self._frames.copy(), self.initial_nocopy()]

  def step(self, action):
    reward, done, instr = self.step_recv(self.step_send(action))
    return np.float32(reward), np.bool_(done), [self._frames.copy(), instr]

  # split-phase calls for vectorised actors (runtime/actor_group.py): send
  # the step of every env first, then collect the replies, so the envs of a
  # group step in parallel; the frame is read in place from `frame_view`
  def step_send(self, action):
    if self._chan is not None:
      t = self._chan_send(_M_STEP, action)
      if t is not None:
        return t
    return self._send('step', (action,))

  def step_recv(self, seq):
    """-> (reward, done, instruction); the frame is in `frame_view`."""
    if isinstance(seq, tuple):
      return self._chan_recv(seq[1])
    reward, done, instr = self._recv(seq)
    return reward, done, instr

  def initial_nocopy(self):
    if self._chan is not None:
      return self._chan_recv(self._chan_send(_M_INITIAL)[1])[2]
    (instr,) = self._rpc('initial')
    return instr

  @property
  def frame_view(self):
    """The shared-memory frame of the last initial()/step() (overwritten by
    the next call)."""
    return self._frames

  def close(self):
    if self._closed or self._process is None:
      self._closed = True
      return
    self._closed = True
    try:
      self._conn.send(None)
    except (OSError, BrokenPipeError):
      pass
    if self._group is not None:
      with self._group['lock']:
        self._group['open'] -= 1
        if self._group['open'] > 0:
          return  # the worker keeps serving the group's other envs
    self._process.join(timeout=30)
    if self._process.is_alive():
      self._kill_worker()
      self._process.terminate()
      self._process.join()

  @property
  def is_alive(self):
    return self._process is not None and self._process.is_alive()
