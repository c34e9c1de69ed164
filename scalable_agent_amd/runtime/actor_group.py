"""Vectorised actor groups in their own processes (--actor_groups=G).

The reference runs every actor as a TF thread of the learner process
(experiment.py:534-546: one env per actor, per-step `dynamic_batching`
inference, experiment.py:240-321 for the unroll loop); the threads share
one interpreter, so with tens of actors the learner's own host work waits on
the GIL.  Here the `num_actors` envs are split over G group processes, each
forked before the learner initialises the GPU:

  group g:  M = num_actors / G envs (EnvProcess children, stepped in
            parallel: every env's step is sent before any reply is read)
            one VectorInfer: a pinned [M] input slab -> one H2D -> one
            captured hipGraph (torso/core/heads/sampler, LSTM state resident
            on the device) -> one D2H of the packed outputs
            writes every step of every env straight into its claimed column
            of the learner's time-major TrajectoryQueue slab
  learner:  consumes full slabs (experiment._TrajFeeder), publishes weights
            into a SharedWeights seqlock region with ONE async D2H copy per
            step; groups pick a new version up with an async H2D copy into a
            staging buffer, validated by the seqlock before it becomes the
            inference snapshot (never a torn snapshot).

Each env's unroll keeps the reference's layout: element 0 repeats the last
element of the previous unroll, the recorded agent state is the state at the
start of the unroll.  An env worker that dies mid-unroll is replaced and its
column continues from the new episode's first frame with done=True (the
learner's V-trace and the LSTM reset treat it as an episode boundary).
"""

import logging
import mmap
import os
import time

import numpy as np

log = logging.getLogger('scalable_agent_amd')


class SharedWeights(object):
  """fp32 parameter snapshots in an anonymous shared mapping (inherited by
  forked groups): TWO buffers, each with its own seqlock count (odd = being
  written), plus `latest` (the buffer of the newest complete snapshot) and
  `version` (number of completed publishes; 0 = none yet).

  Learner: `publish(flat_params)` enqueues ONE async D2H copy, ordered after
  the learner's stream, into the buffer that is NOT `latest`, straight from
  the device into the (hipHostRegister-ed) mapping; the next publish (or
  `flush()`) that finds the copy landed flips `latest` to it.  A publish
  while the previous copy is still in flight is skipped (the groups take the
  next one), so `latest` always names a complete snapshot and readers never
  wait on the learner's GPU work.
  Group: ActorGroupWorker._sync_weights (copy `latest`, then re-check its
  seqlock count: a torn copy is discarded)."""

  HDR = 4096
  MAGIC = 0x5341574549474854

  def __init__(self, name, numel=0, create=False):
    """name: a POSIX shm name ('/...'); the learner creates it once it
    knows the parameter count, the groups (forked earlier) attach to it."""
    self.name = name
    self._path = '/dev/shm' + name
    self._owner = create
    if create:
      fd = os.open(self._path, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o600)
      os.ftruncate(fd, self.HDR + 8 * int(numel))
    else:
      fd = os.open(self._path, os.O_RDWR)
    size = os.fstat(fd).st_size
    self._mm = mmap.mmap(fd, size)
    os.close(fd)
    self.numel = (size - self.HDR) // 8
    # [0] latest buffer (-1 none), [1] version, [2:4] per-buffer seqlock,
    # [4] magic (written last by the creator)
    self._hdr = np.frombuffer(self._mm, dtype=np.int64, count=5)
    if create:
      self._hdr[0] = -1
      self._hdr[4] = self.MAGIC
    self._all = np.frombuffer(self._mm, dtype=np.float32,
                              count=2 * self.numel, offset=self.HDR)
    self.data = [self._all[:self.numel], self._all[self.numel:]]
    self._pinned = False
    self._tensors = None
    self._pending = None
    self._stream = None
    self._snap = None
    self.skipped = 0

  # --------------------------------------------------------------- both
  def version(self):
    return int(self._hdr[1])

  def latest(self):
    return int(self._hdr[0])

  def seq(self, b):
    return int(self._hdr[2 + b])

  def tensors(self, device):
    """Torch views of the two buffers (host-registered on a GPU device)."""
    import torch
    from .traj_queue import _hip_host_register
    if self._tensors is None:
      if device.type == 'cuda':
        self._pinned = _hip_host_register(self._all.ctypes.data,
                                          8 * self.numel)
      self._tensors = [torch.from_numpy(d) for d in self.data]
    return self._tensors

  # --------------------------------------------------------------- learner
  def _finish(self, block):
    if self._pending is None:
      return True
    b, ev = self._pending
    if not block and not ev.query():
      return False
    ev.synchronize()
    self._pending = None
    self._hdr[2 + b] += 1  # even: complete
    self._hdr[0] = b
    self._hdr[1] += 1
    return True

  def _target(self):
    b = 1 - self.latest() if self.latest() >= 0 else 0
    self._hdr[2 + b] += 1  # odd: being written
    return b

  def publish(self, flat_params):
    import torch
    if not flat_params.is_cuda:
      b = self._target()
      self.data[b][...] = flat_params.detach().numpy()
      self._pending = (b, _Done())
      self._finish(block=True)
      return True
    if not self._finish(block=False):
      self.skipped += 1
      return False
    host = self.tensors(flat_params.device)
    if self._stream is None:
      self._stream = torch.cuda.Stream(flat_params.device)
    # the D2H reads a device-side snapshot taken on the learner's stream (a
    # few us of HBM copy), never flat_params itself: the next optimizer step
    # may overwrite the parameters while the slow D2H is still in flight.
    # The snapshot is only rewritten after the previous D2H completed
    # (_finish above), so it is never torn either.
    cur = torch.cuda.current_stream(flat_params.device)
    if self._snap is None or self._snap.shape != flat_params.shape:
      self._snap = torch.empty_like(flat_params.detach())
    self._snap.copy_(flat_params.detach())
    self._stream.wait_stream(cur)
    b = self._target()
    with torch.cuda.stream(self._stream):
      host[b].copy_(self._snap, non_blocking=self._pinned)
      ev = torch.cuda.Event()
      ev.record(self._stream)
    self._pending = (b, ev)
    return True

  def flush(self):
    self._finish(block=True)

  @classmethod
  def attach(cls, name, alive, timeout_s=600):
    """Group side: wait until the learner created `name` (alive() False or
    the timeout -> None)."""
    deadline = time.time() + timeout_s
    while alive() and time.time() < deadline:
      try:
        w = cls(name)
        if w.numel > 0 and int(w._hdr[4]) == cls.MAGIC:
          return w
        w.close()
      except (OSError, ValueError):
        pass
      time.sleep(0.01)
    return None

  def close(self):
    self.flush() if self._owner else None
    self._tensors = None
    self.data = self._all = self._hdr = None
    try:
      self._mm.close()
    except BufferError:
      pass  # views still referenced elsewhere; the mapping dies with them
    if self._owner:
      try:
        os.unlink(self._path)
      except OSError:
        pass

  # --------------------------------------------------------------- group
  def read_into(self, out):
    """Host reader: consistent copy of the latest snapshot -> version."""
    while True:
      v, b = self.version(), self.latest()
      if b < 0:
        return 0
      s = self.seq(b)
      if s & 1:
        continue
      out[...] = self.data[b]
      if self.seq(b) == s:
        return v


class _Done(object):
  def query(self):
    return True

  def synchronize(self):
    pass


def board_geometry(num_actors, groups, splits, lanes=1):
  """(slots, rows per slot) of each inference board for this actor layout:
  group g posts to board g % lanes, slots from (g // lanes) * splits."""
  parts = split_actors(num_actors, groups)
  splits = max(1, int(splits))
  rows = max(max(len(p) for p in split_actors(len(g), min(splits, len(g))))
             for g in parts)
  lanes = max(1, min(int(lanes), len(parts)))
  return -(-len(parts) // lanes) * splits, rows


def split_actors(num_actors, groups):
  """Actor indices per group: contiguous, sizes differ by at most one."""
  groups = max(1, min(int(groups), int(num_actors)))
  base, extra = divmod(int(num_actors), groups)
  out, start = [], 0
  for g in range(groups):
    n = base + (1 if g < extra else 0)
    out.append(list(range(start, start + n)))
    start += n
  return out


class ActorGroupWorker(object):
  """Body of one group process (see the module docstring)."""

  def __init__(self, gid, spec, tq, weights, counters, device_str):
    self.gid = gid
    self.spec = spec
    self.tq = tq
    self.weights = weights
    self.counters = counters
    self.device_str = device_str
    self.restarts = 0
    self.board_mode = False

  def run(self):
    import torch
    from .. import py_process
    from ..actor import encode_instruction
    from ..experiment import _make_agent, create_environment
    from ..inference import InferenceModel, VectorInfer

    sp = self.spec
    flags = sp['flags']
    envs = [create_environment(flags, lvl, seed)
            for lvl, seed in zip(sp['levels'], sp['seeds'])]
    # forked before this process touches the GPU
    py_process.start_all(envs, per_worker=getattr(flags, 'envs_per_worker', 1))
    board = sp.get('board')
    if board is not None:
      # CPU-only group: inference is served from the learner process
      from .inference_board import BoardClient
      parent = os.getppid()
      alive = lambda: os.getppid() == parent
      K = max(1, min(int(sp['splits']), len(envs)))
      vis = [BoardClient(board, sp['slot0'] + k, len(part), alive)
             for k, part in enumerate(split_actors(len(envs), K))]
      self.board_mode = True
      try:
        self._loop(envs, None, vis, encode_instruction, py_process)
      except EOFError:
        pass  # the learner closed the board: shutting down
      finally:
        py_process.close_all(envs)
      return
    try:
      device = torch.device(self.device_str)
      if device.type == 'cuda':
        torch.cuda.set_device(device)
      agent = _make_agent(flags, sp['num_actions'], sp['frame_shape'], device,
                          flags.seed, dtype=sp['dtype'])
      model = InferenceModel(agent, device, sp['use_instr'],
                             seed=flags.seed + 7919 * (self.gid + 1))
      K = max(1, min(int(sp['splits']), len(envs)))
      vis = [VectorInfer(model, len(part), sp['frame_shape'],
                         sp['num_actions'])
             for part in split_actors(len(envs), K)]
      parent = os.getppid()
      self.weights = SharedWeights.attach(
          self.weights, lambda: os.getppid() == parent and not self.tq.closed)
      if self.weights is None:
        return
      self._loop(envs, model, vis, encode_instruction, py_process)
    finally:
      py_process.close_all(envs)

  # ------------------------------------------------------------ weights
  def _sync_weights(self, model, state):
    """Non-blocking fetch of a newer snapshot: an async H2D of the `latest`
    buffer into a staging buffer; once it has landed and that buffer's
    seqlock count is unchanged, a D2D copy (ordered before the next
    inference) makes it the inference snapshot."""
    if self.board_mode:
      state['version'] = max(1, state['version'])  # weights live in the server
      return
    import torch
    w = self.weights
    v = w.version()
    if model.device.type != 'cuda':
      if v and v != state['version']:
        host = np.empty(w.numel, np.float32)
        state['version'] = w.read_into(host)
        model.flat.params.copy_(torch.from_numpy(host))
        model._refresh_cache()
      return
    if state.get('inflight') is not None:
      v, b, s, ev = state['inflight']
      if not ev.query():
        return
      state['inflight'] = None
      if w.seq(b) == s:  # not overwritten while the copy ran
        with torch.cuda.stream(model.stream):
          model.flat.params.copy_(state['staging'], non_blocking=True)
          model._refresh_cache()
        state['version'] = v
      return
    if v == 0 or v == state['version']:
      return
    b = w.latest()
    s = w.seq(b)
    if s & 1:
      return
    if state.get('staging') is None:
      state['staging'] = torch.empty(w.numel, dtype=torch.float32,
                                     device=model.device)
      state['copy_stream'] = torch.cuda.Stream(model.device)
    host = w.tensors(model.device)
    cs = state['copy_stream']
    # the previous D2D out of the staging buffer must be done first
    cs.wait_stream(model.stream)
    with torch.cuda.stream(cs):
      state['staging'].copy_(host[b], non_blocking=w._pinned)
      ev = torch.cuda.Event()
      ev.record(cs)
    state['inflight'] = (v, b, s, ev)

  # ------------------------------------------------------------ loop
  def _loop(self, envs, model, vis, encode_instruction, py_process):
    """K splits of the group's envs, each with its own VectorInfer, run as a
    pipeline: while split k's inference runs on the GPU, the host steps the
    envs of the split whose inference just finished (their env processes
    step in parallel), so neither the GPU latency nor the env latency is
    exposed once per step of the group."""
    K = len(vis)
    sizes = [vi.rows for vi in vis]
    offs = np.cumsum([0] + sizes)
    splits = [_Split(self, envs[offs[k]:offs[k + 1]], vis[k],
                     self.spec['level_index'][offs[k]:offs[k + 1]],
                     encode_instruction, py_process) for k in range(K)]
    wstate = {'version': -1}
    parent = os.getppid()
    # measurement only (SA_MEASURE_KNOBS=1 SA_GROUP_PROFILE=1): where a
    # group's time goes, logged every 2 s (profiles/r6_e2e.md)
    from ..utils.knobs import measure_env
    prof = ({'wait': 0.0, 'env': 0.0, 'record': 0.0, 'launch': 0.0,
             'idle': 0.0, 'steps': 0, 't0': time.perf_counter()}
            if measure_env('SA_GROUP_PROFILE') == '1' else None)
    for sp in splits:
      sp.prof = prof
    # the first snapshot (e.g. a restored checkpoint) before any inference
    while wstate['version'] <= 0:
      if os.getppid() != parent or self.tq.closed:
        return
      self._sync_weights(model, wstate)
      time.sleep(0.002)
    # a split is either waiting for its columns (all-or-nothing claims: a
    # split never holds columns while it waits, so slabs always fill) or has
    # one inference in flight
    pending = list(splits)
    last_check = time.time()
    while True:
      progressed = False
      for sp in splits:
        if sp in pending:
          got = sp.try_begin_unroll()
          if got == -2:
            return
          if not got:
            continue
          pending.remove(sp)
          self._sync_weights(model, wstate)
          sp.launch()
          progressed = True
          continue
        sp.finish_step()  # wait for its inference, step its envs, record
        progressed = True
        if sp.t == sp.T:
          sp.commit()
          pending.append(sp)
          continue
        self._sync_weights(model, wstate)
        sp.launch()
      if not progressed:
        if prof is not None:
          t_idle = time.perf_counter()
        time.sleep(0.0002)  # every split waits for queue room
        if prof is not None:
          prof['idle'] += time.perf_counter() - t_idle
      if prof is not None and time.perf_counter() - prof['t0'] > 2.0:
        dt = time.perf_counter() - prof['t0']
        n = max(1, prof['steps'])
        log.info('group %d profile: %d split steps/s; per split step: '
                 'inference wait %.0f us, env step %.0f us, record %.0f us, '
                 'launch %.0f us; idle %.0f %%', self.gid, n / dt,
                 1e6 * prof['wait'] / n, 1e6 * prof['env'] / n,
                 1e6 * prof['record'] / n, 1e6 * prof['launch'] / n,
                 100 * prof['idle'] / dt)
        for k in ('wait', 'env', 'record', 'launch', 'idle'):
          prof[k] = 0.0
        prof['steps'] = 0
        prof['t0'] = time.perf_counter()
      if time.time() - last_check > 1.0:
        last_check = time.time()
        if os.getppid() != parent or self.tq.closed:
          return  # the learner went away / closed the queue


class _Split(object):
  """One pipeline stage of a group: its envs, their per-env bookkeeping
  (FlowEnvironment semantics) and their claimed trajectory-queue columns."""

  def __init__(self, worker, envs, vi, level_index, encode_instruction,
               py_process):
    sp = worker.spec
    self.w = worker
    self.envs = envs
    self.vi = vi
    self.level_index = level_index
    self.encode = encode_instruction
    self.pp = py_process
    self.T = sp['unroll_length']
    self.action_set = sp['action_set']
    self.use_instr = sp['use_instr']
    M = len(envs)
    self.reward = np.zeros(M, np.float32)
    self.done = np.ones(M, np.bool_)
    self.ep_ret = np.zeros(M, np.float32)
    self.ep_step = np.zeros(M, np.int32)
    self.run_ret = np.zeros(M, np.float32)
    self.run_step = np.zeros(M, np.int32)
    self.action = np.zeros(M, np.int64)
    self.logits = np.zeros((M, sp['num_actions']), np.float32)
    self.baseline = np.zeros(M, np.float32)
    self.c = np.zeros((M, vi.c.shape[1]), np.float32)
    self.h = np.zeros((M, vi.h.shape[1]), np.float32)
    self.instr = [env.initial_nocopy() for env in envs]
    self.cols = []
    self.t = 0
    self.prof = None  # _loop's measurement dict (SA_GROUP_PROFILE)

  def try_begin_unroll(self):
    """Claims one column per env at once (or none): True when claimed
    (element 0 = the previous unroll's last element, and the agent state at
    the unroll start, are written), False if the queue has no room yet, -2
    when it is closed."""
    got = self.w.tq.claim_n(len(self.envs), timeout_ms=0)
    if got == -2:
      return -2
    if got == -1:
      return False
    self.cols = got
    for i, (s, col, v) in enumerate(got):
      v['level'][col] = self.level_index[i]
      v['c'][col] = self.c[i]
      v['h'][col] = self.h[i]
    self.t = 0
    self._record(0)
    return True

  def commit(self):
    for s, col, v in self.cols:
      self.w.tq.commit(s)
    self.cols = []

  def _record(self, t):
    use_instr = self.use_instr
    for i, (s, col, v) in enumerate(self.cols):
      v['frame'][t, col] = self.envs[i].frame_view
      v['reward'][t, col] = self.reward[i]
      v['done'][t, col] = self.done[i]
      v['episode_return'][t, col] = self.ep_ret[i]
      v['episode_step'][t, col] = self.ep_step[i]
      v['action'][t, col] = self.action[i]
      v['policy_logits'][t, col] = self.logits[i]
      v['baseline'][t, col] = self.baseline[i]
      if use_instr and 'instr_ids' in v:
        v['instr_ids'][t, col], v['instr_len'][t, col] = self.encode(
            self.instr[i])

  def launch(self):
    t0 = time.perf_counter() if self.prof is not None else 0.0
    self._launch()
    if self.prof is not None:
      self.prof['launch'] += time.perf_counter() - t0

  def _launch(self):
    inp = self.vi.inputs
    inp['last_action'][:] = self.action
    inp['reward'][:] = self.reward
    inp['done'][:] = self.done
    for i, env in enumerate(self.envs):
      inp['frame'][i] = env.frame_view
      if self.use_instr:
        inp['instr_ids'][i], inp['instr_len'][i] = self.encode(self.instr[i])
    self.vi.launch()

  def finish_step(self):
    prof = self.prof
    t0 = time.perf_counter() if prof is not None else 0.0
    pp = self.pp
    a, lg, b, c2, h2 = self.vi.wait()
    if prof is not None:
      t1 = time.perf_counter()
      prof['wait'] += t1 - t0
    self.action[:] = a
    self.logits[:] = lg
    self.baseline[:] = b
    self.c[:] = c2
    self.h[:] = h2
    envs = self.envs
    seqs = [None] * len(envs)
    for i, env in enumerate(envs):
      try:
        seqs[i] = env.step_send(self.action_set[int(a[i])])
      except pp.EnvRestartedError:
        seqs[i] = None
    for i, env in enumerate(envs):
      try:
        if seqs[i] is None:
          raise pp.EnvRestartedError('send failed')
        r, d, self.instr[i] = env.step_recv(seqs[i])
      except pp.EnvRestartedError as e:
        w = self.w
        w.restarts += 1
        w.counters[w.gid] = w.restarts
        log.warning('actor group %d: %s; episode truncated (the column '
                    'continues from a fresh episode)', w.gid, e)
        self.instr[i] = env.initial_nocopy()
        r, d = 0.0, True
      self.reward[i] = r
      self.done[i] = d
      self.run_ret[i] += r
      self.run_step[i] += 1
      self.ep_ret[i] = self.run_ret[i]
      self.ep_step[i] = self.run_step[i]
      if d:
        self.run_ret[i] = 0.0
        self.run_step[i] = 0
    if prof is not None:
      t2 = time.perf_counter()
      prof['env'] += t2 - t1
    self.t += 1
    self._record(self.t)
    if prof is not None:
      prof['record'] += time.perf_counter() - t2
      prof['steps'] += 1


def _group_main(gid, spec, tq, weights, counters, device_str):
  import faulthandler
  import signal
  faulthandler.enable()
  signal.signal(signal.SIGINT, signal.SIG_IGN)
  logging.basicConfig(level=logging.INFO,
                      format='[%(asctime)s %(levelname)s group%(gid)s] '
                             '%(message)s'.replace('%(gid)s', str(gid)))
  try:
    ActorGroupWorker(gid, spec, tq, weights, counters, device_str).run()
  except Exception:  # pylint: disable=broad-except
    log.exception('actor group %d failed', gid)
    os._exit(3)
  os._exit(0)


class ActorGroups(object):
  """Learner-side handle: forks the groups (call BEFORE the learner process
  initialises the GPU), liveness checks, shutdown."""

  def __init__(self, flags, level_names, actor_levels, actor_seeds, tq,
               weights, frame_shape, action_set, use_instr, device_str,
               dtype, board=None):
    """board: None (GPU groups), one InferenceBoard, or a list of them (one
    per lane: group g posts to board g % len(list), board_geometry)."""
    import multiprocessing
    boards = (None if board is None else
              list(board) if isinstance(board, (list, tuple)) else [board])
    ctx = multiprocessing.get_context('fork')
    self.tq = tq
    self.counters = ctx.RawArray('q', max(1, flags.actor_groups))
    self.procs = []
    index = {l: i for i, l in enumerate(level_names)}
    for gid, members in enumerate(split_actors(flags.num_actors,
                                               flags.actor_groups)):
      spec = dict(flags=flags, levels=[actor_levels[i] for i in members],
                  seeds=[actor_seeds[i] for i in members],
                  level_index=[index[actor_levels[i]] for i in members],
                  num_actions=len(action_set), action_set=action_set,
                  frame_shape=tuple(frame_shape), use_instr=use_instr,
                  unroll_length=flags.unroll_length, dtype=dtype,
                  splits=flags.actor_group_splits,
                  board=boards[gid % len(boards)] if boards else None,
                  slot0=(gid // len(boards) if boards else gid) *
                  max(1, flags.actor_group_splits))
      p = ctx.Process(target=_group_main,
                      args=(gid, spec, tq, weights, self.counters, device_str),
                      daemon=False, name='actor-group-%d' % gid)
      p.start()
      self.procs.append(p)

  @property
  def env_restarts(self):
    return int(sum(self.counters))

  def check(self):
    for p in self.procs:
      if p.exitcode is not None:
        raise RuntimeError('actor group %s exited with code %s' %
                           (p.name, p.exitcode))

  def close(self, timeout=30):
    self.tq.close()
    deadline = time.time() + timeout
    for p in self.procs:
      p.join(max(0.1, deadline - time.time()))
      if p.is_alive():
        p.terminate()
        p.join(5)
