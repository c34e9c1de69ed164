"""Batched actor inference served from the learner process over shared memory.

Actor-group processes (runtime/actor_group.py) can either run their own
inference on the GPU (a second GPU context per group) or, with
`--inference_server`, stay CPU-only and post their rows to this board:

  board (anonymous MAP_SHARED, created before the groups are forked):
    header  : seq word (bumped on every request, the server's futex), closed
              flag, per-slot state words (0 idle, 1 request, 2 response) and
              per-slot row counts
    inputs  : every input field for ALL rows (slot s owns rows [s*M, s*M+M)),
              field-major - ONE H2D copy moves the whole board to the device,
              the server's row mask (row_mask, written by the server only)
              included
    outputs : slot-major [action | logits | baseline | c | h] per slot, so a
              slot's response is ONE D2H copy and responding to one slot
              never overwrites the rows another worker is still reading
  server (a thread in the learner process, one GPU context in total):
    wait for request slots -> mask of their rows -> H2D inputs + mask ->
    ONE captured graph over all rows (torso, core, heads + Gumbel sampler; the
    LSTM state of every row resident on the device, updated only where the
    mask is set) -> the masked rows' outputs -> state 2 + futex wake.  On a
    GPU the graph's epilogue writes those rows straight into the registered
    host board (no D2H copy per slot); elsewhere they are copied back.
    On a GPU with the HIP backend the loop is a C++ thread
    (csrc/board_server.cpp, no Python and no GIL per batch); the graphs are
    captured here first.  SA_BOARD_NATIVE=0 keeps the Python thread.  With
    depth=2 the C++ loop keeps two batches in flight over two buffer sets
    (the next batch's H2D and host work under the current batch's graph).

Replaces the reference's per-request dynamic batching (experiment.py:534-546
+ batcher.cc) for process actors: the "batch" is every slot that is ready
when the server looks, the batch shape is fixed (no padding buckets).
"""

import logging
import mmap
import os
import threading
import time

import numpy as np

from . import native

log = logging.getLogger('scalable_agent_amd')

_ALIGN = 256
IDLE, REQUEST, RESPONSE = 0, 1, 2


def _align(x):
  return (x + _ALIGN - 1) // _ALIGN * _ALIGN


class InferenceBoard(object):
  """The shared request/response board (see the module docstring)."""

  HDR = 4096

  def __init__(self, num_slots, rows, frame_shape, num_actions, instr_len=16,
               core_size=256):
    self.S, self.M = int(num_slots), int(rows)
    assert 0 < self.S <= 250
    R = self.R = self.S * self.M
    self.num_actions, self.core = int(num_actions), int(core_size)
    fields = [('last_action', (), np.int64), ('reward', (), np.float32),
              ('done', (), np.bool_), ('frame', tuple(frame_shape), np.uint8),
              ('instr_ids', (int(instr_len),), np.int64),
              ('instr_len', (), np.int64),
              ('row_mask', (), np.float32)]  # written by the server only
    self.in_fields, off = [], 0
    for name, shape, dt in fields:
      nb = R * int(np.prod(shape, dtype=np.int64)) * np.dtype(dt).itemsize
      self.in_fields.append((name, (R,) + tuple(shape), np.dtype(dt), off, nb))
      off = _align(off + nb)
    self.in_bytes = off
    outs = [('action', (), np.int64), ('logits', (num_actions,), np.float32),
            ('baseline', (), np.float32), ('c', (core_size,), np.float32),
            ('h', (core_size,), np.float32)]
    self.out_fields, off = [], 0
    for name, shape, dt in outs:
      nb = self.M * int(np.prod(shape, dtype=np.int64)) * np.dtype(dt).itemsize
      self.out_fields.append((name, (self.M,) + tuple(shape), np.dtype(dt), off,
                              nb))
      off = _align(off + nb)
    self.slot_out_bytes = off
    self.out_bytes = off * self.S
    self.nbytes = self.HDR + self.in_bytes + self.out_bytes
    self._mm = mmap.mmap(-1, self.nbytes)
    self.buf = np.frombuffer(self._mm, dtype=np.uint8)
    self.base = self.buf.ctypes.data
    self.words = self.buf[:self.HDR].view(np.uint32)
    # words[0] seq, [1] closed, [16 + s] state, [16 + S + s] rows of slot s
    self.seq_addr = self.base
    self.inputs = {n: self.buf[self.HDR + o:self.HDR + o + nb].view(dt).reshape(s)
                   for n, s, dt, o, nb in self.in_fields}

  # -------------------------------------------------------------- words
  def state_addr(self, slot):
    return self.base + 4 * (16 + slot)

  def state(self, slot):
    return int(self.words[16 + slot])

  def set_rows(self, slot, n):
    self.words[16 + self.S + slot] = int(n)

  def rows_of(self, slot):
    return int(self.words[16 + self.S + slot])

  @property
  def closed(self):
    return bool(self.words[1])

  def close(self):
    self.words[1] = 1
    native.futex_wake(self.seq_addr)
    for s in range(self.S):
      native.futex_wake(self.state_addr(s))

  def slot_outputs(self, slot):
    """numpy views of slot's outputs (action, logits, baseline, c, h)."""
    o0 = self.HDR + self.in_bytes + slot * self.slot_out_bytes
    return tuple(self.buf[o0 + o:o0 + o + nb].view(dt).reshape(s)
                 for n, s, dt, o, nb in self.out_fields)


class BoardClient(object):
  """Worker side of one board slot, with VectorInfer's interface (inputs /
  launch / wait / rows / c / h) so the actor-group pipeline drives either."""

  def __init__(self, board, slot, rows, alive=None):
    assert rows <= board.M
    self.board, self.slot, self.rows = board, int(slot), int(rows)
    lo, hi = slot * board.M, slot * board.M + rows
    self.inputs = {n: v[lo:hi] for n, v in board.inputs.items()}
    self._outs = tuple(o[:rows] for o in board.slot_outputs(slot))
    self.c, self.h = self._outs[3], self._outs[4]
    self._alive = alive or (lambda: True)
    board.set_rows(slot, rows)

  def launch(self):
    b = self.board
    native.atomic_store_u32(b.state_addr(self.slot), REQUEST)
    native.atomic_add_u32(b.seq_addr, 1)
    native.futex_wake(b.seq_addr)

  def wait(self):
    b = self.board
    addr = b.state_addr(self.slot)
    while native.atomic_load_u32(addr) != RESPONSE:
      if b.closed or not self._alive():
        raise EOFError('inference board closed')
      native.futex_wait(addr, REQUEST, 50)
    return self._outs


class BoardServer(object):
  """Learner-process side: one captured inference graph over the board."""

  def __init__(self, model, board, use_graph=True, gather_us=0,
               min_ready=None, depth=1):
    import torch
    self.torch = torch
    self.model, self.board = model, board
    # native loop's batching window (NativeBoardServer.set_batching): launch
    # once min_ready slots (default half the board) are ready or gather_us
    # after the first
    self.gather_us = int(gather_us)
    self.min_ready = (max(1, board.S // 2) if min_ready is None
                      else int(min_ready))
    # batches in flight in the native loop (1 or 2; the Python loop is 1).
    # Depth 2 measured slower end to end (profiles/r6_e2e.md): every launch
    # runs the graph over the whole board, so launching earlier only makes
    # the batches smaller
    self.depth = int(depth)
    assert self.depth in (1, 2)
    dev = model.device
    self.cuda = dev.type == 'cuda'
    self.use_graph = bool(use_graph) and self.cuda
    b = board
    # the board's input + output regions as host tensors (pinned on a GPU)
    self._host_in = torch.from_numpy(b.buf[b.HDR:b.HDR + b.in_bytes])
    self._host_out = torch.from_numpy(b.buf[b.HDR + b.in_bytes:])
    self.pinned = False
    if self.cuda:
      from .traj_queue import _hip_host_register
      torch.cuda.init()
      self.pinned = _hip_host_register(b.base + b.HDR, b.in_bytes + b.out_bytes)
    self.c = torch.zeros(b.R, b.core, device=dev)
    self.h = torch.zeros(b.R, b.core, device=dev)
    # direct output: the graph's epilogue packs the ready rows into the
    # registered host board itself (HIP backend on a GPU)
    self._out_addr = 0
    if self.pinned and getattr(model.agent, 'backend', '') == 'hip':
      from .traj_queue import _hip_host_device_ptr
      d = _hip_host_device_ptr(b.base + b.HDR)  # the registration's start
      self._out_addr = d + b.in_bytes if d else 0
    # buffer set 0 (set 1 is allocated by the depth-2 native loop)
    self._sets = [self._buffers(0)]
    (self.in_dev, self.out_dev, self.mask_dev, self.mask_host,
     self._dev_in) = self._sets[0]
    # graphs: has_instr -> graph over set 0, (1, has_instr) -> over set 1
    self._graphs = {}
    self._thread = None
    self._native = None
    self._stop = False
    self.error = None
    self._batches = 0
    self._rows = 0

  @property
  def direct_out(self):
    """True when the graph writes the responses into the host board."""
    return self._out_addr != 0

  def _buffers(self, k):
    """Buffer set k: device inputs, outputs, row mask (device view inside
    the inputs + host) and the typed views of the inputs.  Set 0's host mask
    is the board's own row_mask field, so the input H2D carries it; set 1
    (depth 2) has a pinned mask of its own, copied after its inputs."""
    torch, b, dev = self.torch, self.board, self.model.device
    # zero-filled: the capture's warm-up steps read the board before any
    # worker wrote it (and a zero mask packs no rows)
    in_dev = torch.zeros(b.in_bytes, dtype=torch.uint8, device=dev)
    out_dev = torch.zeros(b.out_bytes, dtype=torch.uint8, device=dev)
    tdt = lambda dt: torch.from_numpy(np.empty(0, dt)).dtype
    dev_in = [in_dev[o:o + nb].view(tdt(dt)).view(*s)
              for n, s, dt, o, nb in b.in_fields]
    mask_dev = dev_in[-1].view(b.R, 1)
    if k == 0:
      mask_host = torch.from_numpy(b.inputs['row_mask'])
    else:
      mask_host = torch.zeros(b.R, dtype=torch.float32)
      if self.cuda:
        mask_host = mask_host.pin_memory()
    return in_dev, out_dev, mask_dev, mask_host, dev_in[:-1]

  @property
  def batches(self):
    return self._batches + (self._native.batches() if self._native else 0)

  @property
  def rows_served(self):
    return self._rows + (self._native.rows_served() if self._native else 0)

  @property
  def native(self):
    """True when the serving loop is the C++ thread."""
    return self._native is not None

  def _epilogue_ext(self):
    """The HIP extension when the fused board epilogue applies (HIP
    backend on a GPU), else None (torch ops: CPU boards, the torch
    backend)."""
    if not self.cuda or getattr(self.model.agent, 'backend', '') != 'hip':
      return None
    from .. import ops
    return ops.ext()

  def _body(self, has_instr, k=0):
    torch = self.torch
    b = self.board
    _, out_dev, mask_dev, _, dev_in = self._sets[k]
    la, rw, dn, fr, ids, ln = dev_in
    action, logits, baseline, c2, h2 = self.model.step_device(
        la, rw, dn, fr, ids, ln, self.c, self.h, has_instr=has_instr)
    C = self._epilogue_ext()
    if C is not None:
      # ONE launch for the masked state update and the slot-major output
      # packing (the torch form below is 12 dependent launches, ~57 us of
      # every board launch: tools/micro/board_trace.py)
      C.board_epilogue([action, logits, baseline, c2, h2],
                       [o for _, _, _, o, _ in b.out_fields], out_dev,
                       b.M, b.slot_out_bytes, mask_dev, c2, h2, self.c,
                       self.h, out_addr=self._out_addr)
      return
    m = mask_dev
    self.c.copy_(torch.where(m > 0, c2, self.c))
    self.h.copy_(torch.where(m > 0, h2, self.h))
    out = out_dev.view(b.S, b.slot_out_bytes)
    for (n, s, dt, o, nb), v in zip(b.out_fields,
                                    (action, logits, baseline, c2, h2)):
      per = nb // b.M  # bytes per row
      src = v.reshape(b.S, b.M, -1).contiguous().view(torch.uint8).view(
          b.S, b.M * per)
      out[:, o:o + b.M * per].copy_(src)

  def _capture(self, has_instr, k=0):
    torch = self.torch
    s = self.model.stream
    with torch.cuda.stream(s):
      c0, h0 = self.c.clone(), self.h.clone()
      for _ in range(2):
        self._body(has_instr, k)
      self.c.copy_(c0)
      self.h.copy_(h0)
      s.synchronize()
      g = torch.cuda.CUDAGraph()
      with torch.cuda.graph(g, stream=s, capture_error_mode='thread_local'):
        self._body(has_instr, k)
    return g

  def prepare(self, has_instr=False):
    """Captures the graph before any traffic (main thread)."""
    if self.use_graph:
      with self.torch.no_grad():
        self._graphs[has_instr] = self._capture(has_instr)

  def serve_once(self, timeout_ms=50):
    """One batch over every slot in REQUEST state; False when none came."""
    torch = self.torch
    b, m = self.board, self.model
    seq = native.atomic_load_u32(b.seq_addr)
    ready = [s for s in range(b.S) if b.state(s) == REQUEST]
    if not ready:
      native.futex_wait(b.seq_addr, seq, timeout_ms)
      return False
    mask = self.mask_host
    mask.zero_()
    rows = 0
    for s in ready:
      n = b.rows_of(s)
      mask[s * b.M:s * b.M + n] = 1.0
      rows += n
    has_instr = bool(m.use_instruction and
                     int(b.inputs['instr_len'].max(initial=0)) > 0)
    with torch.no_grad(), m._lock:
      if not self.cuda:
        self.in_dev.copy_(self._host_in)  # the row mask included
        self._body(has_instr)
        self._host_out.copy_(self.out_dev)
      else:
        with torch.cuda.stream(m.stream):
          self.in_dev.copy_(self._host_in, non_blocking=self.pinned)
          if self.use_graph:
            g = self._graphs.get(has_instr)
            if g is None:
              g = self._graphs[has_instr] = self._capture(has_instr)
            g.replay()
          else:
            self._body(has_instr)
          so = b.slot_out_bytes
          for s in ready if not self.direct_out else ():
            self._host_out[s * so:(s + 1) * so].copy_(
                self.out_dev[s * so:(s + 1) * so], non_blocking=self.pinned)
          m.stream.synchronize()
    for s in ready:
      native.atomic_store_u32(b.state_addr(s), RESPONSE)
      native.futex_wake(b.state_addr(s))
    self._batches += 1
    self._rows += rows
    return True

  # ------------------------------------------------------------ thread
  def _run(self):
    try:
      while not self._stop and not self.board.closed:
        self.serve_once()
    except Exception as e:  # pylint: disable=broad-except
      self.error = e
      log.exception('inference server failed')
      self.board.close()

  def _native_ok(self):
    # the graphs' sampler must keep its state on the device (PhiloxStream of
    # the HIP backend): a torch.Generator needs CUDAGraph.replay()'s host
    # prologue, which a C++ hipGraphLaunch does not run
    return (self.use_graph and self.pinned and
            os.environ.get('SA_BOARD_NATIVE', '1') != '0' and
            getattr(self.model.agent, 'backend', '') == 'hip')

  def _start_native(self):
    from .. import ops
    b, m = self.board, self.model
    variants = (False, True) if m.use_instruction else (False,)
    for v in variants:  # every graph the loop may launch, captured up front
      if v not in self._graphs:
        self.prepare(has_instr=v)
    exe = {v: self._graphs[v].raw_cuda_graph_exec() for v in variants}
    instr_off = [o for n, _, _, o, _ in b.in_fields if n == 'instr_len'][0]
    self._native = ops.ext().NativeBoardServer(
        b.base, b.HDR, b.in_bytes, b.slot_out_bytes, b.S, b.M, instr_off,
        self.in_dev.data_ptr(), self.out_dev.data_ptr(),
        self.mask_dev.data_ptr(), self.mask_host.data_ptr(),
        m.stream.cuda_stream, exe.get(False, 0),
        exe.get(True, 0) if m.use_instruction else 0,
        m.device.index if m.device.index is not None else
        self.torch.cuda.current_device())
    if self.depth == 2:
      self._sets.append(self._buffers(1))
      in_dev, out_dev, mask_dev, mask_host, _ = self._sets[1]
      with self.torch.no_grad():
        for v in variants:
          self._graphs[(1, v)] = self._capture(v, k=1)
      self._native.add_buffer(
          in_dev.data_ptr(), out_dev.data_ptr(), mask_dev.data_ptr(),
          mask_host.data_ptr(),
          self._graphs[(1, False)].raw_cuda_graph_exec(),
          self._graphs[(1, True)].raw_cuda_graph_exec()
          if m.use_instruction else 0)
    self._native.set_direct_output(self.direct_out)
    self._native.set_batching(self.min_ready, self.gather_us)
    self._native.start()

  def start(self):
    if self._native_ok():
      self._start_native()
      return
    self._thread = threading.Thread(target=self._run, daemon=True,
                                    name='inference-board-server')
    self._thread.start()

  def check(self):
    if self._native is not None and self.error is None:
      err = self._native.error()
      if err:
        self.error = err
    if self.error is not None:
      raise RuntimeError('inference server failed: %r' % (self.error,))

  def stop(self):
    self._stop = True
    native.futex_wake(self.board.seq_addr)
    if self._native is not None:
      self._native.stop()
    if self._thread is not None:
      self._thread.join(timeout=10)


class BoardLanes(object):
  """Several boards served side by side (`--inference_lanes`): lane l is its
  own board, BoardServer (native thread), InferenceModel (weight snapshot
  and stream), so the lanes' graphs run concurrently on the GPU.  A board
  launch at a few dozen rows is ~25 small kernels that leave most CUs idle
  (profiles/r6_e2e.md), so a second lane adds launches instead of waiting
  behind the first.  Same interface as one BoardServer for the train loop,
  plus publish() to every lane's model."""

  def __init__(self, servers):
    self.servers = list(servers)

  def publish(self, flat_params):
    for s in self.servers:
      s.model.publish(flat_params)

  def prepare(self, has_instr=False):
    for s in self.servers:
      s.prepare(has_instr=has_instr)

  def start(self):
    for s in self.servers:
      s.start()

  def check(self):
    for s in self.servers:
      s.check()

  def stop(self):
    for s in self.servers:
      s.stop()

  @property
  def batches(self):
    return sum(s.batches for s in self.servers)

  @property
  def rows_served(self):
    return sum(s.rows_served for s in self.servers)

