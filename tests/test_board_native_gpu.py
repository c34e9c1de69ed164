"""Native (C++) inference-board serving thread (csrc/board_server.cpp)
against the Python server loop (runtime/inference_board.py): the same
captured graph answers a request bit-identically through either loop, and
the C++ thread serves forked CPU workers end to end (row counts, untouched
state of rows that never asked, close on stop)."""

import multiprocessing as mp
import time

import numpy as np
import pytest
import torch

from scalable_agent_amd.inference import InferenceModel
from scalable_agent_amd.models import Agent
from scalable_agent_amd.runtime import native
from scalable_agent_amd.runtime.inference_board import (
    REQUEST, RESPONSE, BoardClient, BoardServer, InferenceBoard)

pytestmark = pytest.mark.gpu

SHAPE = (24, 32, 3)


def _model(cuda, instr=False):
  agent = Agent(9, torso='deep', frame_shape=SHAPE, seed=2, backend='hip')
  return InferenceModel(agent, cuda, use_instruction=instr, seed=1)


def _fill(board, slot, rows, seed):
  rng = np.random.RandomState(seed)
  cl = BoardClient(board, slot, rows)
  cl.inputs['frame'][:] = rng.randint(0, 256, cl.inputs['frame'].shape)
  cl.inputs['reward'][:] = rng.randn(rows)
  cl.inputs['last_action'][:] = rng.randint(0, 9, rows)
  cl.inputs['done'][:] = False
  return cl


def _out_block(board, slot):
  o0 = board.HDR + board.in_bytes + slot * board.slot_out_bytes
  return board.buf[o0:o0 + board.slot_out_bytes]


def test_native_loop_matches_python_loop(cuda):
  """Also: the graph's epilogue writes the answer straight into the host
  board (direct output, no D2H copy) and only the requesting slot's valid
  rows: the other slots' output blocks and slot 1's unused row keep their
  bytes."""
  board = InferenceBoard(3, 4, SHAPE, 9)
  server = BoardServer(_model(cuda), board)
  assert server._native_ok() and server.direct_out
  server.prepare(has_instr=False)
  cl = _fill(board, 1, 3, seed=5)
  outs = []
  for loop in ('python', 'native'):
    server.c.zero_()
    server.h.zero_()
    board.buf[board.HDR + board.in_bytes:] = 0x5A
    native.atomic_store_u32(board.state_addr(1), REQUEST)
    if loop == 'python':
      assert server.serve_once(timeout_ms=10)
    else:
      from scalable_agent_amd import ops
      b, m = board, server.model
      off = [o for n, _, _, o, _ in b.in_fields if n == 'instr_len'][0]
      ns = ops.ext().NativeBoardServer(
          b.base, b.HDR, b.in_bytes, b.slot_out_bytes, b.S, b.M, off,
          server.in_dev.data_ptr(), server.out_dev.data_ptr(),
          server.mask_dev.data_ptr(), server.mask_host.data_ptr(),
          m.stream.cuda_stream, server._graphs[False].raw_cuda_graph_exec(),
          0, cuda.index or 0)
      ns.set_direct_output(server.direct_out)
      assert ns.serve_once(10) and ns.rows_served() == 3
    assert board.state(1) == RESPONSE
    for s in (0, 2):
      assert np.all(_out_block(board, s) == 0x5A)
    for name, _, _, o, nb in board.out_fields:  # slot 1's row 3 (unused)
      per = nb // board.M
      assert np.all(_out_block(board, 1)[o + 3 * per:o + 4 * per] == 0x5A)
    _, logits, baseline, c, h = [x.copy() for x in cl.wait()]
    outs.append((logits, baseline, c, h, server.c.cpu().clone()))
  for a, b in zip(outs[0], outs[1]):
    assert np.array_equal(np.asarray(a), np.asarray(b))
  # rows of slots that did not ask keep a zero state; slot 1's rows moved
  st = outs[1][4]
  assert float(st[0:4].abs().sum()) == 0.0 and float(st[8:].abs().sum()) == 0.0
  assert float(st[4:7].abs().sum()) > 0.0 and float(st[7].abs().sum()) == 0.0
  board.close()


def _worker(board, slot, rows, n_steps, seed):
  import os
  cl = BoardClient(board, slot, rows)
  rng = np.random.RandomState(seed)
  for _ in range(n_steps):
    cl.inputs['frame'][:] = rng.randint(0, 256, cl.inputs['frame'].shape)
    cl.inputs['done'][:] = False
    cl.launch()
    a, lg, b, c, h = cl.wait()
    assert a.shape == (rows,) and np.all((a >= 0) & (a < 9))
    assert np.all(np.isfinite(lg)) and np.all(np.isfinite(c))
  os._exit(0)


def test_depth2_native_loop_matches_python_loop(cuda):
  """Two batches in flight over two buffer sets (the depth-2 native loop):
  slot 0's batch is still in flight when slot 2's is launched on the
  second set, is answered while it runs, and both answers match the Python
  loop serving the same two requests one after the other."""
  from scalable_agent_amd import ops
  board = InferenceBoard(3, 4, SHAPE, 9)
  server = BoardServer(_model(cuda), board)
  server.prepare(has_instr=False)
  server._sets.append(server._buffers(1))
  with torch.no_grad():
    g1 = server._capture(False, k=1)
  cl0 = _fill(board, 0, 4, seed=6)
  cl2 = _fill(board, 2, 2, seed=7)
  outs = []
  for loop in ('python', 'native'):
    server.c.zero_()
    server.h.zero_()
    if loop == 'python':
      for s in (0, 2):
        native.atomic_store_u32(board.state_addr(s), REQUEST)
        assert server.serve_once(timeout_ms=10)
    else:
      b, m = board, server.model
      off = [o for n, _, _, o, _ in b.in_fields if n == 'instr_len'][0]
      ns = ops.ext().NativeBoardServer(
          b.base, b.HDR, b.in_bytes, b.slot_out_bytes, b.S, b.M, off,
          server.in_dev.data_ptr(), server.out_dev.data_ptr(),
          server.mask_dev.data_ptr(), server.mask_host.data_ptr(),
          m.stream.cuda_stream, server._graphs[False].raw_cuda_graph_exec(),
          0, cuda.index or 0)
      ns.set_direct_output(server.direct_out)
      in1, out1, mask1, mhost1, _ = server._sets[1]
      ns.add_buffer(in1.data_ptr(), out1.data_ptr(), mask1.data_ptr(),
                    mhost1.data_ptr(), g1.raw_cuda_graph_exec(), 0)
      assert ns.depth() == 2
      native.atomic_store_u32(board.state_addr(0), REQUEST)
      assert ns.serve_once(10, drain=False)
      assert board.state(0) == REQUEST  # in flight, not answered yet
      native.atomic_store_u32(board.state_addr(2), REQUEST)
      assert ns.serve_once(10, drain=False)  # launches slot 2, answers 0
      assert board.state(0) == RESPONSE and board.state(2) == REQUEST
      assert ns.serve_once(10)  # nothing new: answers the batch in flight
      assert ns.batches() == 2 and ns.rows_served() == 6
    assert board.state(0) == RESPONSE and board.state(2) == RESPONSE
    outs.append([x.copy() for cl in (cl0, cl2) for x in cl.wait()[1:]] +
                [server.c.cpu().clone()])
  for a, b in zip(outs[0], outs[1]):
    assert np.array_equal(np.asarray(a), np.asarray(b))
  st = outs[1][-1]
  assert float(st[0:4].abs().sum()) > 0.0 and float(st[8:10].abs().sum()) > 0
  assert float(st[4:8].abs().sum()) == 0.0 and float(st[10:].abs().sum()) == 0
  board.close()


@pytest.mark.parametrize('depth', [1, 2])
def test_native_thread_serves_forked_workers(cuda, depth):
  board = InferenceBoard(4, 8, SHAPE, 9)
  # the forked workers only use the shared board and futexes, never HIP
  ctx = mp.get_context('fork')
  procs = [ctx.Process(target=_worker, args=(board, s, r, 20, s))
           for s, r in ((0, 8), (1, 5), (3, 2))]
  for p in procs:
    p.start()
  server = BoardServer(_model(cuda), board, depth=depth)
  server.start()
  assert server.native and server._native.depth() == depth
  deadline = time.time() + 60
  while any(p.is_alive() for p in procs) and time.time() < deadline:
    server.check()
    time.sleep(0.01)
  for p in procs:
    p.join(10)
    assert p.exitcode == 0
  server.check()
  assert server.rows_served == 20 * (8 + 5 + 2)
  assert server.batches >= 20
  server.stop()
  st = server.c.cpu()
  assert float(st[16:24].abs().sum()) == 0.0  # slot 2 never asked
  assert float(st[8 + 5:16].abs().sum()) == 0.0  # slot 1's unused rows
  board.close()


def test_board_epilogue_matches_torch_ops(cuda):
  """The fused board epilogue (one launch: masked LSTM state update +
  slot-major packing of every output field) against the torch ops it
  replaces in BoardServer._body, on a 3-slot x 5-row board."""
  from scalable_agent_amd import ops
  C = ops.ext()
  S, M, A, H = 3, 5, 9, 256
  R = S * M
  board = InferenceBoard(S, M, (8, 8, 3), A)
  g = torch.Generator().manual_seed(3)
  action = torch.randint(0, A, (R,), generator=g).to(cuda)
  logits = torch.randn(R, A, generator=g).to(cuda)
  baseline = torch.randn(R, generator=g).to(cuda)
  c2, h2 = torch.randn(R, H, generator=g).to(cuda), torch.randn(R, H, generator=g).to(cuda)
  c0, h0 = torch.randn(R, H, generator=g).to(cuda), torch.randn(R, H, generator=g).to(cuda)
  mask = (torch.rand(R, 1, generator=g) > 0.5).float().to(cuda)
  out = torch.zeros(board.out_bytes, dtype=torch.uint8, device=cuda)
  ref = torch.zeros_like(out)
  c, h = c0.clone(), h0.clone()
  C.board_epilogue([action, logits, baseline, c2, h2],
                   [o for _, _, _, o, _ in board.out_fields], out, M,
                   board.slot_out_bytes, mask, c2, h2, c, h)
  rc = torch.where(mask > 0, c2, c0)
  rh = torch.where(mask > 0, h2, h0)
  view = ref.view(S, board.slot_out_bytes)
  for (n, s, dt, o, nb), v in zip(board.out_fields,
                                  (action, logits, baseline, c2, h2)):
    per = nb // M
    view[:, o:o + M * per].copy_(
        v.reshape(S, M, -1).contiguous().view(torch.uint8).view(S, M * per))
  torch.cuda.synchronize()
  assert torch.equal(c, rc) and torch.equal(h, rh)
  assert torch.equal(out, ref)
  # out_addr (the direct-output form): only the masked rows are packed, the
  # bytes of every other row stay as they were
  out2 = torch.full_like(out, 0x5A)
  c, h = c0.clone(), h0.clone()
  C.board_epilogue([action, logits, baseline, c2, h2],
                   [o for _, _, _, o, _ in board.out_fields], out, M,
                   board.slot_out_bytes, mask, c2, h2, c, h,
                   out_addr=out2.data_ptr())
  ref2 = torch.full_like(out, 0x5A)
  v2, vr = ref2.view(S, board.slot_out_bytes), ref.view(S, board.slot_out_bytes)
  for r in torch.nonzero(mask.view(-1) > 0).view(-1).tolist():
    s_, m_ = divmod(r, M)
    for _, _, _, o, nb in board.out_fields:
      per = nb // M
      v2[s_, o + m_ * per:o + (m_ + 1) * per] = vr[s_, o + m_ * per:o + (m_ + 1) * per]
  torch.cuda.synchronize()
  assert torch.equal(c, rc) and torch.equal(h, rh)
  assert torch.equal(out2, ref2)
  board.close()
