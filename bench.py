#!/usr/bin/env python3
"""Headline benchmark: learner env-frames/s, IMPALA deep ResNet + LSTM-256.

Config (BASELINE.json): B=32 per learner, unroll T=100 (T+1=101 frames per
sequence), 4 action repeats -> 12 800 env frames per learner step, synthetic
72x96x3 uint8 frames, 9 actions, random-init weights.

Precision: the reported `value` is measured at the REFERENCE's precision,
fp32 (reference experiment.py:153-189, 118, 413-415 all run fp32): exact-fp32
MFMA conv kernels (v_mfma_f32_16x16x4_f32), fp32 LSTM recurrence, fp32
V-trace / loss / RMSProp.  The bf16 learner (bf16 conv/GEMM operands, fp32
accumulation and state) is measured in the same run as a second field
(`config.bf16`), unless --dtype bf16 makes it the headline.

One process per GPU; N>1 is weak scaling (each learner consumes its own B=32
batch, gradients summed with one RCCL all-reduce).  Every timed step does the
full learner work of experiment.py:346-427: H2D of the next batch from pinned
host memory (StagingArea equivalent, overlapped on a copy stream), T+1-step
re-unroll, V-trace, loss, backward, gradient all-reduce, RMSProp with
on-device LR decay, frame-counter increment.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype fp32|bf16]

Multi-GPU: either launched by torch.distributed.run (one rank per GPU, the
env carries RANK/WORLD_SIZE/...), or plain `python bench.py --gpus N`: then
this process is only a launcher - it never imports torch or touches a GPU -
and starts N fresh rank processes itself (the reference's N-process local
cluster, experiment.py:497-512, minus gRPC), relays rank 0's JSON line and
exits non-zero if any rank fails or overruns its time limit.
"""

import argparse
import gc
import json
import os
import sys
import time


def _pdeathsig():
  """preexec_fn of a rank (runs in the GPU-free child before it starts
  python): the kernel SIGKILLs the rank if the launcher dies."""
  import ctypes
  import signal
  try:
    ctypes.CDLL('libc.so.6', use_errno=True).prctl(1, int(signal.SIGKILL))
  except OSError:  # pragma: no cover - not Linux
    pass


def _gpu_shortfall(n, device, env):
  """Message when `--gpus n` asks for more GPUs than are visible (sysfs +
  *_VISIBLE_DEVICES only: this process never touches the GPU), else None.
  A gloo rehearsal (SA_DIST_BACKEND=gloo) may share cards."""
  if device == 'cpu' or env.get('SA_DIST_BACKEND') == 'gloo':
    return None
  import importlib.util
  # the module file alone: the package __init__ would import torch
  spec = importlib.util.spec_from_file_location('_sa_affinity', os.path.join(
      os.path.dirname(os.path.abspath(__file__)), 'scalable_agent_amd',
      'parallel', 'affinity.py'))
  aff = importlib.util.module_from_spec(spec)
  spec.loader.exec_module(aff)
  have = aff.visible_gpu_count(env.get('SA_SYSFS_ROOT', '/sys'), env)
  if have is None or have >= n:
    return None
  return ('bench.py: --gpus %d but only %d GPU(s) are visible (KFD topology '
          'and *_VISIBLE_DEVICES); one rank per GPU over RCCL needs %d '
          'distinct GPUs (SA_DIST_BACKEND=gloo rehearses ranks sharing a '
          'card)' % (n, have, n))


def _self_launch(argv):
  """`--gpus N` (N>1) with no WORLD_SIZE in the env: run N ranks as child
  processes of this (GPU-free) launcher.  Returns the exit code.

  Lifetime: each rank runs in its own process group (so a kill reaches its
  children too) with PR_SET_PDEATHSIG, so ranks never outlive the launcher;
  SIGTERM / SIGINT to the launcher kill every rank group first.  The limit
  (SA_BENCH_TIMEOUT_S, default 540 s) stays under a 600 s driver timeout.
  Rank 0's stdout goes to a file and its JSON line is relayed only when
  every rank exits 0."""
  import signal
  import socket
  import subprocess
  import tempfile
  ap = argparse.ArgumentParser(add_help=False)
  ap.add_argument('--gpus', type=int, default=1)
  ap.add_argument('--device', default='auto')
  known, _ = ap.parse_known_args(argv)
  n = known.gpus
  msg = _gpu_shortfall(n, known.device, os.environ)
  if msg:
    sys.stderr.write(msg + '\n')
    return 2
  s = socket.socket()
  s.bind(('127.0.0.1', 0))
  port = s.getsockname()[1]
  s.close()
  limit = float(os.environ.get('SA_BENCH_TIMEOUT_S', '540'))
  procs = []
  out0 = tempfile.TemporaryFile(mode='w+')

  def kill_all():
    for p in procs:
      if p.poll() is None:
        try:
          os.killpg(p.pid, signal.SIGKILL)
        except OSError:
          pass
    for p in procs:
      p.wait()

  def on_signal(signum, _frame):
    sys.stderr.write('bench.py launcher: signal %d; killing the ranks\n' %
                     signum)
    kill_all()
    os._exit(128 + signum)

  signal.signal(signal.SIGTERM, on_signal)
  signal.signal(signal.SIGINT, on_signal)
  try:
    for r in range(n):
      env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r),
                 WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK='0',
                 MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
      env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
      # rank 0 owns the one JSON line; the others' stdout is dropped
      procs.append(subprocess.Popen(
          [sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
          stdout=out0 if r == 0 else subprocess.DEVNULL,
          start_new_session=True, preexec_fn=_pdeathsig))
    t0 = time.time()
    last_note = t0
    while True:
      codes = [p.poll() for p in procs]
      bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
      if bad:
        r, c = bad[0]
        sys.stderr.write('bench.py launcher: rank %d exited with %d; '
                         'stopping the other ranks\n' % (r, c))
        kill_all()
        return c if c > 0 else 1
      if all(c == 0 for c in codes):
        out0.seek(0)
        sys.stdout.write(out0.read())
        sys.stdout.flush()
        return 0
      now = time.time()
      if now - t0 > limit:
        sys.stderr.write('bench.py launcher: ranks still running after '
                         '%.0f s; killing them\n' % limit)
        kill_all()
        return 124
      if now - last_note > 60:
        last_note = now
        sys.stderr.write('bench.py launcher: %d/%d ranks running (%.0f s)\n'
                         % (sum(c is None for c in codes), n, now - t0))
        sys.stderr.flush()
      time.sleep(0.2)
  finally:
    kill_all()


def _wants_self_launch(argv):
  if 'WORLD_SIZE' in os.environ:
    return False
  ap = argparse.ArgumentParser(add_help=False)
  ap.add_argument('--gpus', type=int, default=1)
  known, _ = ap.parse_known_args(argv)
  return known.gpus > 1


# Hardware queues per process before the first HIP call (inherited by
# self-launched ranks): enough that the compute, H2D copy, early all-reduce
# and RCCL's own streams each get a queue instead of sharing
# (scalable_agent_amd/parallel/streams.py, profiles/r6_dp_queues.txt)
os.environ.setdefault('GPU_MAX_HW_QUEUES', '8')

if __name__ == '__main__' and _wants_self_launch(sys.argv[1:]):
  sys.exit(_self_launch(sys.argv[1:]))

import torch  # noqa: E402  (after the launcher: it must not load torch)

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from scalable_agent_amd import flags as flags_lib  # noqa: E402
from scalable_agent_amd.envs.synthetic import (  # noqa: E402
    add_synthetic_instructions, make_synthetic_batch)
from scalable_agent_amd.learner import FlatStaging, Learner  # noqa
from scalable_agent_amd.models import Agent  # noqa: E402
from scalable_agent_amd.models.agent import torso_precision  # noqa: E402
from scalable_agent_amd import parallel  # noqa: E402
from scalable_agent_amd.utils.knobs import measure_env, set_knobs  # noqa: E402

METRIC = ('learner env-frames/sec, IMPALA deep-ResNet+LSTM, batch=32 '
          'unroll=100, 1/2/4/8 GPU')
BASELINE_FPS = 250000.0  # BASELINE.md §B best published single-learner figure


def measure(args, dtype, device, backend, rank, world):
  """Builds one learner at `dtype` and times K steps after W warmups.
  Returns a dict of per-rank results (dt is the MAX over ranks)."""
  flags = flags_lib.default_flags(
      batch_size=args.batch_size, unroll_length=args.unroll_length,
      torso=args.torso, dtype=dtype, height=args.height, width=args.width,
      popart=args.popart > 0)
  num_actions = 9
  frame_shape = (args.height, args.width, args.channels)
  cdt = torch.bfloat16 if dtype == 'bf16' else torch.float32
  agent = Agent(num_actions, torso=args.torso, frame_shape=frame_shape,
                seed=flags.seed, backend=backend, compute_dtype=cdt,
                pipeline_chunks=args.pipeline_chunks,
                num_value_heads=max(1, args.popart))
  learner = Learner(agent, flags, device, world_size=world)
  if world > 1:
    parallel.broadcast_params(learner.flat.params)

  host_batches = [
      make_synthetic_batch(args.batch_size, args.unroll_length, frame_shape,
                           num_actions, seed=1000 * rank + i, pin_memory=False)
      for i in range(2)]
  if args.instructions:
    # DMLab-style levels: instruction strings through the language LSTM
    # (reference experiment.py:123-146) as part of the core input
    host_batches = [add_synthetic_instructions(hb, agent.embed.shape[0],
                                               seed=77 + i)
                    for i, hb in enumerate(host_batches)]
  if args.popart > 0:
    # DMLab-30-style multi-task batch: a task (value head) per batch column
    g = torch.Generator().manual_seed(5 + rank)
    host_batches = [hb._replace(level_name=torch.randint(
        0, args.popart, (args.batch_size,), generator=g))
                    for hb in host_batches]
  cuda = device.type == 'cuda'
  use_graph = bool(args.graph) and cuda
  graphs = []
  if cuda:
    # ONE copy stream per process, reused by every measurement: a stream
    # created after the first learner's streams can land on the compute
    # stream's hardware queue (HIP deals streams round-robin over
    # GPU_MAX_HW_QUEUES = 4), and the 67 MB prefetch then serialises with
    # the step (the bf16 field measured 5.8 ms = 4.6 ms of kernels + the
    # 1.2 ms copy, against 4.6 ms when it ran first)
    copy_stream = parallel.stream_plan(device).copy
    # one flat pinned host buffer per batch and one flat device buffer per
    # staging slot: the per-step prefetch is ONE H2D copy
    host_flat = [FlatStaging(hb, 'cpu', pin=True).load(hb)
                 for hb in host_batches]
    dev_flat = [FlatStaging(hb, device).load(hb) for hb in host_batches]
    slots = [d.views for d in dev_flat]
    if use_graph:
      # one captured graph per staging slot (static input addresses)
      for sl in slots:
        learner.capture(sl, clone=False)
        # split mode (world>1): the torso-feature tensors live in this
        # slot's graph pool; keeping them per slot stops the next capture
        # from freeing them (experiment.py keeps them the same way)
        graphs.append((learner._graph, learner._static_in,
                       learner._static_loss,
                       getattr(learner, '_graph_keep', None)))
    slot_free = [torch.cuda.Event(), torch.cuda.Event()]
    slot_ready = [torch.cuda.Event(), torch.cuda.Event()]
    for e in slot_ready + slot_free:
      e.record()
    comp = torch.cuda.current_stream(device)
    # standalone H2D bandwidth of one batch slab on the copy stream (reported:
    # the per-step prefetch hides behind compute only while it is shorter)
    h2d_ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize(device)
    with torch.cuda.stream(copy_stream):
      h2d_ev[0].record(copy_stream)
      dev_flat[1].copy_from(host_flat[1])
      h2d_ev[1].record(copy_stream)
    torch.cuda.synchronize(device)
    h2d_ms = h2d_ev[0].elapsed_time(h2d_ev[1])
    h2d_mb = dev_flat[1].nbytes / 1e6
  # diagnostic only (never the reported benchmark): SA_BENCH_SKIP_H2D=1 drops
  # the per-step host->device prefetch of the next batch
  skip_h2d = measure_env('SA_BENCH_SKIP_H2D') == '1'
  # who orders the prefetch against the steps.  'host' (default): the host
  # waits for slot j's previous step before enqueuing the copy into it and for
  # the copy before launching the step that reads it, so neither stream holds
  # a device-side wait on the other.  'device': stream-waits on the two
  # events.  Measured with tools/micro/step_jitter.py: the device-side waits
  # cost 0.15-0.2 ms per step plus 1-4 ms outlier steps (fp32 9.50 ms mean vs
  # 9.13 with no copy at all); host-side 9.15 (bf16: 4.63 / 4.41 / 4.44).
  # The host stays a step ahead: it is released ~1.2 ms into step k (copy
  # done) and enqueues step k+1 in 2-4 ms
  host_sync = measure_env('SA_BENCH_PREFETCH_SYNC', 'host') != 'device'

  def run_step(k):
    i = k % 2
    if not cuda:
      return learner.step(host_batches[i])
    # prefetch batch k+1 into the other slot while computing on slot i
    j = (k + 1) % 2
    if host_sync:
      slot_ready[i].synchronize()
    else:
      comp.wait_event(slot_ready[i])
    if use_graph:
      (learner._graph, learner._static_in, learner._static_loss,
       learner._graph_keep) = graphs[i]
      loss = learner.graph_step()
    else:
      loss = learner.step(slots[i])
    slot_free[i].record(comp)
    with torch.cuda.stream(copy_stream):
      if host_sync:
        slot_free[j].synchronize()  # step k-1, slot j's reader, is done
      else:
        copy_stream.wait_event(slot_free[j])
      if not skip_h2d:
        dev_flat[j].copy_from(host_flat[(k + 1) % len(host_flat)])
      slot_ready[j].record(copy_stream)
    return loss

  def sync():
    if cuda:
      torch.cuda.synchronize(device)
    if world > 1:
      torch.distributed.barrier()
    if cuda:
      torch.cuda.synchronize(device)

  for k in range(args.warmup):
    run_step(k)
  sync()
  t0 = time.perf_counter()
  for k in range(args.warmup, args.warmup + args.steps):
    loss = run_step(k)
  t_enq = time.perf_counter() - t0  # host time to enqueue the K steps
  sync()
  dt = time.perf_counter() - t0
  dist_extra = {}
  if world > 1:
    # per-rank step time (the reported dt is the max), the all-reduce window
    # of the last step (begin of the early bucket -> end of the last one, so
    # it spans the overlapped torso backward) and a standalone all-reduce of
    # the whole flat gradient buffer (the bare collective's cost)
    per = [torch.zeros(1, dtype=torch.float64, device=device)
           for _ in range(world)]
    torch.distributed.all_gather(
        per, torch.tensor([dt], dtype=torch.float64, device=device))
    dt = max(float(x.item()) for x in per)
    dist_extra['per_rank_ms_per_step'] = [
        round(1000 * float(x.item()) / args.steps, 3) for x in per]
    if learner.grad_sync is not None:
      dist_extra['allreduce_window_ms'] = round(
          1000 * learner.grad_sync.last_time_s, 3)
      g = learner.flat.grads
      reps = 10
      sync()
      t1 = time.perf_counter()
      for _ in range(reps):
        torch.distributed.all_reduce(g)
      sync()
      dist_extra['allreduce_ms_standalone'] = round(
          1000 * (time.perf_counter() - t1) / reps, 3)
      dist_extra['allreduce_mbytes'] = round(g.numel() * 4 / 1e6, 2)
  res = {
      'dt': dt, 'loss_finite': bool(torch.isfinite(loss).item()),
      'enqueue_s': t_enq, 'frames_per_step': learner.frames_per_step,
      'health': learner.health(), 'torso': torso_precision(agent),
      'hip_graph': use_graph, 'h2d_prefetch': not skip_h2d,
      'h2d_prefetch_sync': 'host' if host_sync else 'device',
      'h2d_slab': ({'mbytes': round(h2d_mb, 1), 'ms': round(h2d_ms, 3),
                    'gbps': round(h2d_mb / max(h2d_ms, 1e-6), 1)} if cuda else None),
      'dist_extra': dist_extra,
  }
  del learner, agent, graphs
  gc.collect()
  if cuda:
    torch.cuda.synchronize(device)
    torch.cuda.empty_cache()
  return res


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--gpus', type=int, default=1)
  ap.add_argument('--steps', type=int, default=20)
  ap.add_argument('--warmup', type=int, default=5)
  ap.add_argument('--batch_size', type=int, default=32)
  ap.add_argument('--unroll_length', type=int, default=100)
  ap.add_argument('--torso', default='deep')
  ap.add_argument('--height', type=int, default=72)
  ap.add_argument('--width', type=int, default=96)
  ap.add_argument('--channels', type=int, default=3)
  ap.add_argument('--backend', default='auto', choices=['auto', 'torch', 'hip'])
  ap.add_argument('--dtype', default='fp32', choices=['fp32', 'bf16'],
                  help='precision of the reported value (fp32 = reference)')
  ap.add_argument('--also_bf16', type=int, default=1,
                  help='with --dtype fp32: also time the bf16 learner')
  ap.add_argument('--instructions', type=int, default=0,
                 help='1: DMLab-style batches with instruction strings '
                      '(language LSTM in the core input).')
  ap.add_argument('--popart', type=int, default=0,
                  help='K > 0: multi-task PopArt learner with K value heads '
                       '(DMLab-30: 30), random task per batch column')
  ap.add_argument('--graph', type=int, default=1)
  ap.add_argument('--device', default='auto')
  ap.add_argument('--pipeline_chunks', type=int, default=1,
                  help='time chunks of the torso || LSTM pipeline (1 = off)')
  args = ap.parse_args()
  if args.torso == 'shallow' and args.dtype == 'bf16' and args.backend != 'torch':
    raise SystemExit('bench.py: --dtype bf16 --torso shallow: the shallow '
                     'torso has exact-fp32 HIP kernels only')

  if args.device in ('auto', 'cuda') or args.device.startswith('cuda:'):
    if torch.cuda.device_count() > 0:  # does not initialise the GPU
      # this rank's host side (pinned staging, feeder) on its GPU's NUMA
      # node, before any pinned allocation (sysfs only; no-op if unknown)
      parallel.pin_to_gpu_numa(parallel.world_info()[2] %
                               torch.cuda.device_count())
  world_env = parallel.world_info()[1]
  if (world_env > 1 and args.device != 'cpu' and
      os.environ.get('SA_DIST_BACKEND') != 'gloo'):
    local_world = int(os.environ.get('LOCAL_WORLD_SIZE', str(world_env)))
    have = torch.cuda.device_count()  # does not initialise the GPU
    if have < local_world:
      raise SystemExit(
          'bench.py: %d ranks on this node but only %d visible GPU(s); RCCL '
          'needs one distinct GPU per rank (SA_DIST_BACKEND=gloo rehearses '
          'ranks sharing a card)' % (local_world, have))
  local = parallel.world_info()[2]
  if args.device == 'auto':
    # one-card rehearsal (SA_DIST_BACKEND): ranks share the visible GPUs
    if torch.cuda.is_available():
      local = local % torch.cuda.device_count()
    device = torch.device('cuda', local) if torch.cuda.is_available() else \
        torch.device('cpu')
  else:
    device = torch.device(args.device)
  if device.type == 'cuda':
    torch.cuda.set_device(device)
    # the process's streams, created and first used in their fixed order
    # BEFORE RCCL's init (a stream takes its hardware queue at its first
    # use: parallel/streams.py)
    parallel.stream_plan(device)
  rank, world, local = parallel.init_distributed()
  if args.gpus != world:
    raise SystemExit('bench.py: --gpus %d but WORLD_SIZE=%d' %
                     (args.gpus, world))
  if device.type == 'cuda':
    # one collective: the communicator is up before the first measured step
    parallel.warmup_collective(device)

  backend = args.backend
  if backend == 'auto':
    backend = 'torch'
    if device.type == 'cuda':
      from scalable_agent_amd import ops
      ops.load()  # a GPU run without the kernels fails loudly (no silent torch)
      backend = 'hip'

  main_res = measure(args, args.dtype, device, backend, rank, world)
  extra = None
  if (args.dtype == 'fp32' and args.also_bf16 and backend == 'hip' and
      args.torso == 'deep'):  # the shallow torso has fp32 kernels only
    extra = measure(args, 'bf16', device, backend, rank, world)

  def fps(r):
    return r['frames_per_step'] * args.steps / r['dt']

  value = fps(main_res)
  if rank == 0:
    dist_info = parallel.backend_info()
    cfg = {'model': 'IMPALA %s-ResNet+LSTM-256' % args.torso
                    if args.torso == 'deep' else 'IMPALA shallow+LSTM',
           'global_batch': args.batch_size * world,
           'seq_len': args.unroll_length,
           'frame': '%dx%dx%d' % (args.height, args.width, args.channels),
           'parallelism': 'dp%d' % world, 'backend': backend,
           'torso_kernels': main_res['torso'],
           'hip_graph': main_res['hip_graph'],
           'loss_finite': main_res['loss_finite'],
           'learner_health': main_res['health'],
           'pipeline_chunks': args.pipeline_chunks,
           'instructions': bool(args.instructions),
           'popart_tasks': args.popart,
           'host_enqueue_ms_per_step': round(
               1000 * main_res['enqueue_s'] / args.steps, 3),
           'h2d_prefetch': main_res['h2d_prefetch'],
           'h2d_prefetch_sync': main_res['h2d_prefetch_sync'],
           'h2d_slab': main_res['h2d_slab'],
           'dist': dict(dist_info, **main_res['dist_extra']),
           # every SA_* variable this run was started with (experiment
           # switches only act in SA_MEASURE_KNOBS runs / builds:
           # csrc/kernels/knobs.h, utils/knobs.py)
           'knobs': set_knobs(),
           'baseline_ref': 'IMPALA paper best 1-GPU learner 250K '
                           'frames/s (BASELINE.md B), fp32 P100',
           # the ratio sets this learner-only synthetic number against the
           # paper's end-to-end system (actors + learner, shallow model)
           'vs_baseline_kind': 'learner-only vs paper end-to-end'}
    if extra is not None:
      cfg['bf16'] = {'value': round(fps(extra), 1),
                     'ms_per_step': round(1000 * extra['dt'] / args.steps, 3),
                     'vs_baseline': round(fps(extra) / BASELINE_FPS, 3),
                     'torso_kernels': extra['torso'],
                     'loss_finite': extra['loss_finite'],
                     'learner_health': extra['health'],
                     'h2d_slab': extra['h2d_slab']}
  rec = None
  if rank == 0:
    rec = {
        'metric': METRIC, 'value': round(value, 1), 'unit': 'env-frames/s',
        'n_gpus': world if device.type == 'cuda' else 0,
        'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(1000 * main_res['dt'] / args.steps, 3),
        'higher_is_better': True, 'scaling': 'weak',
        'vs_baseline': round(value / BASELINE_FPS, 3),
        'dtype': args.dtype,
        'data': 'synthetic (random uint8 frames, random-init weights)',
        'config': cfg,
    }
  if world > 1:
    # every rank got here (its measurements finished) before rank 0 reports:
    # a rank that failed earlier never joins, so no line is printed
    done = torch.ones(1, device=device if device.type == 'cuda' else 'cpu')
    torch.distributed.all_reduce(done)
    if int(done.item()) != world:
      raise SystemExit('bench.py: not every rank finished')
  if rank == 0:
    print(json.dumps(rec), flush=True)
  parallel.cleanup()


if __name__ == '__main__':
  main()
