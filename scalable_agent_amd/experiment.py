"""Importance Weighted Actor-Learner Architectures: train / test drivers.

Same CLI and run modes as the reference experiment.py:
  * `--mode=train`, single machine (`--task=-1`, :479-672): env processes,
    `num_actors` actor threads whose per-step inference is dynamically batched
    onto the GPU, a bounded unroll queue, the learner loop (V-trace, RMSProp,
    frame counter), per-episode logging + summaries, DMLab-30 scores,
    checkpoints every `save_checkpoint_secs`, auto-restore on start;
  * distributed (`--job_name=learner|actor --task=i`, :497-512, README :55-71):
    actor processes run the agent on their own CPU with weights pulled from the
    learner and ship unrolls to it - here through a shared-memory slot ring
    and a shared-memory weight snapshot on one node (runtime/shm_transport.py)
    instead of TF gRPC;
  * `--mode=test` (:675-708): restores the latest checkpoint, runs each level
    until `test_num_episodes` episodes, prints the mean return and DMLab-30
    scores;
  * data-parallel learners (new): launch with torch.distributed.run, one rank
    per GPU; gradients are summed with RCCL (see parallel/).

Log lines kept verbatim: 'Level: %s Episode return: %f', 'Mean episode
return: %f', 'No cap.: %f Cap 100: %f'.
"""

import collections
import logging
import os
import queue
import sys
import threading
import time

import numpy as np

from . import dmlab30
from . import environments
from . import flags as flags_lib
from . import py_process
from .utils.knobs import measure_env

log = logging.getLogger('scalable_agent_amd')


# --------------------------------------------------------------- env factory
def env_kind(flags, level_name):
  if flags.env != 'auto':
    return flags.env
  if level_name.startswith('doom_'):
    return 'doom'
  if level_name.startswith('synthetic'):
    return 'synthetic'
  return 'dmlab'


def frame_shape_for(flags, level_name):
  kind = env_kind(flags, level_name)
  if kind == 'doom':
    from .envs.doom import DOOM_H, DOOM_W
    return (DOOM_H, DOOM_W, 3)
  if flags.obs_shape:
    return tuple(int(x) for x in flags.obs_shape.lower().split('x'))
  return (flags.height, flags.width, 3)


def action_set_for(flags, level_name):
  if env_kind(flags, level_name) == 'doom':
    from .envs.doom import DOOM_ACTION_SET
    return DOOM_ACTION_SET
  return environments.DEFAULT_ACTION_SET


def _supervision(flags, seed):
  """EnvProcess keyword args: hang watchdog + env-side fault injection."""
  from .runtime.faults import FaultSpec
  return dict(timeout=flags.env_timeout_secs,
              fault_inject=FaultSpec(flags.fault_inject).env_spec(),
              fault_seed=seed)


def create_environment(flags, level_name, seed, is_test=False):
  """Returns an unstarted EnvProcess (reference create_environment :430-459)."""
  kind = env_kind(flags, level_name)
  shape = frame_shape_for(flags, level_name)
  sup = _supervision(flags, seed)
  if kind == 'doom':
    from .envs.doom import PyProcessDoom
    return py_process.EnvProcess(PyProcessDoom, shape, level_name, None,
                                 flags.num_action_repeats, seed, **sup)
  if kind == 'synthetic':
    from .envs.synthetic import SyntheticEnv
    cfg = {'benchmark_mode': flags.benchmark_mode}
    return py_process.EnvProcess(
        SyntheticEnv, shape, level_name, cfg, flags.num_action_repeats, seed,
        frame_shape=shape, episode_length=flags.synthetic_episode_length, **sup)
  if level_name in dmlab30.ALL_LEVELS:
    level_name = 'contributed/dmlab30/' + level_name
  config = {
      'width': shape[1], 'height': shape[0],
      'datasetPath': flags.dataset_path, 'logLevel': 'WARN',
      'gpuDeviceIndex': '0', 'renderer': flags.renderer,
      'benchmark_mode': flags.benchmark_mode,
  }
  if is_test:
    config['allowHoldOutLevels'] = 'true'
    config['mixerSeed'] = 0x600D5EED
  return py_process.EnvProcess(environments.PyProcessDmLab, shape, level_name,
                               config, flags.num_action_repeats, seed, **sup)


def level_names_for(flags):
  if flags.level_name == 'dmlab30':
    src = (dmlab30.LEVEL_MAPPING.keys() if flags.mode == 'train'
           else dmlab30.LEVEL_MAPPING.values())
    return list(src)
  return [flags.level_name]


def uses_instruction(flags, level_names):
  return all(env_kind(flags, l) == 'dmlab' for l in level_names)


# --------------------------------------------------------------- helpers
def _device(flags, local_rank=0):
  """The rank's device: 'auto' / 'cuda' (no index) -> cuda:local_rank
  (modulo the visible GPUs: a one-card multi-rank rehearsal shares it)."""
  import torch
  if flags.device in ('auto', 'cuda'):
    if torch.cuda.is_available():
      return torch.device('cuda', local_rank % torch.cuda.device_count())
    if flags.device == 'cuda':
      raise RuntimeError('--device=cuda but no GPU is visible')
    return torch.device('cpu')
  return torch.device(flags.device)


def num_value_heads(flags):
  """PopArt: one normalised value output per task (level)."""
  return len(level_names_for(flags)) if flags.popart else 1


def _make_agent(flags, num_actions, frame_shape, device, seed, dtype=None):
  import torch
  from .models import Agent
  backend = 'torch'
  if device.type == 'cuda' and getattr(flags, 'backend', 'auto') != 'torch':
    from . import ops
    ops.load()  # fail loudly on a GPU box without the kernels
    backend = 'hip'
  elif getattr(flags, 'backend', 'auto') == 'hip':
    raise ValueError('--backend=hip needs a GPU device')
  dtype = dtype or flags.dtype
  cdt = torch.bfloat16 if dtype == 'bf16' else torch.float32
  return Agent(num_actions, torso=flags.torso, frame_shape=frame_shape,
               seed=seed, backend=backend, compute_dtype=cdt,
               num_value_heads=num_value_heads(flags),
               pipeline_chunks=getattr(flags, 'pipeline_chunks', 1))


class EpisodeLogger(object):
  """Per-episode logs, summaries and DMLab-30 scores (experiment.py:629-667)."""

  def __init__(self, flags, level_names, writer):
    self.flags = flags
    self.writer = writer
    self.level_names = level_names
    self.level_returns = {l: [] for l in level_names}
    self.episodes = 0
    self.recent_returns = collections.deque(maxlen=100)

  def log_batch(self, level_name_per_b, done, episode_return, episode_step,
                frames):
    """done/returns/steps: numpy [T, B] (already shifted to env_outputs[1:])."""
    ts, bs = np.nonzero(done)
    for t, b in zip(ts, bs):
      level = level_name_per_b[b]
      ret = float(episode_return[t, b])
      ep_frames = int(episode_step[t, b]) * self.flags.num_action_repeats
      log.info('Level: %s Episode return: %f', level, ret)
      self.episodes += 1
      self.recent_returns.append(ret)
      if self.writer is not None:
        self.writer.add_scalars({'%s/episode_return' % level: ret,
                                 '%s/episode_frames' % level: ep_frames},
                                frames)
      if self.flags.level_name == 'dmlab30':
        self.level_returns[level].append(ret)
    if (self.flags.level_name == 'dmlab30' and
        min(map(len, self.level_returns.values())) >= 1):
      no_cap = dmlab30.compute_human_normalized_score(self.level_returns,
                                                      per_level_cap=None)
      cap_100 = dmlab30.compute_human_normalized_score(self.level_returns,
                                                       per_level_cap=100)
      if self.writer is not None:
        self.writer.add_scalars({'dmlab30/training_no_cap': no_cap,
                                 'dmlab30/training_cap_100': cap_100}, frames)
      self.level_returns = {l: [] for l in self.level_names}


# --------------------------------------------------------------- feeder
def _h2d_stream(device):
  """The process's ONE host->device prefetch stream, created before any
  other stream (train() calls this first): HIP deals streams round-robin over
  GPU_MAX_HW_QUEUES = 4 hardware queues, and a copy stream created after the
  learner's / inference's streams can share the compute stream's queue, which
  serialises the ~1.2 ms slab copy with the learner step (measured in
  bench.py: the bf16 step 4.6 -> 5.8 ms)."""
  from .parallel.streams import stream_plan
  return stream_plan(device).copy


class _TrajFeeder(object):
  """Learner side of the trajectory queue (runtime/traj_queue.py).

  Per step: acquire a full slab (one [T+1, B] batch the actors wrote in
  place), ONE async H2D copy of it into the idle device slot on a copy
  stream, the compute stream waits on that copy's event and replays the
  slot's captured learner graph.  While step k computes on slot k % 2 the
  copy of step k+1 lands in the other slot (StagingArea, experiment.py:
  587-597).  A slab is released as soon as its copy event has completed
  (polled: the host never waits on compute)."""

  def __init__(self, tq, learner, device, use_graph):
    import collections
    import torch
    self.torch = torch
    self.tq = tq
    self.learner = learner
    self.device = device
    self.cuda = device.type == 'cuda'
    self.use_graph = use_graph and self.cuda
    n = 2 if self.cuda else 1
    self.slots = [torch.empty(tq.layout.nbytes, dtype=torch.uint8, device=device)
                  for _ in range(n)]
    self.views = [tq.layout.torch_views(s) for s in self.slots]
    self.graphs = [None] * n
    self.pending = collections.deque()
    self.k = 0
    self.host_sync = measure_env('SA_H2D_SYNC', 'host') != 'device'
    if self.cuda:
      self.copy_stream = _h2d_stream(device)
      self.free = [torch.cuda.Event() for _ in range(n)]
      for e in self.free:
        e.record()

  def prepare(self):
    """Captures both slots' learner graphs up front, on zero-filled slots
    (the graph does not depend on the values), BEFORE the actor threads
    start: no other thread touches the GPU during the captures."""
    if not self.use_graph:
      return
    learner = self.learner
    for j in range(len(self.slots)):
      self.slots[j].zero_()
      self.torch.cuda.synchronize(self.device)
      learner.capture(self.views[j], clone=False)
      self.graphs[j] = (learner._graph, learner._static_in,
                        learner._static_loss,
                        getattr(learner, '_graph_keep', None))

  def _reap(self, block):
    while self.pending:
      slab, ev = self.pending[0]
      if not ev.query():
        if not block:
          return
        ev.synchronize()
      self.pending.popleft()
      self.tq.release(slab)
      block = False

  def step(self, timeout_s, poison=False, check=None):
    """-> (loss, host info dict, seconds waited for a full slab).
    self.last_host_s: host time of the step's data path (slab hand-off,
    H2D enqueue, graph launch, slab release) excluding the wait."""
    torch = self.torch
    t0 = time.time()
    while True:
      self._reap(block=False)
      slab = self.tq.acquire(timeout_ms=200)
      if slab >= 0:
        break
      if slab == -2:
        raise RuntimeError('trajectory queue closed')
      if check is not None:
        check()  # e.g. an actor-group process died
      if time.time() - t0 > timeout_s:
        raise RuntimeError('learner starved: no full batch for %.0fs' %
                           timeout_s)
    t1 = time.time()
    wait = t1 - t0
    hv = self.tq.host_views(slab)
    info = {'level': hv['level'].copy(), 'done': hv['done'][1:].copy(),
            'episode_return': hv['episode_return'][1:].copy(),
            'episode_step': hv['episode_step'][1:].copy(),
            'action': hv['action'][1:].copy()}
    if poison:
      hv['reward'][1:, 0] = float('nan')  # fault injection: poisoned batch
    learner = self.learner
    if not self.cuda:
      self.slots[0].copy_(self.tq.host_tensor(slab))
      self.tq.release(slab)
      loss = learner.step(self.views[0])
      self.k += 1
      self.last_host_s = time.time() - t1
      return loss, info, wait
    j = self.k % 2
    # host-side ordering (as bench.py): device-side waits between the copy
    # and compute streams cost 0.15-0.2 ms per learner step plus outliers;
    # the host instead waits for slot j's last graph before the copy and for
    # the copy before the launch (the previous step keeps the GPU busy)
    host_sync = self.host_sync
    with torch.cuda.stream(self.copy_stream):
      if host_sync:
        self.free[j].synchronize()
      else:
        self.copy_stream.wait_event(self.free[j])  # slot j's last graph is done
      self.slots[j].copy_(self.tq.host_tensor(slab), non_blocking=True)
      copied = torch.cuda.Event()
      copied.record(self.copy_stream)
    comp = torch.cuda.current_stream(self.device)
    if host_sync:
      copied.synchronize()
    else:
      comp.wait_event(copied)
    self.pending.append((slab, copied))
    if self.use_graph:
      if self.graphs[j] is None:
        copied.synchronize()  # capture runs on the data in place
        learner.capture(self.views[j], clone=False)
        self.graphs[j] = (learner._graph, learner._static_in,
                          learner._static_loss,
                          getattr(learner, '_graph_keep', None))
      # split-backward graphs: each slot keeps its own pool tensors
      # (features / leaf gradients) alive alongside its graphs
      (learner._graph, learner._static_in, learner._static_loss,
       learner._graph_keep) = self.graphs[j]
      loss = learner.graph_step()
    else:
      loss = learner.step(self.views[j])
    self.free[j].record(comp)
    self.k += 1
    self._reap(block=len(self.pending) > 2)
    self.last_host_s = time.time() - t1
    return loss, info, wait

  def close(self):
    self._reap(block=True)

  def drain(self, timeout_s=10.0):
    """Waits (bounded, polling) until every H2D copy still reading a host
    slab has completed -> True; False if one is still in flight at the
    deadline (e.g. after a GPU fault), when the slabs must stay registered."""
    if not self.cuda:
      return True
    deadline = time.time() + timeout_s
    while self.pending:
      if self.pending[0][1].query():
        self.pending.popleft()  # the queue is closing: no release needed
        continue
      if time.time() > deadline:
        return False
      time.sleep(0.001)
    return True


# --------------------------------------------------------------- train
# --actor_groups=-1 on a GPU: from this many actors on, CPU actor groups of
# ~AUTO_GROUP_ENVS envs (at least 2 groups) with the inference board instead
# of one GPU group process (profiles/r6_e2e.md: config #2, 48 actors,
# 335-352 K vs 291-305 K frames/s; config #4, 150 actors, 540-551 K with
# bf16 inference)
AUTO_BOARD_ACTORS = 32
AUTO_GROUP_ENVS = 40


def auto_board_groups(num_actors):
  """CPU actor groups the auto layout uses with the inference board."""
  return max(2, -(-num_actors // AUTO_GROUP_ENVS))


def _checker(groups, server):
  """Health probe the trajectory feeder runs while it waits for a slab."""
  if groups is None and server is None:
    return None

  def check():
    if server is not None:
      server.check()
    if groups is not None:
      groups.check()
  return check


class _Terminated(BaseException):
  """Raised in the main thread by SIGTERM: stop cleanly and checkpoint."""


def _install_sigterm_handler():
  import signal
  if threading.current_thread() is not threading.main_thread():
    return

  def handler(signum, frame):
    del signum, frame
    raise _Terminated()

  signal.signal(signal.SIGTERM, handler)


def train(flags):
  """Single-machine or data-parallel learner(s) with local actors."""
  import torch
  from . import checkpoint as ckpt_lib
  from . import inference as inference_lib
  from . import parallel
  from .actor import Actor, stack_unrolls
  from .learner import FlatStaging, Learner, batch_to_device
  from .runtime.faults import FaultSpec
  from .summary import SummaryWriter
  from .utils.timing import StepTimer
  from .utils.tracing import trace

  faults = FaultSpec(flags.fault_inject)
  level_names = level_names_for(flags)
  task_index = {l: i for i, l in enumerate(level_names)}
  action_set = action_set_for(flags, level_names[0])
  num_actions = len(action_set)
  frame_shape = frame_shape_for(flags, level_names[0])
  use_instr = uses_instruction(flags, level_names)

  if flags.task >= 0 and flags.job_name == 'actor':
    from .runtime import shm_transport
    return shm_transport.run_actor_process(flags, level_names, action_set,
                                           frame_shape, use_instr)

  rank, world, local_rank = parallel.world_info()
  numa = getattr(flags, 'numa_affinity', 'auto')
  on_gpu = flags.device.startswith('cuda') or (
      flags.device == 'auto' and torch.cuda.device_count() > 0)
  local_world = int(os.environ.get('LOCAL_WORLD_SIZE', str(world)))
  if numa == 'on' or (numa == 'auto' and on_gpu and
                      parallel.auto_pin_wanted(local_world)):
    # before the actor processes fork and before any pinned allocation:
    # the rank's host-side data path lives next to its GPU (sysfs only, the
    # GPU is not initialised yet; device_count() does not initialise it).
    # 'auto' pins only when this node's ranks cover every socket: the
    # forked actors inherit the mask, and a lone rank would otherwise leave
    # them half of a 2-socket machine.
    parallel.pin_to_gpu_numa(local_rank % max(1, torch.cuda.device_count()))
  # many actor threads share the GIL with the learner thread: a short switch
  # interval bounds how long the learner waits for it between GPU launches
  sys.setswitchinterval(min(sys.getswitchinterval(), 0.0005))
  # Env processes (and actor-group processes) are forked BEFORE the GPU is
  # initialised.
  distributed_actors = flags.task >= 0 and flags.job_name == 'learner'
  n_groups = flags.actor_groups
  if n_groups < 0:  # auto (profiles/r6_e2e.md)
    on_gpu = (flags.device.startswith('cuda') or
              (flags.device == 'auto' and torch.cuda.device_count() > 0))
    n_groups = 1 if on_gpu else 0
    if on_gpu and flags.num_actors >= AUTO_BOARD_ACTORS:
      # one GPU group process is Python-bound (~300 K frames/s at 48 or 150
      # actors); CPU groups posting to the learner-process inference board
      # scale further
      n_groups = min(auto_board_groups(flags.num_actors), flags.num_actors)
      flags.inference_server = True
  flags.actor_groups = n_groups
  use_groups = (n_groups > 0 and not distributed_actors and
                flags.trajectory_queue and not flags.deterministic)
  envs, actors_levels, actor_seeds = [], [], []
  groups = shared_w = board = server = None
  if not distributed_actors:
    for i in range(flags.num_actors):
      actors_levels.append(level_names[i % len(level_names)])
      actor_seeds.append(flags.seed * 1000003 * (rank + 1) + i + 1)
  if use_groups:
    from .runtime.actor_group import ActorGroups, SharedWeights
    from .runtime.traj_queue import BatchLayout, TrajectoryQueue
    layout = BatchLayout(flags.unroll_length + 1, flags.batch_size,
                         frame_shape, num_actions, use_instruction=use_instr)
    tq = TrajectoryQueue(layout, max(3, -(-flags.num_actors //
                                          flags.batch_size) + 2))
    # created (sized) once the learner exists; the groups attach by name
    shared_w_name = '/sa_w_%d_%d' % (os.getpid(), rank)
    if flags.inference_device != 'auto':
      group_dev = flags.inference_device
    elif flags.device not in ('auto', 'cuda'):
      group_dev = flags.device
    else:  # device_count() does not initialise the GPU in this process
      ndev = torch.cuda.device_count()
      group_dev = 'cuda:%d' % (local_rank % ndev) if ndev else 'cpu'
    if flags.inference_server:
      from .runtime.actor_group import board_geometry
      from .runtime.inference_board import InferenceBoard
      lanes = max(1, min(flags.inference_lanes, n_groups))
      slots, rows = board_geometry(flags.num_actors, n_groups,
                                   flags.actor_group_splits, lanes)
      board = [InferenceBoard(slots, rows, frame_shape, num_actions)
               for _ in range(lanes)]
      group_dev = 'cpu (board served by the learner process)'
    groups = ActorGroups(
        flags, level_names, actors_levels, actor_seeds, tq, shared_w_name,
        frame_shape, action_set, use_instr, group_dev,
        flags.dtype if flags.inference_dtype == 'auto' else
        flags.inference_dtype, board=board)
    log.info('%d actor group(s) over %d envs, inference on %s',
             len(groups.procs), flags.num_actors, group_dev)
  elif not distributed_actors:
    for level, seed in zip(actors_levels, actor_seeds):
      envs.append(create_environment(flags, level, seed))
    py_process.start_all(envs, per_worker=flags.envs_per_worker)

  device = _device(flags, parallel.world_info()[2])
  if device.type == 'cuda':
    torch.cuda.set_device(device)
    # the process's streams, created and first used in their fixed order
    # BEFORE RCCL's init (parallel/streams.py: a stream takes its hardware
    # queue at its first use; the H2D feeder stream is the plan's first)
    _h2d_stream(device)
  rank, world, local_rank = parallel.init_distributed(
      timeout_s=flags.collective_timeout_secs)
  if flags.num_learners and flags.num_learners != world:
    raise ValueError(
        '--num_learners=%d but WORLD_SIZE=%d: launch one process per learner '
        '(python -m torch.distributed.run --nproc-per-node %d ...)' %
        (flags.num_learners, world, flags.num_learners))
  _install_sigterm_handler()
  if device.type == 'cuda':
    # one collective: the communicator is up before the first learner step
    parallel.warmup_collective(device)
  torch.manual_seed(flags.seed + rank)
  logdir = flags.logdir if rank == 0 else os.path.join(flags.logdir,
                                                       'rank%d' % rank)
  os.makedirs(logdir, exist_ok=True)
  writer = SummaryWriter(logdir) if rank == 0 else None

  agent = _make_agent(flags, num_actions, frame_shape, device, flags.seed)
  learner = Learner(agent, flags, device, world_size=world)
  restored = ckpt_lib.restore(flags.logdir, learner)
  if restored is not None:
    log.info('Restored checkpoint at %d frames', restored)
  elif flags.import_tf_checkpoint:
    # a reference (TF) run's model.ckpt-N: weights, RMSProp slots, frames
    from . import tf_checkpoint
    frames = tf_checkpoint.import_tf_checkpoint(flags.import_tf_checkpoint,
                                                learner=learner)
    log.info('Imported TF checkpoint %s (frames %s)',
             flags.import_tf_checkpoint, frames)
  if world > 1:
    parallel.broadcast_params(learner.flat.params)
  saver = ckpt_lib.PeriodicSaver(flags.logdir, learner, flags,
                                 flags.save_checkpoint_secs,
                                 flags.keep_checkpoints) if rank == 0 else None

  unroll_queue = queue.Queue(maxsize=max(2 * flags.batch_size,
                                         flags.num_actors))
  stop = threading.Event()
  threads = []
  actors = []
  transport = None
  infer = None
  if distributed_actors:
    from .runtime import shm_transport
    transport = shm_transport.LearnerTransport(flags, frame_shape,
                                               num_actions, learner)
    threading.Thread(target=transport.pump, args=(unroll_queue, stop),
                     daemon=True).start()
  elif use_groups:
    use_traj = True
    actor_errors = []
    tq.pin()
    feeder = _TrajFeeder(tq, learner, device,
                         flags.use_hip_graph and device.type == 'cuda')
    feeder.prepare()
    if board is not None:
      # the groups' inference: one captured graph over the whole board, on
      # its own stream of the learner's GPU context
      from .runtime.inference_board import BoardServer
      inf_device = (device if flags.inference_device == 'auto' else
                    torch.device(flags.inference_device))
      from .runtime.inference_board import BoardLanes
      servers = []
      for lane, lane_board in enumerate(board):
        inf_agent = _make_agent(
            flags, num_actions, frame_shape, inf_device, flags.seed,
            dtype=(flags.dtype if flags.inference_dtype == 'auto' else
                   flags.inference_dtype))
        lane_model = inference_lib.InferenceModel(
            inf_agent, inf_device, use_instr,
            seed=flags.seed + 17 * rank + 7919 * lane)
        servers.append(BoardServer(lane_model, lane_board,
                                   gather_us=flags.inference_gather_us,
                                   depth=flags.inference_board_depth))
      # the train loop publishes to every lane's model
      server = model = BoardLanes(servers)
      model.publish(learner.flat.params)
      server.prepare(has_instr=use_instr)
      server.start()
    else:
      shared_w = SharedWeights(shared_w_name, learner.flat.numel, create=True)
      shared_w.publish(learner.flat.params)  # groups start on these weights
      shared_w.flush()
  else:
    inf_device = (device if flags.inference_device == 'auto' else
                  torch.device(flags.inference_device))
    inf_dtype = (flags.dtype if flags.inference_dtype == 'auto' else
                 flags.inference_dtype)
    inf_agent = _make_agent(flags, num_actions, frame_shape, inf_device,
                            flags.seed, dtype=inf_dtype)
    model = inference_lib.InferenceModel(inf_agent, inf_device, use_instr,
                                         seed=flags.seed + 17 * rank)
    model.publish(learner.flat.params)
    infer = inference_lib.make_batched_infer(
        model, flags.inference_min_batch, flags.inference_max_batch,
        flags.inference_timeout_ms)
    actor_errors = []
    # time-major trajectory queue: actors write batches in place (no
    # stacking / transposing / staging memcpy on the learner); the
    # deterministic mode keeps the sorted unroll queue (column order would
    # follow actor timing)
    use_traj = not flags.deterministic and flags.trajectory_queue
    if use_traj:
      from .runtime.traj_queue import BatchLayout, TrajectoryQueue
      layout = BatchLayout(flags.unroll_length + 1, flags.batch_size,
                           frame_shape, num_actions, use_instruction=use_instr)
      num_slabs = max(3, -(-flags.num_actors // flags.batch_size) + 2)
      tq = TrajectoryQueue(layout, num_slabs,
                           pin_device=device if device.type == 'cuda' else None)
      feeder = _TrajFeeder(tq, learner, device,
                           flags.use_hip_graph and device.type == 'cuda')
      feeder.prepare()

    def actor_loop_traj(actor, level_index):
      try:
        while not stop.is_set():
          if not actor.unroll_into(tq, level_index, stop):
            break
      except Exception as e:  # pylint: disable=broad-except
        if not stop.is_set():
          actor_errors.append(e)
          log.exception('actor failed')

    def actor_loop(actor):
      try:
        while not stop.is_set():
          out = actor.unroll()
          while not stop.is_set():
            try:
              unroll_queue.put(out, timeout=0.5)
              break
            except queue.Full:
              pass
      except Exception as e:  # pylint: disable=broad-except
        if not stop.is_set():
          actor_errors.append(e)
          log.exception('actor failed')

    for i, env in enumerate(envs):
      actor = Actor(environments.FlowEnvironment(env), infer,
                    actors_levels[i], action_set, flags.unroll_length,
                    num_actions, use_instruction=use_instr,
                    stall_ms=faults.get('actor_stall'))
      actors.append(actor)
      if use_traj:
        t = threading.Thread(target=actor_loop_traj,
                             args=(actor, task_index[actors_levels[i]]),
                             daemon=True, name='actor-%d' % i)
      else:
        t = threading.Thread(target=actor_loop, args=(actor,), daemon=True,
                             name='actor-%d' % i)
      t.start()
      threads.append(t)

  if distributed_actors:
    use_traj = False
  episode_logger = EpisodeLogger(flags, level_names, writer)
  if flags.deterministic:
    torch.use_deterministic_algorithms(True, warn_only=True)
  timer = StepTimer(learner.frames_per_step)
  t_loop0 = time.time()
  last_summary = time.time()
  last_log_frames = int(learner.frames.item())
  reported_skips = 0
  steps = 0
  checks_ok = 0
  first_loss = float('nan')
  use_graph = flags.use_hip_graph and device.type == 'cuda'
  staging = dev_stage = copied = None
  host_ms, loop_ms = [], []
  failed = False
  try:
    frames = int(learner.frames.item())
    while frames < flags.total_environment_frames:
      if flags.max_learner_steps and steps >= flags.max_learner_steps:
        break
      if use_traj:
        t_step = time.time()
        with trace('learner_step'):
          loss, info, wait = feeder.step(
              flags.queue_timeout_secs,
              poison=faults.get('learner_nan') == steps + 1,
              check=_checker(groups, server))
        timer.add_wait(wait)
        steps += 1
        if (world > 1 and flags.consistency_check_steps and
            steps % flags.consistency_check_steps == 0):
          if not parallel.param_checksum_consistent(learner.flat.params):
            raise RuntimeError('data-parallel replicas diverged at step %d' %
                               steps)
          checks_ok += 1
        if steps == 1:
          first_loss = float(loss)
        if infer is not None or server is not None:
          model.publish(learner.flat.params)
        elif shared_w is not None:
          shared_w.publish(learner.flat.params)
        # host frame counter (the device counter drives the LR schedule;
        # reading it every step would sync the host with the GPU)
        frames += learner.frames_per_step
        timer.step()
        batch_levels = [level_names[i] for i in info['level']]
        episode_logger.log_batch(batch_levels, info['done'],
                                 info['episode_return'], info['episode_step'],
                                 frames)
        if steps > 2:  # the first steps include graph warmup
          host_ms.append(1e3 * feeder.last_host_s)
          loop_ms.append(1e3 * (time.time() - t_step - wait))
        host_actions = info['action']
      if not use_traj:
        t_wait = time.time()
        unrolls = []
        while len(unrolls) < flags.batch_size:
          try:
            unrolls.append(unroll_queue.get(timeout=flags.queue_timeout_secs))
          except queue.Empty:
            raise RuntimeError(
                'learner starved: no unroll for %.0fs (actors alive: %s)' %
                (flags.queue_timeout_secs,
                 [t.is_alive() for t in threads] or 'remote'))
        timer.add_wait(time.time() - t_wait)
        if flags.deterministic:
          # batch order independent of actor timing: sort by actor identity
          unrolls.sort(key=lambda u: (u.level_name, float(u.agent_state[0][0])))
        host = stack_unrolls(unrolls, use_instruction=use_instr, pin=False)
        if faults.get('learner_nan') == steps + 1:
          host.env_outputs.reward[1:, 0] = float('nan')  # poisoned batch
        dev_batch = host
        if learner.popart is not None:
          # PopArt: the device batch carries task indices instead of names
          dev_batch = host._replace(level_name=torch.tensor(
              [task_index[l] for l in host.level_name], dtype=torch.int64))
        with trace('h2d'):
          if device.type == 'cuda':
            # the batch goes into one of two pinned flat buffers and reaches
            # the device (the graph's static slot) with ONE async copy
            if staging is None:
              staging = [FlatStaging(dev_batch, 'cpu', pin=True)
                         for _ in range(2)]
              dev_stage = FlatStaging(dev_batch, device)
              copied = [None, None]
            slot = steps % 2
            if copied[slot] is not None:
              copied[slot].synchronize()  # its previous H2D copy has landed
            staging[slot].load(dev_batch)
            dev_stage.copy_from(staging[slot])
            copied[slot] = torch.cuda.Event()
            copied[slot].record()
            data = dev_stage.views
          else:
            data = batch_to_device(dev_batch, device)
        with trace('learner_step'):
          if use_graph:
            if learner._graph is None:
              learner.capture(data, clone=False)
            loss = learner.graph_step()
          else:
            loss = learner.step(data)
        steps += 1
        if (world > 1 and flags.consistency_check_steps and
            steps % flags.consistency_check_steps == 0):
          if not parallel.param_checksum_consistent(learner.flat.params):
            raise RuntimeError('data-parallel replicas diverged at step %d' %
                               steps)
          checks_ok += 1
        if steps == 1:
          first_loss = float(loss)
        if infer is not None:
          model.publish(learner.flat.params)
        elif transport is not None:
          transport.publish_weights()
        frames = int(learner.frames.item())
        timer.step()
        # episode logging on env_outputs[1:] (experiment.py:372-375, 632-647)
        eo = host.env_outputs
        episode_logger.log_batch(host.level_name, eo.done[1:].numpy(),
                                 eo.info.episode_return[1:].numpy(),
                                 eo.info.episode_step[1:].numpy(), frames)
        host_actions = host.agent_outputs.action[1:].numpy()
      if writer is not None and (time.time() - last_summary >=
                                 flags.save_summaries_secs):
        last_summary = time.time()
        lr = learner.opt.current_lr(frames - learner.frames_per_step)
        scalars = {'learning_rate': lr,
                   'total_loss': float(loss),
                   'frames_per_sec': timer.frames_per_sec(),
                   'learner_steps_per_sec': timer.steps_per_sec(),
                   'queue_wait_frac': timer.wait_fraction(),
                   'env_restarts': (sum(a.env_restarts for a in actors) +
                                    (groups.env_restarts if groups else 0))}
        scalars.update(learner.health())
        if server is not None and server.batches:
          scalars['inference_batch_size_mean'] = (server.rows_served /
                                                  server.batches)
        if infer is not None and infer.stats()['batches']:
          st = infer.stats()
          scalars['inference_batch_size_mean'] = (st['requests'] /
                                                  st['batches'])
        if learner.grad_sync is not None:
          scalars['allreduce_ms'] = 1e3 * learner.grad_sync.last_time_s
        writer.add_scalars(scalars, frames)
        if host_ms:
          scalars['learner_host_ms'] = float(np.median(host_ms[-100:]))
          scalars['learner_loop_host_ms'] = float(np.median(loop_ms[-100:]))
        writer.add_histogram('action', host_actions, frames)
        writer.flush()
      if frames - last_log_frames >= flags.log_every_frames:
        last_log_frames = frames
        log.info('frames %d  %.0f frames/s  %.2f steps/s  loss %.3f  '
                 'queue-wait %.0f%%  learner host %.2f ms/step (data path) '
                 '%.2f ms/step (loop incl. logging)', frames,
                 timer.frames_per_sec(), timer.steps_per_sec(), float(loss),
                 100 * timer.wait_fraction(),
                 float(np.median(host_ms[-100:])) if host_ms else 0.0,
                 float(np.median(loop_ms[-100:])) if loop_ms else 0.0)
        health = learner.health()
        if health['skipped_updates'] > reported_skips:
          # loud, not fatal: the guard already dropped those updates
          log.warning('learner dropped %d update(s) so far (%d LSTM unroll '
                      'timeout(s), %d conv hand-off timeout(s), rest '
                      'non-finite gradients)', health['skipped_updates'],
                      health['lstm_timeouts'], health['conv_timeouts'])
          reported_skips = health['skipped_updates']
      if saver is not None:
        saver.maybe_save()
  except _Terminated:
    log.warning('SIGTERM: stopping and checkpointing at %d frames',
                int(learner.frames.item()))
  except BaseException:
    failed = True
    raise
  finally:
    stop.set()
    if use_traj:
      # every in-flight H2D of a host slab must finish before the slabs are
      # unregistered; after a failure the wait is bounded (a GPU fault may
      # never complete the copies: then the slabs stay registered)
      drained = feeder.drain(10.0 if failed else 600.0)
      tq.close(unregister=drained)
    if infer is not None:
      infer.close()
    if groups is not None:
      for b in board or ():
        b.close()
      groups.close()
      if server is not None:
        server.stop()
      if shared_w is not None:
        shared_w.close()
    for t in threads:
      t.join(timeout=5)
    py_process.close_all(envs)
    if transport is not None:
      transport.close()
    if saver is not None:
      saver.maybe_save(force=True)
    if writer is not None:
      writer.close()
    parallel.cleanup()
  # per-rank summary (data-parallel runs: every rank trains on its OWN
  # actors' unrolls; the replicas stay identical through the all-reduce)
  log.info('rank %d/%d: %d learner steps, %d env frames (all ranks), %d '
           'episodes from this rank\'s actors, %d replica-consistency checks '
           'passed, first loss %.6f', rank, world, steps,
           int(learner.frames.item()), episode_logger.episodes, checks_ok,
           first_loss)
  if server is not None and server.batches:
    # the inference board's serving rate (profiles/r6_e2e.md)
    dt = max(1e-9, time.time() - t_loop0)
    log.info('inference board: %d launches (%.0f/s), %.1f rows per launch, '
             '%.0f rows/s', server.batches, server.batches / dt,
             server.rows_served / server.batches, server.rows_served / dt)
  return learner


# --------------------------------------------------------------- test
def test(flags):
  """Evaluates the latest checkpoint (experiment.py:675-708)."""
  import torch
  from . import checkpoint as ckpt_lib
  from . import inference as inference_lib
  from .actor import Actor

  level_names = level_names_for(flags)
  action_set = action_set_for(flags, level_names[0])
  frame_shape = frame_shape_for(flags, level_names[0])
  use_instr = uses_instruction(flags, level_names)
  envs = [create_environment(flags, l, seed=1, is_test=True)
          for l in level_names]
  py_process.start_all(envs)
  device = _device(flags)
  agent = _make_agent(flags, len(action_set), frame_shape, device, flags.seed)
  path = ckpt_lib.latest_checkpoint(flags.logdir)
  if path is None:
    raise FileNotFoundError('no checkpoint in %s' % flags.logdir)
  model = inference_lib.InferenceModel(agent, device, use_instr)
  ckpt_lib.restore_agent(model.agent, ckpt_lib.load_state(path))
  level_returns = {l: [] for l in level_names}
  try:
    for env, level in zip(envs, level_names):
      log.info('Testing level: %s', level)
      actor = Actor(environments.FlowEnvironment(env), model.infer, level,
                    action_set, flags.unroll_length, len(action_set),
                    use_instruction=use_instr)
      returns = level_returns[level]
      while True:
        out = actor.unroll()
        d = out.env_outputs.done[1:]
        returns.extend(out.env_outputs.info.episode_return[1:][d].tolist())
        if len(returns) >= flags.test_num_episodes:
          log.info('Mean episode return: %f', np.mean(returns))
          break
  finally:
    py_process.close_all(envs)
  if flags.level_name == 'dmlab30':
    no_cap = dmlab30.compute_human_normalized_score(level_returns,
                                                    per_level_cap=None)
    cap_100 = dmlab30.compute_human_normalized_score(level_returns,
                                                     per_level_cap=100)
    log.info('No cap.: %f Cap 100: %f', no_cap, cap_100)
  return level_returns


def main(argv=None):
  # before the first HIP call (and inherited by the env / actor processes
  # forked below): see parallel/streams.py reserve_hw_queues
  from .parallel.streams import reserve_hw_queues
  reserve_hw_queues()
  logging.basicConfig(level=logging.INFO,
                      format='[%(asctime)s %(levelname)s] %(message)s')
  flags = flags_lib.parse_flags(argv if argv is not None else sys.argv[1:])
  if flags.mode == 'train':
    train(flags)
  else:
    test(flags)


if __name__ == '__main__':
  main()
