"""IMPALA learner: re-unroll, V-trace, losses, TF-RMSProp, frame counter.

Semantics follow `build_learner` (experiment.py:346-427):
  1. unroll the agent over all T+1 steps from the unroll-start LSTM state;
  2. bootstrap from baseline[T]; shift agent/env outputs by one step;
  3. clip rewards (abs_one | soft_asymmetric); discounts = (~done) * gamma;
  4. V-trace from logits (rho_bar = c_bar = rho_bar_pg = 1);
  5. loss = PG + baseline_cost * 0.5 sum(adv^2) + entropy_cost * (-sum H);
  6. RMSProp with LR linearly decayed by the env-frame counter;
  7. frames += B * T * repeats * world_size.

MI355X execution: everything runs on the GPU (the reference pins V-trace to
the CPU, experiment.py:386-397).  With the HIP backend the V-trace + loss +
their gradients are one fused kernel, the optimizer is one fused kernel over a
flat parameter buffer, and the whole fwd+bwd+optimizer step is captured into a
HIP graph (torch.cuda.CUDAGraph is hipGraph on ROCm) replayed per step from
static staging slots; the data-parallel gradient sum is one RCCL all-reduce on
the flat gradient buffer.
"""

import os
import time

import torch

from . import losses as losses_lib
from . import vtrace as vtrace_lib
from .optim import FlatParams, RMSProp
from .structs import ActorOutput, AgentOutput, StepOutput, StepOutputInfo
from .utils.tracing import trace
from .utils.knobs import measure_env


def compute_loss(agent, data, flags, use_fused=False, popart=None,
                 aux=None):
  """Total loss for one time-major batch (ActorOutput of tensors).

  popart: optional PopArt; then data.level_name is a [B] task-index tensor,
  values are normalised per task, and the V-trace targets are left in
  aux['targets'] for the post-step statistics update.
  """
  env_outputs = data.env_outputs
  agent_outputs = data.agent_outputs
  instr = env_outputs.observation[1]
  task_ids = data.level_name if popart is not None else None
  if (use_fused and agent.fused_core_ready(instr) and
      agent.num_actions <= 31 and
      agent.num_actions + agent.num_value_heads <= 64 and
      (agent.num_value_heads == 1 or task_ids is not None)):
    # HIP learner path: fused core + fused heads/V-trace/loss; same math.
    # PopArt (multi-task heads, de-normalised V-trace, normalised baseline
    # error and advantages) runs inside the same kernels.
    from . import ops
    core_out, _ = agent.unroll_core(agent_outputs.action, env_outputs,
                                    data.agent_state)
    return ops.heads_vtrace_loss(
        core_out, agent.policy_w, agent.policy_b, agent.baseline_w,
        agent.baseline_b, agent_outputs.policy_logits, agent_outputs.action,
        env_outputs.reward, env_outputs.done, discounting=flags.discounting,
        reward_clipping=flags.reward_clipping,
        baseline_cost=flags.baseline_cost, entropy_cost=flags.entropy_cost,
        task_ids=task_ids, popart=popart,
        aux=aux if popart is not None else None)
  learner_outputs, _ = agent.unroll(agent_outputs.action, env_outputs,
                                    data.agent_state, sample=False,
                                    task_ids=task_ids)
  bootstrap_value = learner_outputs.baseline[-1]

  behaviour_logits = agent_outputs.policy_logits[1:]
  actions = agent_outputs.action[1:]
  rewards = env_outputs.reward[1:]
  done = env_outputs.done[1:]
  target_logits = learner_outputs.policy_logits[:-1]
  values = learner_outputs.baseline[:-1]

  if use_fused and popart is None:
    from . import ops
    return ops.vtrace_loss(
        behaviour_logits, target_logits, actions, rewards, done, values,
        bootstrap_value, discounting=flags.discounting,
        reward_clipping=flags.reward_clipping,
        baseline_cost=flags.baseline_cost, entropy_cost=flags.entropy_cost)

  norm_values = values
  if popart is not None:
    sigma, mu = popart.stats_for(task_ids)          # [B] each, no grad
    values = values * sigma + mu                     # unnormalised
    bootstrap_value = bootstrap_value * sigma + mu

  clipped_rewards = losses_lib.clip_rewards(rewards, flags.reward_clipping)
  discounts = (~done.to(torch.bool)).to(values.dtype) * flags.discounting
  vt = vtrace_lib.from_logits(
      behaviour_policy_logits=behaviour_logits,
      target_policy_logits=target_logits, actions=actions,
      discounts=discounts, rewards=clipped_rewards, values=values,
      bootstrap_value=bootstrap_value)
  pg_advantages = vt.pg_advantages
  if popart is None:
    baseline_err = vt.vs - values
  else:
    baseline_err = (vt.vs - mu) / sigma - norm_values
    pg_advantages = pg_advantages / sigma
    if aux is not None:
      aux['targets'] = vt.vs.detach()
  total = losses_lib.compute_policy_gradient_loss(target_logits, actions,
                                                  pg_advantages)
  total = total + flags.baseline_cost * losses_lib.compute_baseline_loss(
      baseline_err)
  total = total + flags.entropy_cost * losses_lib.compute_entropy_loss(
      target_logits)
  return total


def batch_to_device(data, device, non_blocking=True):
  """Moves a nested ActorOutput of tensors (or None/strings) to `device`."""
  def mv(x):
    if torch.is_tensor(x):
      return x.to(device, non_blocking=non_blocking)
    if isinstance(x, tuple):
      return type(x)(*[mv(e) for e in x]) if hasattr(x, '_fields') else tuple(
          mv(e) for e in x)
    return x
  return mv(data)


class Learner:
  """Owns the agent's flat parameters, optimizer state and frame counter."""

  def __init__(self, agent, flags, device, process_group=None, world_size=1):
    self.flags = flags
    self.device = torch.device(device)
    self.agent = agent.to(self.device)
    self.flat = FlatParams(self.agent)
    use_hip = getattr(agent, 'backend', 'torch') == 'hip'
    self.use_fused = use_hip
    lstm_err = None
    if use_hip and getattr(flags, 'deterministic', False):
      # bf16 torso: per-workgroup weight-gradient slots summed in a fixed
      # order instead of float atomics (the fp32 torso and the learner-head /
      # column-sum reductions always reduce in a fixed order)
      from . import ops
      ops.load().conv_tune('deterministic', 1)
    if use_hip and self.device.type == 'cuda':
      # a cooperative LSTM unroll that timed out skips the update (and is
      # counted) instead of applying gradients of stale activations
      from .ops import lstm as lstm_ops
      lstm_err = lstm_ops.persistent_error_word(self.device)
    # data-parallel mean: the 1/world factor is folded into the update
    # (the all-reduce itself always sums)
    grad_scale = float(getattr(flags, 'grad_scale', 1.0))
    if world_size > 1 and getattr(flags, 'grad_reduce', 'sum') == 'mean':
      grad_scale /= world_size
    self.opt = RMSProp(self.flat, flags.learning_rate, flags.decay,
                       flags.momentum, flags.epsilon,
                       flags.total_environment_frames, use_hip=use_hip,
                       skip_nonfinite=getattr(flags, 'skip_nonfinite', True),
                       lstm_err=lstm_err, grad_scale=grad_scale)
    self.frames = torch.zeros((), dtype=torch.int64, device=self.device)
    self.world_size = world_size
    self.pg = process_group
    self.frames_per_step = (flags.batch_size * flags.unroll_length *
                            flags.num_action_repeats * world_size)
    self.last_loss = None
    self._graph = None
    # graph_step's early all-reduce hand-off: host-side (default) or
    # device-side stream order (SA_EARLY_SYNC=device)
    self._early_host = measure_env('SA_EARLY_SYNC', 'host') != 'device'
    self._early_ev = None
    self._early_stream = None
    self._static_in = None
    self._static_loss = None
    self.grad_sync = None
    self.popart = None
    self._aux = {}
    self._seed_one = None  # backward seed (see _fwd_late)
    # weight-gradient GEMMs on a side stream next to the torso backward
    # (opt-in: measured within run-to-run noise, profiles/experiments.md)
    self._overlap = measure_env('SA_OVERLAP_WGRAD', '0') == '1'
    if getattr(flags, 'popart', False):
      from .popart import PopArt
      self.popart = PopArt(self.agent.num_value_heads, flags.popart_beta,
                           self.device)
    # data-parallel overlap: backward in two phases - heads/core/torso-FC
    # (whose gradients are all-reduced at once, asynchronously) then the
    # conv torso - so the bulk of the all-reduce runs under the torso
    # backward.  Needs the torso parameters at the tail of
    # the flat buffer.
    self._split = False
    self._split_pairs = None
    if world_size > 1:
      from .parallel import GradientSynchronizer
      self.grad_sync = GradientSynchronizer(self.flat, process_group,
                                            reduce='sum')
      off = self._torso_offset()
      if getattr(flags, 'grad_overlap', True) and off is not None:
        self.grad_sync.set_split(off)
        self._split = self.grad_sync.split is not None
      if self.device.type == 'cuda':
        # the early all-reduce's issuing stream, from the fixed stream plan
        # (created here, before any capture, not lazily after it)
        from .parallel.streams import stream_plan
        self._early_stream = stream_plan(self.device).early

  def _torso_offset(self):
    """Flat offset where the conv-torso parameters start, if they are
    exactly the buffer's tail."""
    torso = [o for (n, _), o in zip(self.flat.named, self.flat.offsets)
             if n.startswith('convnet.')]
    other = [o for (n, _), o in zip(self.flat.named, self.flat.offsets)
             if not n.startswith('convnet.')]
    if not torso or not other or min(torso) < max(other):
      return None
    return min(torso)

  # ------------------------------------------------------------ eager step
  def _grad_ctx(self):
    from .ops import grad_sink
    return (grad_sink.direct_grads(self.use_fused),
            grad_sink.overlap_weight_grads(self.use_fused and self._overlap))

  def _fwd_late(self, data):
    """Forward + the backward down to the torso features (all of it when
    not splitting)."""
    self.flat.zero_grad()
    pairs = [] if self._split else None
    self.agent._split_torso = pairs
    try:
      with trace('forward'):
        loss = compute_loss(self.agent, data, self.flags, self.use_fused,
                            self.popart, self._aux)
    finally:
      self.agent._split_torso = None
    with trace('backward'):
      a, b = self._grad_ctx()
      with a, b:
        # a persistent ones seed: loss.backward() would fill a fresh one
        # (a kernel launch in the serial chain of every step)
        one = self._seed_one
        if one is None or one.shape != loss.shape or one.dtype != loss.dtype \
            or one.device != loss.device:
          one = self._seed_one = torch.ones_like(loss)
        loss.backward(one)
    self._split_pairs = pairs
    return loss

  def _bwd_torso(self):
    """Second backward phase: the conv torso from its features' gradient."""
    pairs = self._split_pairs
    if not pairs:
      return
    with trace('backward_torso'):
      a, b = self._grad_ctx()
      with a, b:
        torch.autograd.backward([f for f, _ in pairs],
                                [leaf.grad for _, leaf in pairs])

  def _fwd_bwd(self, data):
    loss = self._fwd_late(data)
    self._bwd_torso()
    self._split_pairs = None
    return loss

  def _apply(self):
    if self.grad_sync is not None:
      if self.opt.lstm_err is not None:
        # a stale LSTM unroll / conv backward on THIS rank poisons the
        # reduced gradient, so every rank's guard skips the same step and
        # the replicas stay identical (the error words are counted locally)
        from . import ops
        s = self.flat.sentinel
        ops.poison_on_error(self.flat.grads[s:s + 1], self.opt.lstm_err)
      with trace('allreduce'):
        self.grad_sync.all_reduce()
    with trace('optimizer'):
      self.opt.step(self.frames)
    if self.popart is not None:
      # data-parallel: every rank applies the same update from its own
      # targets; ranks stay consistent because the statistics are all-reduced
      targets = self._aux['targets']
      tasks = self._popart_tasks
      if self.grad_sync is not None:
        targets, tasks = _gather_targets(targets, tasks)
      self.popart.update(targets, tasks, self.agent.baseline_w.data,
                         self.agent.baseline_b.data)
    self.frames.add_(self.frames_per_step)

  def _begin_early_device_ordered(self):
    """The early bucket's all-reduce, issued from the early stream (its own
    hardware queue) behind a device-side wait on the work enqueued so far on
    the current stream."""
    early = self._early_stream
    if early is None:
      self.grad_sync.begin_early()
      return
    early.wait_stream(torch.cuda.current_stream(self.device))
    with torch.cuda.stream(early):
      self.grad_sync.begin_early()

  def step(self, data):
    """One learner update from a device-resident time-major batch."""
    self._popart_tasks = data.level_name if self.popart is not None else None
    loss = self._fwd_late(data)
    if self._split:
      self._begin_early_device_ordered()  # under the torso backward
    self._bwd_torso()
    self._split_pairs = None
    self.flat.rebind_grads()
    self._apply()
    self.last_loss = loss.detach()
    return self.last_loss

  # ------------------------------------------------------------ graph step
  def capture(self, example, warmup=2, clone=True):
    """Captures fwd+bwd into a HIP graph on static input slots.

    clone=False: `example` (already on the device) IS the static slot, e.g.
    the views of a `FlatStaging` device buffer that one H2D copy refills."""
    assert self.device.type == 'cuda'
    self._static_in = batch_to_device(example, self.device)
    if clone:  # the static slot owns its memory
      self._static_in = _map_tensors(self._static_in, lambda t: t.clone())
    # the process's one capture stream (parallel/streams.py: a new stream per
    # capture would shift which hardware queue every later stream gets)
    from .parallel.streams import stream_plan
    s = stream_plan(self.device).capture
    s.wait_stream(torch.cuda.current_stream(self.device))
    saved_p = self.flat.params.clone()
    with torch.cuda.stream(s):
      for _ in range(warmup):
        self._fwd_bwd(self._static_in)
    torch.cuda.current_stream(self.device).wait_stream(s)
    self.flat.rebind_grads()
    g = torch.cuda.CUDAGraph()
    # thread_local: actor-inference threads keep using the GPU (and the
    # caching allocator) while the learner captures
    mode = measure_env('SA_CAPTURE_MODE', 'thread_local')
    if self._split:
      # two graphs on one pool, replayed in capture order: forward + late
      # backward, then the torso backward (the early all-reduce is launched
      # between the two replays)
      pool = torch.cuda.graph_pool_handle()
      with torch.cuda.graph(g, pool=pool, capture_error_mode=mode):
        self._static_loss = self._fwd_late(self._static_in).detach()
      g2 = torch.cuda.CUDAGraph()
      with torch.cuda.graph(g2, pool=pool, capture_error_mode=mode):
        self._bwd_torso()
      # the features / their gradients live in the pool: keep them
      self._graph_keep = self._split_pairs
      self._split_pairs = None
      self.flat.params.copy_(saved_p)
      self._graph = (g, g2)
      return
    with torch.cuda.graph(g, capture_error_mode=mode):
      # detached: holding the autograd graph would keep its AccumulateGrad
      # nodes (and the streams they were created on) alive into later
      # captures and eager steps
      self._static_loss = self._fwd_bwd(self._static_in).detach()
    self.flat.params.copy_(saved_p)
    self._graph = g

  def load_static(self, data, non_blocking=True):
    _copy_into(self._static_in, data, non_blocking)

  def graph_step(self):
    if self.popart is not None:
      self._popart_tasks = self._static_in.level_name
    if isinstance(self._graph, tuple):
      self._graph[0].replay()
      if self._early_host:
        # the early bucket's all-reduce is enqueued once the host has seen
        # the first graph end, from an idle stream, so the RCCL stream never
        # sits in a device-side wait on the compute stream: a queue blocked
        # on a compute-stream event slows the compute stream's own dispatch
        # (~0.15 ms per learner step on one GPU, tools/micro/step_jitter.py
        # dpA vs dpB).  The torso backward is already enqueued meanwhile
        if self._early_ev is None:
          self._early_ev = torch.cuda.Event()
        if self._early_stream is None:
          from .parallel.streams import stream_plan
          self._early_stream = stream_plan(self.device).early
        self._early_ev.record()
        self._graph[1].replay()
        self._early_ev.synchronize()
        with torch.cuda.stream(self._early_stream):
          self.grad_sync.begin_early()
      else:
        self._begin_early_device_ordered()
        self._graph[1].replay()
    else:
      self._graph.replay()
    self._apply()
    self.last_loss = self._static_loss
    return self._static_loss

  def health(self):
    """{'skipped_updates', 'lstm_timeouts', 'conv_timeouts'} since
    construction (one device read): updates the step guard dropped
    (non-finite gradients, an abandoned LSTM unroll or an expired hand-off
    wait in the fused conv backward) and how many were LSTM / conv
    timeouts."""
    skipped, timeouts, conv_timeouts = self.opt.health()
    return {'skipped_updates': skipped, 'lstm_timeouts': timeouts,
            'conv_timeouts': conv_timeouts}

  # ------------------------------------------------------------ state
  def state_dict(self):
    sd = {'params': self.flat.state_dict(), 'opt': self.opt.state_dict(),
          'frames': int(self.frames.item())}
    if self.popart is not None:
      sd['popart'] = self.popart.state_dict()
    return sd

  def load_state_dict(self, sd):
    self.flat.load_state_dict(sd['params'])
    self.opt.load_state_dict(sd['opt'])
    self.frames.fill_(int(sd['frames']))
    if self.popart is not None and 'popart' in sd:
      self.popart.load_state_dict(sd['popart'])


def _gather_targets(targets, tasks):
  """All ranks' PopArt targets/tasks (so every replica updates identically)."""
  import torch.distributed as dist
  world = dist.get_world_size()
  t_all = [torch.empty_like(targets) for _ in range(world)]
  k_all = [torch.empty_like(tasks) for _ in range(world)]
  dist.all_gather(t_all, targets.contiguous())
  dist.all_gather(k_all, tasks.contiguous())
  return torch.cat(t_all, 1), torch.cat(k_all, 0)


class FlatStaging(object):
  """A learner batch laid out in ONE flat byte buffer (256-B aligned
  segments, one per tensor), with views nested like the batch.

  A pinned host FlatStaging and a device FlatStaging of the same layout turn
  the per-step StagingArea put (reference experiment.py:587-597) into ONE
  hipMemcpyAsync of `nbytes` instead of one copy (and one pinned-pointer
  query) per tensor; the device views can be the graph's static inputs.
  """

  def __init__(self, template, device, pin=False):
    leaves = []
    _map_tensors(template, lambda t: leaves.append(t) or t)
    offs, off = [], 0
    for t in leaves:
      off = (off + 255) // 256 * 256
      offs.append(off)
      off += t.numel() * t.element_size()
    self.nbytes = off
    raw = torch.empty(off + 256, dtype=torch.uint8, device=device)
    if pin:
      raw = raw.pin_memory()
    shift = (-raw.data_ptr()) % 256  # segment offsets are base-relative
    self._raw = raw
    self.flat = raw[shift:shift + max(off, 1)]
    it = iter(range(len(leaves)))

    def view(t):
      o = offs[next(it)]
      nb = t.numel() * t.element_size()
      return self.flat[o:o + nb].view(t.dtype).view(t.shape)

    self.views = _map_tensors(template, view)

  def load(self, batch):
    _copy_into(self.views, batch, False)
    return self

  def copy_from(self, other, non_blocking=True):
    self.flat[:self.nbytes].copy_(other.flat[:other.nbytes],
                                  non_blocking=non_blocking)


def _map_tensors(x, fn):
  if torch.is_tensor(x):
    return fn(x)
  if isinstance(x, tuple):
    vals = [_map_tensors(e, fn) for e in x]
    return type(x)(*vals) if hasattr(x, '_fields') else tuple(vals)
  return x


def _copy_into(dst, src, non_blocking):
  if torch.is_tensor(dst):
    dst.copy_(src, non_blocking=non_blocking)
    return
  if isinstance(dst, tuple):
    for d, s in zip(dst, src):
      _copy_into(d, s, non_blocking)
