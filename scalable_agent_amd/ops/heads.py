"""Fused policy/baseline heads + V-trace + IMPALA loss (HIP learner path).

Reference: heads experiment.py:200-210; learner loss :360-407 (bootstrap from
the last baseline, one-step time shift, reward clipping, discounts, V-trace
from logits vtrace.py:71-161, PG + baseline + entropy losses :324-343).

Forward: ONE kernel (learner_head_fwd, a workgroup per batch column) computes
the heads for all T+1 steps, V-trace, the loss sums and the analytic
gradients w.r.t. the logits/values.  Backward: ONE kernel (learner_head_bwd)
scales them by the incoming loss gradient, maps them through the heads
(dcore) and accumulates the heads' weight/bias gradients (ops.grad_sink).
Multi-task PopArt (K value heads, per-column task index, de-normalised
V-trace, normalised baseline error and scaled advantages) runs in the same
two kernels; the PopArt statistics update stays a few device tensor ops
(popart.py).
"""

import torch

from . import grad_sink
from ._ext import ext

_CLIP = {'abs_one': 0, 'soft_asymmetric': 1}
_TICKETS = {}


def _ticket(device):
  """Per-device completion counter of the fwd kernel (self-resetting)."""
  t = _TICKETS.get(device)
  if t is None:
    t = torch.zeros(1, dtype=torch.int32, device=device)
    _TICKETS[device] = t
  return t


class _HeadsVTraceLoss(torch.autograd.Function):

  @staticmethod
  def forward(ctx, core, wp, bp, wb, bb, behaviour, actions, rewards, done,
              cfg, task, mu, nu, aux):
    outs = ext().learner_head_fwd(
        core, wp, bp, wb.reshape(-1), bb.reshape(-1), behaviour, actions,
        rewards, done, _ticket(core.device), cfg['discounting'],
        _CLIP[cfg['reward_clipping']], 1.0, 1.0, cfg['baseline_cost'],
        cfg['entropy_cost'], task=task, mu=mu, nu=nu,
        want_vs=aux is not None)
    loss, dl, dv = outs[:3]
    if aux is not None:
      aux['targets'] = outs[3]
    ctx.task = task
    ctx.save_for_backward(core, dl, dv, wp, bp, wb, bb)
    return loss[0]

  @staticmethod
  def backward(ctx, g):
    core, dl, dv, wp, bp, wb, bb = ctx.saved_tensors
    (gwp, gbp, gwb, gbb), direct = grad_sink.sinks([wp, bp, wb, bb])
    gs = g.reshape(1).to(torch.float32).contiguous()
    dcore = ext().learner_head_bwd(gs, core, dl, dv, wp, wb.reshape(-1), gwp,
                                   gbp, gwb.view(-1), gbb.view(-1),
                                   task=ctx.task)
    return (dcore,) + grad_sink.returned((gwp, gbp, gwb, gbb), direct) + (
        None,) * 9


def heads_vtrace_loss(core_out, policy_w, policy_b, baseline_w, baseline_b,
                      behaviour_logits, actions, rewards, done, discounting,
                      reward_clipping, baseline_cost, entropy_cost,
                      task_ids=None, popart=None, aux=None):
  """core_out [T+1,B,256] f32 from the learner unroll; behaviour_logits /
  actions / rewards / done: the FULL [T+1,B,...] batch tensors (rows 1..T
  are used, as in experiment.py:360-375).  Returns the total loss (sum).

  Multi-task value heads: baseline_w [256, K], baseline_b [K] and task_ids
  [B] (the head of each batch column).  popart: a PopArt whose mu / nu
  de-normalise the values inside the kernel (popart.py); aux: a dict that
  receives 'targets' = the V-trace targets vs [T, B] for its update."""
  cfg = dict(discounting=float(discounting), reward_clipping=reward_clipping,
             baseline_cost=float(baseline_cost),
             entropy_cost=float(entropy_cost))
  task = None if task_ids is None else task_ids.to(torch.int64).contiguous()
  mu = nu = None
  if popart is not None:
    mu, nu = popart.mu, popart.nu
  return _HeadsVTraceLoss.apply(
      core_out.contiguous(), policy_w, policy_b, baseline_w, baseline_b,
      behaviour_logits.to(torch.float32).contiguous(),
      actions.to(torch.int64).contiguous(),
      rewards.to(torch.float32).contiguous(),
      done.to(torch.bool).contiguous(), cfg, task, mu, nu, aux)


class PhiloxStream(object):
  """(seed, offset) counter for the actor sampler: every call draws from a
  fresh Philox4x32-10 counter block, so samples never repeat and a run is
  reproducible from its seed (the device-side analogue of a torch
  Generator).  With `device`, the offset lives in device memory and the
  sampler advances it on the device, so a captured inference graph draws new
  samples on every replay.  The device counter is the pair {offset, waves
  done} that the sampler kernel itself moves to the next offset (no separate
  increment kernel per step)."""

  def __init__(self, seed, device=None):
    self.seed = int(seed) & ((1 << 63) - 1)
    self.offset = 0
    self.counter = (None if device is None else
                    torch.zeros(2, dtype=torch.int64, device=device))

  @property
  def device_offset(self):
    """The device counter's offset (host read; tests and checkpoints)."""
    return int(self.counter[0].item())

  def manual_seed(self, seed):
    self.seed = int(seed) & ((1 << 63) - 1)
    self.offset = 0
    if self.counter is not None:
      self.counter.zero_()
    return self

  def next_offset(self):
    o = self.offset
    self.offset += 1
    return o


def actor_heads_sample(core_out, policy_w, policy_b, baseline_w, baseline_b,
                       stream):
  """Actor inference heads + sampling in one kernel (actor_io.hip):
  core_out [B,256] f32 -> (action [B] int64, logits [B,A], baseline [B]).
  `stream`: a PhiloxStream (advanced by one)."""
  args = (core_out.float().contiguous(), policy_w.contiguous(),
          policy_b.contiguous(), baseline_w.reshape(-1).contiguous(),
          baseline_b.reshape(-1).contiguous(), stream.seed)
  if stream.counter is not None and stream.counter.device == core_out.device:
    logits, baseline, action = ext().actor_head_sample(*args, 0,
                                                       stream.counter)
  else:
    logits, baseline, action = ext().actor_head_sample(*args,
                                                       stream.next_offset())
  return action, logits, baseline
