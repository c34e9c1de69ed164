"""Fused V-trace + IMPALA loss (csrc/kernels/vtrace_loss.hip).

Forward computes the loss sums AND the analytic gradients w.r.t. the target
logits and the values in the same launch (V-trace targets are stop-gradient,
vtrace.py:279-280), so backward is a scale by the incoming grad.
"""

import torch

from ._ext import ext, check_cuda

_CLIP = {'abs_one': 0, 'soft_asymmetric': 1}


def _prep(behaviour_logits, target_logits, actions, rewards, done, values,
          bootstrap):
  f = lambda t: t.detach().to(torch.float32).contiguous()
  return (f(behaviour_logits), f(target_logits),
          actions.detach().to(torch.int64).contiguous(), f(rewards),
          done.detach().to(torch.bool).contiguous(), f(values), f(bootstrap))


def vtrace_fused_forward(behaviour_logits, target_logits, actions, rewards,
                         done, values, bootstrap, discounting=0.99,
                         reward_clipping='abs_one', baseline_cost=0.5,
                         entropy_cost=0.00025, clip_rho=1.0, clip_pg_rho=1.0,
                         want_targets=True):
  """Raw kernel call: returns (loss[4], dlogits, dvalues[, vs, pg_adv])."""
  args = _prep(behaviour_logits, target_logits, actions, rewards, done, values,
               bootstrap)
  check_cuda(*args)
  inf = float('inf')
  return ext().vtrace_loss(
      *args, float(discounting), _CLIP[reward_clipping],
      inf if clip_rho is None else float(clip_rho),
      inf if clip_pg_rho is None else float(clip_pg_rho),
      float(baseline_cost), float(entropy_cost), bool(want_targets))


class _VTraceLoss(torch.autograd.Function):

  @staticmethod
  def forward(ctx, target_logits, values, behaviour_logits, actions, rewards,
              done, bootstrap, cfg):
    out = vtrace_fused_forward(behaviour_logits, target_logits, actions,
                               rewards, done, values, bootstrap,
                               want_targets=False, **cfg)
    loss, dlogits, dvalues = out[0], out[1], out[2]
    ctx.save_for_backward(dlogits, dvalues)
    ctx.logits_dtype = target_logits.dtype
    ctx.values_dtype = values.dtype
    return loss[0]

  @staticmethod
  def backward(ctx, g):
    dlogits, dvalues = ctx.saved_tensors
    return ((dlogits * g).to(ctx.logits_dtype),
            (dvalues * g).to(ctx.values_dtype),
            None, None, None, None, None, None)


def vtrace_loss(behaviour_logits, target_logits, actions, rewards, done,
                values, bootstrap, discounting=0.99, reward_clipping='abs_one',
                baseline_cost=0.5, entropy_cost=0.00025):
  """Total IMPALA loss (sum reductions) with fused analytic backward."""
  cfg = dict(discounting=discounting, reward_clipping=reward_clipping,
             baseline_cost=baseline_cost, entropy_cost=entropy_cost)
  return _VTraceLoss.apply(target_logits, values, behaviour_logits, actions,
                           rewards, done, bootstrap, cfg)
