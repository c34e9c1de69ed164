"""IMPALA losses (reference experiment.py:324-343, 377-407).

All reductions are SUMS over T x B, exactly as in the reference.  These are the
pure-PyTorch semantic versions; the learner uses the fused HIP
V-trace+loss kernel (`ops.vtrace_loss`) which returns the same scalars and
analytic gradients.
"""

import torch


def compute_baseline_loss(advantages):
  # 0.5 * sum(adv^2): d(loss)/d(baseline) = -advantage (experiment.py:324-328).
  return .5 * torch.sum(advantages ** 2)


def compute_entropy_loss(logits):
  policy = torch.softmax(logits, dim=-1)
  log_policy = torch.log_softmax(logits, dim=-1)
  entropy_per_timestep = torch.sum(-policy * log_policy, dim=-1)
  return -torch.sum(entropy_per_timestep)


def compute_policy_gradient_loss(logits, actions, advantages):
  cross_entropy = torch.nn.functional.cross_entropy(
      logits.reshape(-1, logits.shape[-1]), actions.reshape(-1).long(),
      reduction='none').view_as(advantages)
  return torch.sum(cross_entropy * advantages.detach())


def clip_rewards(rewards, mode):
  """Reward clipping for the loss (experiment.py:377-382)."""
  if mode == 'abs_one':
    return torch.clamp(rewards, -1, 1)
  elif mode == 'soft_asymmetric':
    squeezed = torch.tanh(rewards / 5.0)
    # Negative rewards are given less weight than positive rewards.
    return torch.where(rewards < 0, .3 * squeezed, squeezed) * 5.
  raise ValueError('unknown reward_clipping %r' % mode)
