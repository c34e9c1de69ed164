"""Action distributions for Discrete and Tuple-of-Discrete action spaces
(reference algorithms/utils/action_distributions.py:1-201; its
`MemActionSpace` import targets a module missing from the reference, so that
branch is dropped).

`CategoricalActionDistribution` normalises raw logits with log-softmax and
adds a symmetric KL to a prior (uniform by default) and to another
distribution.  `TupleActionDistribution` treats sub-spaces as independent
heads over one flat logits tensor: log-prob, entropy and KL are sums over
heads; sub-spaces outside `mask` get uniform logits.
"""

import torch
from torch.distributions import Categorical
from torch.nn import functional as F

from ..envs.gym_compat import Discrete, Tuple
from ..utils.utils import log


def calc_num_logits(action_space):
  if isinstance(action_space, Discrete):
    return action_space.n
  if isinstance(action_space, Tuple):
    return sum(calc_num_logits(s) for s in action_space.spaces)
  raise NotImplementedError('Action space type %s not supported!' %
                            type(action_space))


def get_action_distribution(action_space, raw_logits, mask=None):
  assert calc_num_logits(action_space) == raw_logits.shape[-1]
  if isinstance(action_space, Discrete):
    return CategoricalActionDistribution(raw_logits)
  if isinstance(action_space, Tuple):
    return TupleActionDistribution(action_space, logits_flat=raw_logits,
                                   mask=mask)
  raise NotImplementedError('Action space type %s not supported!' %
                            type(action_space))


def sample_actions_log_probs(distribution):
  if isinstance(distribution, TupleActionDistribution):
    return distribution.sample_actions_log_probs()
  actions = distribution.sample()
  return actions, distribution.log_prob(actions)


class CategoricalActionDistribution(Categorical):

  def __init__(self, raw_logits, prior_probs=None):
    super().__init__(logits=F.log_softmax(raw_logits, dim=-1))
    n = raw_logits.shape[-1]
    if prior_probs is None:
      self.prior_probs = torch.full((n,), 1.0 / n, device=raw_logits.device)
    else:
      self.prior_probs = torch.as_tensor(prior_probs, dtype=torch.float32,
                                         device=raw_logits.device)
    self.log_prior_probs = self.prior_probs.log()

  def _kl(self, other_log_probs):
    return (self.probs * (self.logits - other_log_probs)).sum(-1)

  def _kl_inverse(self, other_log_probs):
    return (other_log_probs.exp() * (other_log_probs - self.logits)).sum(-1)

  def _kl_symmetric(self, other_log_probs):
    return 0.5 * (self._kl(other_log_probs) +
                  self._kl_inverse(other_log_probs))

  def kl_prior(self):
    return self._kl_symmetric(self.log_prior_probs)

  def kl_divergence(self, other):
    return self._kl_symmetric(other.logits)

  def dbg_print(self):
    stats = dict(entropy=self.entropy().mean(), kl_prior=self.kl_prior().mean(),
                 min_logit=self.logits.min(), max_logit=self.logits.max(),
                 min_prob=self.probs.min(), max_prob=self.probs.max())
    log.debug(' '.join('%s=%.3f' % (k, v.item()) for k, v in stats.items()))


class TupleActionDistribution(object):

  def __init__(self, action_space, logits_flat, mask=None):
    self.logit_lengths = [calc_num_logits(s) for s in action_space.spaces]
    self.split_logits = torch.split(logits_flat, self.logit_lengths, dim=1)
    assert len(self.split_logits) == len(action_space.spaces)
    self.distributions = []
    for i, space in enumerate(action_space.spaces):
      logits = self.split_logits[i]
      if mask is not None and i not in mask:
        logits = torch.ones_like(logits)
      self.distributions.append(get_action_distribution(space, logits))

  @staticmethod
  def _flatten_actions(list_of_action_batches):
    return torch.stack(list_of_action_batches, dim=1)

  def _calc_log_probs(self, list_of_action_batches):
    lps = [d.log_prob(a) for d, a in zip(self.distributions,
                                         list_of_action_batches)]
    return torch.stack(lps, dim=1).sum(dim=1)

  def sample_actions_log_probs(self):
    batches = [d.sample() for d in self.distributions]
    return self._flatten_actions(batches), self._calc_log_probs(batches)

  def sample(self):
    return self._flatten_actions([d.sample() for d in self.distributions])

  def log_prob(self, actions):
    batches = [a.squeeze(1) for a in torch.chunk(actions,
                                                 len(self.distributions), 1)]
    return self._calc_log_probs(batches)

  def entropy(self):
    return torch.stack([d.entropy() for d in self.distributions], 1).sum(1)

  def kl_prior(self):
    return torch.stack([d.kl_prior() for d in self.distributions], 1).sum(1)

  def kl_divergence(self, other):
    return torch.stack([d.kl_divergence(o) for d, o in
                        zip(self.distributions, other.distributions)],
                       1).sum(1)

  def dbg_print(self):
    for d in self.distributions:
      d.dbg_print()
