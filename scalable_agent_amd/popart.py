"""PopArt multi-task value normalisation (Hessel et al. 2019, "Multi-task
Deep Reinforcement Learning with PopArt"; north-star config #4 in SURVEY.md
§5.6 - absent from the reference, which has a single unnormalised baseline).

The value head has one output per task (level).  Its outputs are NORMALISED
values n; the unnormalised value of task k is sigma_k * n + mu_k.  Per step:
  * V-trace runs on unnormalised values (targets vs, advantages);
  * baseline loss 0.5 * sum(((vs - mu)/sigma - n)^2), policy-gradient
    advantages divided by sigma (scale-invariant across tasks);
  * after the optimizer step, mu/nu (first/second moments of vs per task,
    exponential moving averages with step size beta) are updated and the
    value-head column of each updated task is rescaled so its unnormalised
    outputs are preserved exactly ("Preserving Outputs"):
        w_k <- w_k * sigma_k / sigma'_k
        b_k <- (sigma_k * b_k + mu_k - mu'_k) / sigma'_k
All of it is device tensor math (no host sync), so it sits inside the
learner's captured step.
"""

import torch

SIGMA_MIN = 1e-4
SIGMA_MAX = 1e6


class PopArt(object):

  def __init__(self, num_tasks, beta=3e-4, device='cpu'):
    self.num_tasks = int(num_tasks)
    self.beta = float(beta)
    self.mu = torch.zeros(self.num_tasks, device=device)
    self.nu = torch.ones(self.num_tasks, device=device)

  def sigma(self):
    var = (self.nu - self.mu * self.mu).clamp(min=SIGMA_MIN ** 2)
    return var.sqrt().clamp(SIGMA_MIN, SIGMA_MAX)

  def stats_for(self, task_ids):
    """-> (sigma, mu) gathered for a [B] tensor of task indices."""
    return self.sigma()[task_ids], self.mu[task_ids]

  @torch.no_grad()
  def update(self, targets, task_ids, value_w, value_b):
    """targets: [T, B] V-trace vs; task_ids: [B]; value_w: [H, K] and
    value_b: [K] are updated in place to preserve outputs."""
    T = targets.shape[0]
    t = targets.float()
    k = task_ids.long()
    cnt = torch.zeros(self.num_tasks, device=t.device).index_add_(
        0, k, torch.full_like(k, T, dtype=torch.float32))
    s1 = torch.zeros(self.num_tasks, device=t.device).index_add_(
        0, k, t.sum(0))
    s2 = torch.zeros(self.num_tasks, device=t.device).index_add_(
        0, k, (t * t).sum(0))
    seen = cnt > 0
    denom = cnt.clamp(min=1)
    # beta-weighted EMA of the per-task batch moments (tasks absent from the
    # batch keep their statistics)
    b = torch.where(seen, torch.full_like(cnt, self.beta), torch.zeros_like(cnt))
    old_sigma, old_mu = self.sigma(), self.mu.clone()
    self.mu.mul_(1 - b).add_(b * s1 / denom)
    self.nu.mul_(1 - b).add_(b * s2 / denom)
    new_sigma = self.sigma()
    value_w.mul_(old_sigma / new_sigma)
    value_b.mul_(old_sigma).add_(old_mu - self.mu).div_(new_sigma)

  def state_dict(self):
    return {'mu': self.mu.detach().clone(), 'nu': self.nu.detach().clone()}

  def load_state_dict(self, sd):
    self.mu.copy_(sd['mu'].to(self.mu.device))
    self.nu.copy_(sd['nu'].to(self.nu.device))
