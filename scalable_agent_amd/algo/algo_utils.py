"""Numerical helpers shared by the env stack and learners (reference
algorithms/utils/algo_utils.py:1-159): RunningMeanStd (parallel-variance
merge), discounted sums and GAE over [T, N] trajectories with episode
terminations, observation-dict helpers and `num_env_steps`.
"""

import numpy as np

EPS = 1e-8


class RunningMeanStd(object):
  """Running mean/variance with Chan et al.'s parallel merge; optionally caps
  the past count so the statistics keep adapting at a fixed rate."""

  def __init__(self, max_past_samples=None, epsilon=1e-4, shape=()):
    self.mean = np.zeros(shape, np.float64)
    self.var = np.ones(shape, np.float64)
    self.count = epsilon
    self.max_past_samples = max_past_samples

  def update(self, x):
    x = np.asarray(x)
    self.update_from_moments(np.mean(x, axis=0), np.var(x, axis=0),
                             x.shape[0])

  def update_from_moments(self, batch_mean, batch_var, batch_count):
    self.mean, self.var, self.count = update_mean_var_count_from_moments(
        self.mean, self.var, self.count, batch_mean, batch_var, batch_count,
        self.max_past_samples)


def update_mean_var_count_from_moments(mean, var, count, batch_mean,
                                       batch_var, batch_count,
                                       max_past_samples=None):
  if max_past_samples is not None:
    count = min(count, max_past_samples)
  delta = batch_mean - mean
  total = count + batch_count
  new_mean = mean + delta * batch_count / total
  m2 = var * count + batch_var * batch_count + \
      np.square(delta) * count * batch_count / total
  return new_mean, m2 / total, total


def maybe_extract_key(data, key):
  if isinstance(data, (list, tuple)) and data and isinstance(data[0], dict):
    return extract_key(data, key) if key in data[0] else None
  if isinstance(data, dict):
    return data.get(key, None)
  return None


def main_observation(data):
  obs = maybe_extract_key(data, 'obs')
  return data if obs is None else obs


def goal_observation(data):
  return maybe_extract_key(data, 'goal')


def extract_keys(list_of_dicts, *keys):
  """List of dicts -> tuple of lists, one per key."""
  return tuple([d[k] for d in list_of_dicts] for k in keys)


def extract_key(list_of_dicts, key):
  return extract_keys(list_of_dicts, key)[0]


def calculate_discounted_sum(x, dones, discount, x_last=None):
  """Backward cumulative sum over a [T, N] trajectory that restarts at
  episode ends: s_t = x_t + discount * s_{t+1} * (1 - done_t)."""
  x = np.asarray(x)
  dones = np.asarray(dones)
  acc = (np.zeros_like(x[0]) if x_last is None
         else np.array(x_last, dtype=np.float32))
  out = np.zeros_like(x)
  for t in range(len(x) - 1, -1, -1):
    acc = x[t] + discount * acc * (1 - dones[t])
    out[t] = acc
  return out


def calculate_gae(rewards, dones, values, gamma, gae_lambda):
  """Generalized Advantage Estimation (Schulman et al. 2016, sec. 3).

  values has one more entry than rewards (the bootstrap).  Returns
  (advantages, discounted returns) as float32.
  """
  rewards = np.asarray(rewards)
  dones = np.asarray(dones)
  values = np.asarray(values)
  assert len(rewards) == len(dones)
  assert len(rewards) + 1 == len(values)
  deltas = rewards + (1 - dones) * (gamma * values[1:]) - values[:-1]
  advantages = calculate_discounted_sum(deltas, dones, gamma * gae_lambda)
  returns = calculate_discounted_sum(rewards, dones, gamma, values[-1])
  return advantages.astype(np.float32), returns.astype(np.float32)


def num_env_steps(infos):
  """Env frames in a batch of experience (`num_frames` per info, else 1)."""
  return sum(info.get('num_frames', 1) for info in infos)


def list_to_string(x, limit=6):
  if len(x) <= limit:
    return str(x)
  return str(x[:3]).replace(']', ',') + ' ... ,' + \
      str(x[-2:]).replace('[', ' ')


def softmax(x):
  ex = np.exp(x - np.max(x))
  return ex / np.sum(ex)


def choice_weighted(arr, logits):
  assert len(arr) == len(logits)
  return np.random.choice(arr, p=softmax(logits))
