"""Port of the reference vtrace_test.py (vtrace_test.py:86-272).

Ground truth is the O(T^2) numpy formula written in paper notation
(vtrace_test.py:44-83); the implementation under test is the PyTorch
reference `scalable_agent_amd.vtrace` (the fused HIP kernel is tested against
it in test_kernels_gpu.py).
"""

import numpy as np
import pytest
import torch

from scalable_agent_amd import vtrace


def _shaped_arange(*shape):
  return np.arange(np.prod(shape), dtype=np.float32).reshape(*shape)


def _softmax(logits):
  return np.exp(logits) / np.sum(np.exp(logits), axis=-1, keepdims=True)


def _ground_truth_calculation(discounts, log_rhos, rewards, values,
                              bootstrap_value, clip_rho_threshold,
                              clip_pg_rho_threshold):
  vs = []
  seq_len = len(discounts)
  rhos = np.exp(log_rhos)
  cs = np.minimum(rhos, 1.0)
  clipped_rhos = rhos
  if clip_rho_threshold:
    clipped_rhos = np.minimum(rhos, clip_rho_threshold)
  clipped_pg_rhos = rhos
  if clip_pg_rho_threshold:
    clipped_pg_rhos = np.minimum(rhos, clip_pg_rho_threshold)
  values_t_plus_1 = np.concatenate([values, bootstrap_value[None, :]], axis=0)
  for s in range(seq_len):
    v_s = np.copy(values[s])
    for t in range(s, seq_len):
      v_s += (np.prod(discounts[s:t], axis=0) * np.prod(cs[s:t], axis=0) *
              clipped_rhos[t] *
              (rewards[t] + discounts[t] * values_t_plus_1[t + 1] - values[t]))
    vs.append(v_s)
  vs = np.stack(vs, axis=0)
  pg_advantages = (clipped_pg_rhos * (rewards + discounts * np.concatenate(
      [vs[1:], bootstrap_value[None, :]], axis=0) - values))
  return vtrace.VTraceReturns(vs=vs, pg_advantages=pg_advantages)


@pytest.mark.parametrize('batch_size', [1, 2])
def test_log_probs_from_logits_and_actions(batch_size):
  seq_len, num_actions = 7, 3
  policy_logits = _shaped_arange(seq_len, batch_size, num_actions) + 10
  actions = np.random.randint(0, num_actions, size=(seq_len, batch_size),
                              dtype=np.int32)
  out = vtrace.log_probs_from_logits_and_actions(
      torch.tensor(policy_logits), torch.tensor(actions))
  mask = actions[..., None] == np.arange(num_actions)
  gt = np.log(_softmax(policy_logits))[mask].reshape(seq_len, batch_size)
  np.testing.assert_allclose(gt, out.numpy(), rtol=1e-6, atol=1e-6)


def _vtrace_values(batch_size, seq_len=5):
  log_rhos = _shaped_arange(seq_len, batch_size) / (batch_size * seq_len)
  log_rhos = 5 * (log_rhos - 0.5)  # [-2.5, 2.5)
  return {
      'log_rhos': log_rhos,
      'discounts': np.array([[0.9 / (b + 1) for b in range(batch_size)]
                             for _ in range(seq_len)], dtype=np.float32),
      'rewards': _shaped_arange(seq_len, batch_size),
      'values': _shaped_arange(seq_len, batch_size) / batch_size,
      'bootstrap_value': _shaped_arange(batch_size) + 1.0,
      'clip_rho_threshold': 3.7,
      'clip_pg_rho_threshold': 2.2,
  }


@pytest.mark.parametrize('batch_size', [1, 5])
def test_vtrace(batch_size):
  values = _vtrace_values(batch_size)
  out = vtrace.from_importance_weights(
      **{k: (torch.tensor(v) if isinstance(v, np.ndarray) else v)
         for k, v in values.items()})
  gt = _ground_truth_calculation(**values)
  np.testing.assert_allclose(gt.vs, out.vs.numpy(), rtol=1e-5, atol=1e-5)
  np.testing.assert_allclose(gt.pg_advantages, out.pg_advantages.numpy(),
                             rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize('batch_size', [1, 2])
def test_vtrace_from_logits(batch_size):
  seq_len, num_actions = 5, 3
  values = {
      'behaviour_policy_logits': _shaped_arange(seq_len, batch_size,
                                                num_actions),
      'target_policy_logits': _shaped_arange(seq_len, batch_size, num_actions),
      'actions': np.random.randint(0, num_actions - 1,
                                   size=(seq_len, batch_size)),
      'discounts': np.array([[0.9 / (b + 1) for b in range(batch_size)]
                             for _ in range(seq_len)], dtype=np.float32),
      'rewards': _shaped_arange(seq_len, batch_size),
      'values': _shaped_arange(seq_len, batch_size) / batch_size,
      'bootstrap_value': _shaped_arange(batch_size) + 1.0,
  }
  t = {k: torch.tensor(v) for k, v in values.items()}
  out = vtrace.from_logits(clip_rho_threshold=None, clip_pg_rho_threshold=None,
                           **t)
  tlp = vtrace.log_probs_from_logits_and_actions(t['target_policy_logits'],
                                                 t['actions'])
  blp = vtrace.log_probs_from_logits_and_actions(t['behaviour_policy_logits'],
                                                 t['actions'])
  log_rhos = tlp - blp
  iw = vtrace.from_importance_weights(
      log_rhos=log_rhos, discounts=t['discounts'], rewards=t['rewards'],
      values=t['values'], bootstrap_value=t['bootstrap_value'],
      clip_rho_threshold=None, clip_pg_rho_threshold=None)
  torch.testing.assert_close(iw.vs, out.vs)
  torch.testing.assert_close(iw.pg_advantages, out.pg_advantages)
  torch.testing.assert_close(blp, out.behaviour_action_log_probs)
  torch.testing.assert_close(tlp, out.target_action_log_probs)
  torch.testing.assert_close(log_rhos, out.log_rhos)


def test_higher_rank_inputs_for_importance_weights():
  T, B = 4, 3
  out = vtrace.from_importance_weights(
      log_rhos=torch.zeros(T, B, 1), discounts=torch.ones(T, B, 1) * 0.9,
      rewards=torch.randn(T, B, 42), values=torch.randn(T, B, 42),
      bootstrap_value=torch.randn(B, 42))
  assert out.vs.shape[-1] == 42


def test_inconsistent_rank_inputs_for_importance_weights():
  T, B = 4, 3
  with pytest.raises(ValueError, match='must have rank 2'):
    vtrace.from_importance_weights(
        log_rhos=torch.zeros(T, B, 1), discounts=torch.ones(T, B, 1),
        rewards=torch.randn(T, B, 42), values=torch.randn(T, B, 42),
        bootstrap_value=torch.randn(B))


def test_long_sequence_scan_matches_serial():
  """The O(log T) affine scan equals the serial recursion at T=100."""
  torch.manual_seed(0)
  T, B = 101, 7
  a = torch.rand(T, B)
  d = torch.randn(T, B)
  out = vtrace._reverse_affine_scan(a, d)
  acc = torch.zeros(B)
  ref = torch.zeros(T, B)
  for t in reversed(range(T)):
    acc = d[t] + a[t] * acc
    ref[t] = acc
  torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
