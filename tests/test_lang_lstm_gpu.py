"""Fused instruction encoder (csrc/kernels/lang_lstm.hip, ops/lang.py)
against the generic torch encoder in float64 (reference experiment.py:
123-146): output at the last valid word (zeros for an empty instruction)
and the gradients of the embedding table, the LSTM kernel and bias, at a
small ragged shape and at the learner's N = T*B = 3232 frames, 16 words."""

import pytest
import torch

from scalable_agent_amd.models import Agent

pytestmark = pytest.mark.gpu


def _rel(a, b):
  a, b = a.double().cpu(), b.double().cpu()
  return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize('N,L,det', [(37, 5, False), (3232, 16, False),
                                     (3232, 16, True)])
def test_language_lstm_matches_torch(cuda, N, L, det):
  # det: deterministic mode sums dx with a one-hot product instead of the
  # backward kernel's embedding-row atomics
  from scalable_agent_amd import ops
  g = torch.Generator().manual_seed(N + L)
  ids = torch.randint(1, 1000, (N, L), generator=g)
  lengths = torch.randint(0, L + 1, (N,), generator=g)
  ids = ids * (torch.arange(L).view(1, L) < lengths.view(N, 1))
  ref_agent = Agent(9, torso='shallow', seed=3, backend='torch',
                    compute_dtype=torch.float64).double()
  out_ref = ref_agent.instruction_encoding((ids, lengths), N, 'cpu')
  w = torch.randn(out_ref.shape, generator=g, dtype=torch.float64)
  (out_ref * w).sum().backward()
  agent = Agent(9, torso='shallow', seed=3, backend='hip').to(cuda)
  out = ops.language_lstm(ids.to(cuda), lengths.to(cuda), agent.embed,
                          agent.language_lstm_kernel, agent.language_lstm_bias)
  assert out.shape == (N, 64) and out.dtype == torch.float32
  assert _rel(out, out_ref) <= 1e-5
  assert torch.all(out[lengths.to(cuda) == 0] == 0)
  prev = torch.are_deterministic_algorithms_enabled()
  torch.use_deterministic_algorithms(det, warn_only=True)
  try:
    (out * w.float().to(cuda)).sum().backward()
  finally:
    torch.use_deterministic_algorithms(prev)
  for name in ('embed', 'language_lstm_kernel', 'language_lstm_bias'):
    gr = getattr(ref_agent, name).grad
    gh = getattr(agent, name).grad
    assert _rel(gh, gr) <= 1e-5, name


def test_instruction_encoding_routes_to_fused_kernel(cuda):
  """The HIP agent's instruction encoder is the fused kernel (graph-safe:
  no host read of the lengths)."""
  agent = Agent(9, torso='deep', seed=1, backend='hip').to(cuda)
  ids = torch.randint(0, 1000, (64, 16), device=cuda)
  lengths = torch.randint(0, 17, (64,), device=cuda)
  s = torch.cuda.Stream()
  with torch.cuda.stream(s):
    out = agent.instruction_encoding((ids, lengths), 64, cuda)  # warm
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g, stream=s):
    out = agent.instruction_encoding((ids, lengths), 64, cuda)
  g.replay()
  torch.cuda.synchronize()
  assert torch.isfinite(out).all()


def test_language_lstm_clamps_lengths_and_ids(cuda):
  """A length past the word dimension is clamped to L (the output is the
  last step's h, never uninitialised memory) and an out-of-range word id
  reads - and gets the gradient of - embedding row 0, in the forward and
  the backward alike."""
  from scalable_agent_amd import ops
  N, L = 40, 6
  g = torch.Generator().manual_seed(5)
  ids = torch.randint(1, 1000, (N, L), generator=g)
  lengths = torch.randint(0, 2 * L, (N,), generator=g)
  ids_bad = ids.clone()
  ids_bad[::3, 1] = 5000
  ids_bad[1::3, 2] = -7
  ids_ok = torch.where((ids_bad >= 0) & (ids_bad < 1000), ids_bad, 0)
  w = torch.randn(N, 64, generator=g)
  outs, grads = [], []
  for i, l in ((ids_bad, lengths), (ids_ok, lengths.clamp(max=L))):
    agent = Agent(9, torso='shallow', seed=3, backend='hip').to(cuda)
    out = ops.language_lstm(i.to(cuda), l.to(cuda), agent.embed,
                            agent.language_lstm_kernel, agent.language_lstm_bias)
    (out * w.to(cuda)).sum().backward()
    outs.append(out.detach())
    grads.append(agent.embed.grad.clone())
  assert torch.isfinite(outs[0]).all()
  assert torch.equal(outs[0], outs[1])
  assert torch.allclose(grads[0], grads[1], rtol=0, atol=1e-6)
