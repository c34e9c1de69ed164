"""Exact-fp32 MFMA GEMM (csrc/kernels/gemm_f32.hip) vs a float64 oracle.

Every learner product of the fused fp32 core (ops/core.py _CoreLSTMF32):
the torso FC with bias + ReLU + the core-input columns (reference
experiment.py:185-198), the LSTM input projection, the masked data
gradients and the split-K weight gradients with the ones-row bias gradient,
at the learner's shapes (N = 3232) and at ragged small shapes.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
  from scalable_agent_amd import ops
  return ops.ext()


def _rel(a, ref):
  a = a.detach().double().cpu()
  ref = ref.detach().double().cpu()
  return (a - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)


def _op(t, tr):
  return t.t() if tr else t


@pytest.mark.parametrize('M,N,K', [(3232, 256, 3456), (3232, 1024, 272),
                                   (3232, 256, 1024), (3232, 3456, 256),
                                   (256, 1024, 3232), (272, 1024, 3232),
                                   (3456, 256, 3232), (36, 44, 28), (8, 4, 4)])
@pytest.mark.parametrize('ta,tb', [(False, False), (False, True), (True, False)])
def test_gemm_f32_plain(cuda, M, N, K, ta, tb):
  if M * N * K > 4e9 and (ta, tb) != (False, False):
    pytest.skip('one layout per large shape is enough')
  g = torch.Generator().manual_seed(M + N + K)
  A = torch.randn(*((K, M) if ta else (M, K)), generator=g)
  B = torch.randn(*((N, K) if tb else (K, N)), generator=g)
  ref = _op(A.double(), ta) @ _op(B.double(), tb)
  C = torch.empty(M, N, device=cuda)
  _C().gemm_f32(A.to(cuda), B.to(cuda), ta, tb, C)
  assert _rel(C, ref) <= 2e-6


def test_gemm_f32_fc_epilogue(cuda):
  """relu(feats W + b) with the [clip(r), one_hot(a), 0...] columns."""
  g = torch.Generator().manual_seed(1)
  M, K, N, ld, A_ = 3232, 3456, 256, 272, 9
  x = torch.randn(M, K, generator=g).clamp(min=0)
  w = torch.randn(K, N, generator=g) / K ** 0.5
  b = torch.randn(N, generator=g)
  r = torch.randn(M, generator=g) * 3
  a = torch.randint(0, A_, (M,), generator=g)
  ref = torch.zeros(M, ld, dtype=torch.float64)
  ref[:, :N] = (x.double() @ w.double() + b.double()).clamp(min=0)
  ref[:, N] = r.double().clamp(-1, 1)
  ref[torch.arange(M), N + 1 + a] = 1.0
  out = torch.full((M, ld), float('nan'), device=cuda)
  _C().gemm_f32(x.to(cuda), w.to(cuda), False, False, out, bias=b.to(cuda),
                relu=True, aug_reward=r.to(cuda), aug_action=a.to(cuda))
  assert _rel(out[:, :N], ref[:, :N]) <= 2e-6
  assert torch.equal(out[:, N:].cpu().double(), ref[:, N:])


def test_gemm_f32_masked_and_weight_grads(cuda):
  """dh = (dG W^T) * (h > 0) and dW += X^T dh with db += colsum(dh)."""
  g = torch.Generator().manual_seed(2)
  M, K, N = 3232, 1024, 256
  dG = torch.randn(M, K, generator=g)
  W = torch.randn(N, K, generator=g) / K ** 0.5
  h = torch.randn(M, 272, generator=g)
  dh_ref = (dG.double() @ W.double().t()) * (h[:, :N].double() > 0)
  dh = torch.empty(M, N, device=cuda)
  hc = h.to(cuda)
  _C().gemm_f32(dG.to(cuda), W.to(cuda), False, True, dh, mask=hc[:, :N])
  assert _rel(dh, dh_ref) <= 2e-6
  X = torch.randn(M, 3456, generator=g)
  dw0 = torch.randn(3456, N, generator=g)
  db0 = torch.randn(N, generator=g)
  dw, db = dw0.to(cuda), db0.to(cuda)
  _C().gemm_f32(X.to(cuda), dh, True, False, dw, accumulate=True, colsum=db)
  dhd = dh.double().cpu()
  assert _rel(dw, dw0.double() + X.double().t() @ dhd) <= 2e-6
  assert _rel(db, db0.double() + dhd.sum(0)) <= 2e-6
  # a column slice of a wider matrix as the transposed A operand
  dwx = torch.zeros(272, K, device=cuda)
  dbx = torch.zeros(K, device=cuda)
  _C().gemm_f32(hc[:, :272], dG.to(cuda), True, False, dwx, accumulate=True,
                colsum=dbx)
  assert _rel(dwx, h.double().t() @ dG.double()) <= 2e-6
  assert _rel(dbx, dG.double().sum(0)) <= 2e-6


def test_gemm_f32_deterministic(cuda):
  g = torch.Generator().manual_seed(3)
  X = torch.randn(3232, 3456, generator=g).to(cuda)
  dh = torch.randn(3232, 256, generator=g).to(cuda)
  outs = []
  for _ in range(2):
    dw = torch.zeros(3456, 256, device=cuda)
    db = torch.zeros(256, device=cuda)
    _C().gemm_f32(X, dh, True, False, dw, accumulate=True, colsum=db)
    outs.append((dw, db))
  assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize('M,N,K', [(256, 1024, 14), (272, 1024, 707), (256, 256, 3233)])
def test_gemm_f32_weight_grad_any_k(cuda, M, N, K):
  """op(A) = A^T, op(B) = B (the weight-gradient form, K = T*B rows) takes
  any K: a data-parallel rank's B*(T+1) need not be a multiple of 4 (two
  ranks of the 4-row dp_check batch: 7 * 2 = 14); the split-K tail chunk is
  row-masked."""
  g = torch.Generator().manual_seed(M + N + K)
  A = torch.randn(K, M, generator=g)
  B = torch.randn(K, N, generator=g)
  ref = A.double().t() @ B.double()
  C = torch.zeros(M, N, device=cuda)
  db = torch.zeros(N, device=cuda)
  _C().gemm_f32(A.to(cuda), B.to(cuda), True, False, C, accumulate=True, colsum=db)
  assert _rel(C, ref) <= 2e-6
  assert _rel(db, B.double().sum(0)) <= 2e-6
