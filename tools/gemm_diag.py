import sys, torch
sys.path.insert(0, '.')
from scalable_agent_amd import ops
C_ = ops.ext()
cuda = torch.device('cuda')
for (M, N, K) in [(3232, 256, 3456), (3232, 1024, 272), (3232, 256, 1024), (256, 1024, 3232), (36, 44, 28)]:
  for ta, tb in [(False, False), (False, True), (True, False), (True, True)]:
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(*((K, M) if ta else (M, K)), generator=g)
    B = torch.randn(*((N, K) if tb else (K, N)), generator=g)
    ref = (A.double().t() if ta else A.double()) @ (B.double().t() if tb else B.double())
    C = torch.empty(M, N, device=cuda)
    C_.gemm_f32(A.to(cuda), B.to(cuda), ta, tb, C)
    d = (C.cpu().double() - ref).abs()
    bad = (d > 1e-4 * ref.abs().max()).nonzero()
    rows = sorted(set(bad[:, 0].tolist()))
    cols = sorted(set(bad[:, 1].tolist()))
    print(M, N, K, ta, tb, 'bad', bad.shape[0], 'rows', rows[:5], '..', rows[-3:] if rows else '', 'ncols', len(cols), cols[:5], flush=True)
