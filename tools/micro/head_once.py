"""Runs the fused learner-head fwd kernel a few times (for rocprofv3 --pmc)."""
import sys
import torch
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__)))))
from scalable_agent_amd import ops  # noqa: E402

C = ops.load()
d = torch.device('cuda')
A, B, T = 9, 32, int(sys.argv[1]) if len(sys.argv) > 1 else 100
T1 = T + 1
args = [torch.randn(T1, B, 256, device=d), torch.randn(256, A, device=d),
        torch.randn(A, device=d), torch.randn(256, device=d),
        torch.randn(1, device=d), torch.randn(T1, B, A, device=d),
        torch.randint(0, A, (T1, B), device=d), torch.randn(T1, B, device=d),
        torch.zeros(T1, B, dtype=torch.bool, device=d),
        torch.zeros(1, dtype=torch.int32, device=d)]
for _ in range(3):
  C.learner_head_fwd(*args, 0.99, 0, 1.0, 1.0, 0.5, 0.01)
torch.cuda.synchronize()
print('ok')
