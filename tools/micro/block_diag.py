import sys, torch
sys.path.insert(0, '.')
from scalable_agent_amd import ops
C_ = ops.load()
d = torch.device('cuda')
for (C, H, W) in [(16, 36, 48), (32, 18, 24), (16, 10, 14)]:
  torch.manual_seed(C + H)
  x = torch.randn(3, H, W, C, device=d).to(torch.bfloat16)
  w1 = torch.randn(3, 3, C, C, device=d) * 0.2
  w2 = torch.randn(3, 3, C, C, device=d) * 0.2
  b1 = torch.randn(C, device=d) * 0.1
  b2 = torch.randn(C, device=d) * 0.1
  t_ref = C_.res_conv_fwd(x, w1, b1, None, True, True)
  y_ref = C_.res_conv_fwd(t_ref, w2, b2, x, False, False)
  t, y = C_.res_block_fwd(x, w1, b1, w2, b2, False)
  dif = (y.float() - y_ref.float()).abs()
  bad = (dif > 0).nonzero()
  print(C, H, W, 't eq', torch.equal(t, t_ref), 'max', dif.max().item(), 'nbad', bad.shape[0],
        'rows', sorted(set(bad[:, 1].tolist()))[:20], 'cols', sorted(set(bad[:, 2].tolist()))[:20],
        'ch', sorted(set(bad[:, 3].tolist()))[:20], flush=True)
