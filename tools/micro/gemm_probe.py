"""Probes which fused GEMM forms torch/hipBLASLt offers on MI355X (bf16 in,
fp32 out; bias+ReLU epilogue; in-place fp32 accumulation) and times them at
the learner's FC / x-projection shapes."""
import torch


def t_us(fn, reps=50):
  for _ in range(3):
    fn()
  torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record()
  for _ in range(reps):
    fn()
  e.record()
  torch.cuda.synchronize()
  return s.elapsed_time(e) / reps * 1e3


def probe(name, fn):
  try:
    out = fn()
    print('%-34s ok  %-14s %7.1f us' % (name, str(out.dtype), t_us(fn)))
  except Exception as ex:  # noqa
    print('%-34s FAIL %s' % (name, str(ex).splitlines()[0][:100]))


def main():
  d = torch.device('cuda')
  N, F, H, G = 3232, 3456, 256, 1024
  feats = torch.randn(N, F, device=d).bfloat16()
  w = (torch.randn(F, H, device=d) * 0.02).bfloat16()
  b = torch.randn(H, device=d).bfloat16()
  h = torch.randn(N, H, device=d).relu().bfloat16()
  wx = (torch.randn(H, G, device=d) * 0.05).bfloat16()
  dxw = torch.randn(N, G, device=d)
  dxw16 = dxw.bfloat16()
  g32 = torch.zeros(H, G, device=d)
  gfc = torch.zeros(F, H, device=d)
  x32 = torch.randn(N, 330, device=d)
  wx32 = torch.randn(330, G, device=d)
  probe('addmm bf16 (fc)', lambda: torch.addmm(b, feats, w))
  probe('_addmm_activation relu bf16', lambda: torch._addmm_activation(b, feats, w))
  probe('mm bf16->fp32 out_dtype (xproj)', lambda: torch.mm(h, wx, out_dtype=torch.float32))
  probe('mm bf16 (xproj)', lambda: torch.mm(h, wx))
  probe('mm fp32 (xproj old, K=330)', lambda: torch.mm(x32, wx32))
  probe('addmm out_dtype accumulate dW', lambda: torch.addmm(g32, h.t(), dxw16, out_dtype=torch.float32, out=g32))
  probe('addmm_ accumulate dW_fc bf16', lambda: torch.addmm(gfc, feats.t(), h, out_dtype=torch.float32, out=gfc))
  probe('mm dfeats bf16', lambda: torch.mm(h, w.t()))
  probe('mm dxw @ wx^T bf16', lambda: torch.mm(dxw16, wx.t()))
  probe('fp32 addmm_ dWh (K=3232)', lambda: g32.addmm_(torch.randn(N, H, device=d).t(), dxw))
  # correctness of the accumulating form
  g = torch.ones(H, G, device=d)
  torch.addmm(g, h.t(), dxw16, out_dtype=torch.float32, out=g)
  ref = 1 + h.float().t() @ dxw16.float()
  print('accumulate max err', float((g - ref).abs().max()), float(ref.abs().max()))


if __name__ == '__main__' and 'backends' not in __import__('sys').argv:
  main()


def compare_backends():
  """hipBLASLt (torch default) vs rocBLAS on the learner GEMM shapes."""
  d = torch.device('cuda')
  N, F, H, G, K = 3232, 3456, 256, 1024, 272
  feats = torch.randn(N, F, device=d).bfloat16()
  w = (torch.randn(F, H, device=d) * 0.02).bfloat16()
  b = torch.randn(H, device=d).bfloat16()
  h = torch.randn(N, K, device=d).relu().bfloat16()
  wx = (torch.randn(K, G, device=d) * 0.05).bfloat16()
  bias = torch.randn(G, device=d)
  dg = torch.randn(N, G, device=d).bfloat16()
  gx = torch.zeros(K, G, device=d)
  gf = torch.zeros(F, H, device=d)
  dh = torch.randn(N, H, device=d).bfloat16()
  hp = torch.randn(N, 256, device=d)
  dg32 = torch.randn(N, G, device=d)
  gwh = torch.zeros(256, G, device=d)
  shapes = [
      ('fc fwd relu', lambda: torch._addmm_activation(b, feats, w)),
      ('xproj fwd', lambda: torch.addmm(bias, h, wx, out_dtype=torch.float32)),
      ('dWx', lambda: torch.addmm(gx, h.t(), dg, out_dtype=torch.float32, out=gx)),
      ('dh', lambda: torch.mm(dg, wx[:256].t())),
      ('dfeats', lambda: torch.mm(dh, w.t())),
      ('dWfc', lambda: torch.addmm(gf, feats.t(), dh, out_dtype=torch.float32, out=gf)),
      ('dWh fp32', lambda: gwh.addmm_(hp.t(), dg32)),
  ]
  for lib in ('hipblaslt', 'ck', 'hipblas'):
    try:
      torch.backends.cuda.preferred_blas_library(lib)
    except Exception as ex:  # noqa
      print(lib, 'unavailable', ex)
      continue
    for name, fn in shapes:
      probe('%s %s' % (lib, name), fn)


if __name__ == '__main__' and 'backends' in __import__('sys').argv:
  compare_backends()
