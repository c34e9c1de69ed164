"""Frame chunking of the HIP torsos (ops/conv_f32.py _chunked, MAX_FRAMES):
large learner batches (the 8-rank single-learner equivalent, 25856 frames)
run as equal chunks of at most MAX_FRAMES frames; per-frame outputs are the
unchunked ones and parameter gradients add up over the chunks.  CPU: a
stand-in autograd Function records the chunk sizes (the GPU kernels' own
chunking test is tests/test_conv_f32_gpu.py)."""

import torch

from scalable_agent_amd.ops import conv_f32


class _PerFrame(torch.autograd.Function):
  """features = frames * w (broadcast), recording each call's frame count."""
  calls = []

  @staticmethod
  def forward(ctx, frames, w):
    _PerFrame.calls.append(frames.shape[0])
    ctx.save_for_backward(frames, w)
    return (frames.float().reshape(frames.shape[0], -1) * w).contiguous()

  @staticmethod
  def backward(ctx, g):
    frames, w = ctx.saved_tensors
    return None, (g * frames.float().reshape(frames.shape[0], -1)).sum(0)


def _run(n, max_frames):
  old = conv_f32.MAX_FRAMES
  conv_f32.MAX_FRAMES = max_frames
  try:
    _PerFrame.calls = []
    g = torch.Generator().manual_seed(0)
    frames = torch.randint(0, 256, (n, 3, 4, 2), generator=g, dtype=torch.uint8)
    w = torch.randn(24, generator=g, requires_grad=True)
    out = conv_f32._chunked(_PerFrame, frames, [w])
    out.sum().backward()
    return out.detach(), w.grad.clone(), list(_PerFrame.calls)
  finally:
    conv_f32.MAX_FRAMES = old


def test_one_chunk_at_or_below_the_limit():
  _, _, calls = _run(3232, 8192)
  assert calls == [3232]
  _, _, calls = _run(8192, 8192)
  assert calls == [8192]


def test_equal_chunks_above_the_limit():
  out1, g1, calls1 = _run(25856, 1 << 30)
  out4, g4, calls4 = _run(25856, 8192)
  assert calls1 == [25856]
  assert calls4 == [6464] * 4          # 4 equal chunks, each <= 8192
  assert torch.equal(out1, out4)
  torch.testing.assert_close(g4, g1, rtol=1e-5, atol=1e-3)


def test_uneven_batch():
  out1, g1, _ = _run(1001, 1 << 30)
  out3, g3, calls = _run(1001, 400)
  assert calls == [334, 334, 333] and sum(calls) == 1001
  assert torch.equal(out1, out3)
  torch.testing.assert_close(g3, g1, rtol=1e-5, atol=1e-3)


def test_default_limit_keeps_the_headline_batch_whole():
  assert conv_f32.MAX_FRAMES >= 32 * 101


def _check_bounds(b, T):
  assert b[0] == 0 and b[-1] == T
  assert all(b1 - b0 >= 1 for b0, b1 in zip(b, b[1:])), b


def test_pipeline_chunk_bounds():
  """Time-chunk boundaries of the torso || LSTM pipeline (agent.py
  _chunk_bounds): equal chunks, SA_PIPELINE_SPLIT proportions, more weights
  than steps, zero weights - every chunk at least one step."""
  from scalable_agent_amd.models.agent import _chunk_bounds
  assert _chunk_bounds(20, 1) == [0, 20]
  assert _chunk_bounds(101, 2) == [0, 50, 101]
  assert _chunk_bounds(20, 3, '9,9,2') == [0, 9, 18, 20]
  for T, chunks, split in [(2, 4, None), (3, 8, None), (2, 1, '1,1,1,1'),
                           (10, 1, '0,0,5'), (10, 1, '5,0,0'),
                           (5, 1, '0,0,0'), (101, 1, '4,1'),
                           (1, 3, '9,9,2'), (7, 1, '1e9,1,1')]:
    b = _chunk_bounds(T, chunks, split)
    _check_bounds(b, T)
  assert len(_chunk_bounds(2, 4)) == 3  # capped at T chunks
