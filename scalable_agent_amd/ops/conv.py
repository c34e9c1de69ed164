"""Deep-ResNet conv torso on the fused gfx950 kernels (csrc/kernels/conv_torso.hip).

Forward per stage s (reference experiment.py:156-176):
  conv_pool_fwd      conv3x3 + bias + maxpool3x3/2 SAME (stage 1 straight from
                     the uint8 frame, x/255 folded into the weights)
  2 x [res_conv_fwd  t = relu(conv(relu(x)) + b)     (stored ReLU'd)
       res_conv_fwd  y = conv(t) + b + x   (+ final ReLU on the last)]
Backward per residual block: two fused dgrad+wgrad+bias passes; per stage head
one pass that gathers the pooled gradient through the saved argmax in LDS.
All activations NHWC bf16; weights/biases fp32 master copies (TF HWIO); their
gradients accumulate in fp32 directly inside the kernels.
"""

import os

import torch

from . import grad_sink
from ._ext import ext
from ..models import layers
from ..utils.knobs import measure_env

TORSO_READY = True
# whole-residual-block forward kernel (res_block_fwd) instead of two
# res_conv_fwd launches - bitwise identical.  At the learner's batch it
# measured slower (206 vs 169 us at 36x48x16, 143 vs 102 at 18x24x32: the
# convs are latency/issue bound, not HBM bound); at actor-inference batches
# (no autograd, <= FUSED_BLOCK_MAX_FRAMES frames) the launch it saves is
# worth more: a board launch 21 -> 15 kernels, 210 -> 190 us of kernels
# (profiles/experiments.md round 6).  SA_FUSED_BLOCK=1 (measurement runs)
# forces it everywhere.
FUSED_BLOCK = measure_env('SA_FUSED_BLOCK', '0') == '1'
FUSED_BLOCK_MAX_FRAMES = 512


def supports(agent):
  """Shapes the fused bf16 kernels cover: the deep ResNet on uint8 frames
  with 3 (RGB: DMLab, Doom) or 4 (stacked Atari frames, BASELINE config #2)
  channels - conv1 packs a pixel's channels into one bf16x4 MFMA operand;
  other inputs take the fp32 kernels, ops/conv_f32.py."""
  return agent.torso_kind == 'deep' and agent.frame_shape[2] in (3, 4)


def _pool_pads(h, w):
  return layers.same_pads(h, 3, 2)[0], layers.same_pads(w, 3, 2)[0]


def deep_param_list(agent):
  """[w, b, (w1, b1, w2, b2) x 2] per stage, in spec order."""
  out = []
  for sp in agent.specs:
    if sp['kind'] == 'conv':
      out += list(agent._conv_params(sp['name']))
    elif sp['kind'] == 'res':
      for sub in ('conv_2d', 'conv_2d_1'):
        out += list(agent._conv_params(sp['name'] + '__' + sub))
  return out


class _DeepTorso(torch.autograd.Function):

  @staticmethod
  def forward(ctx, frames, *params):
    return _deep_forward(ctx, FUSED_BLOCK, frames, params)

  @staticmethod
  def backward(ctx, grad_out):
    return _deep_backward(ctx, grad_out)


class _DeepTorsoInfer(_DeepTorso):
  """Small no-grad batches (actor inference): fused residual blocks."""

  @staticmethod
  def forward(ctx, frames, *params):
    return _deep_forward(ctx, True, frames, params)


def _deep_forward(ctx, fused_block, frames, params):
  C = ext()
  frames = frames.contiguous()
  x = frames
  saved = [frames]
  shapes = []
  p = 0
  for s in range(3):
    w, b = params[p], params[p + 1]
    p += 2
    H, W = x.shape[1], x.shape[2]
    pb_h, pb_w = _pool_pads(H, W)
    if s == 0:
      pooled, arg = C.conv1_pool_fwd(x, w, b, pb_h, pb_w)
    else:
      pooled, arg = C.conv_pool_fwd(x, w, b, pb_h, pb_w)
    shapes.append((H, W, pb_h, pb_w))
    saved += [arg]
    xa = pooled
    for blk in range(2):
      w1, b1, w2, b2 = params[p:p + 4]
      p += 4
      # t is stored ReLU'd: it is only ever consumed as relu(t) (conv 2's
      # input, and the (t > 0) mask in backward), so conv 2 skips its
      # input ReLU and its backward skips the activation ReLU.
      last = (s == 2 and blk == 1)
      if fused_block:
        # both convs of the block in one pass (t never re-read from HBM)
        t, y = C.res_block_fwd(xa, w1, b1, w2, b2, last)
      else:
        t = C.res_conv_fwd(xa, w1, b1, None, True, True)
        y = C.res_conv_fwd(t, w2, b2, xa, last, False)
      saved += [xa, t]
      xa = y
    if s < 2:
      saved += [xa]  # input of the next stage's conv
    x = xa
  ctx.save_for_backward(*saved, x, *params)
  ctx.shapes = shapes
  ctx.nparams = len(params)
  return x.reshape(x.shape[0], -1)


def _deep_backward(ctx, grad_out):
  C = ext()
  t = ctx.saved_tensors
  params = t[-ctx.nparams:]
  out = t[-ctx.nparams - 1]
  saved = list(t[:-ctx.nparams - 1])
  frames = saved[0]
  # unpack per stage: arg, (xa, t) x2, [stage_out]
  stages = []
  k = 1
  for s in range(3):
    arg = saved[k]
    k += 1
    blocks = []
    for _ in range(2):
      blocks.append((saved[k], saved[k + 1]))
      k += 2
    stage_out = None
    if s < 2:
      stage_out = saved[k]
      k += 1
    stages.append((arg, blocks, stage_out))
  # The kernels ACCUMULATE weight/bias gradients: inside
  # grad_sink.direct_grads() straight into the learner's flat gradient
  # buffer (None is returned for those parameters), else into fresh zeros.
  gviews, direct = grad_sink.sinks(params)
  # the torso's final ReLU: dy *= (out > 0), in place on our own bf16 copy
  dy = grad_out.reshape(out.shape)
  if dy.dtype != torch.bfloat16 or not dy.is_contiguous():
    dy = dy.to(torch.bfloat16).contiguous()
  C.relu_mask_bf16_(dy, out)
  p_base = [0, 10, 20]
  for s in reversed(range(3)):
    arg, blocks, _ = stages[s]
    pb = p_base[s]
    for blk in reversed(range(2)):
      xa, tt = blocks[blk]
      i1 = pb + 2 + 4 * blk
      w1, w2 = params[i1], params[i1 + 2]
      dt = C.res_conv_bwd(dy, tt, None, w2, gviews[i1 + 2], gviews[i1 + 3],
                          False)
      dy = C.res_conv_bwd(dt, xa, dy, w1, gviews[i1], gviews[i1 + 1], True)
    H, W, pb_h, pb_w = ctx.shapes[s]
    if s == 0:
      C.conv1_pool_bwd(dy, arg, frames, gviews[pb], gviews[pb + 1], pb_h,
                       pb_w)
    else:
      x_in = stages[s - 1][2]
      dy = C.pool_conv_bwd(dy, arg, x_in, params[pb], gviews[pb],
                           gviews[pb + 1], True, pb_h, pb_w)
  return (None,) + grad_sink.returned(gviews, direct)


def torso_forward(agent, frames):
  """uint8 frames [N,H,W,C] (C = 3 or 4) -> relu'd conv features [N, flat]
  (bf16).  Batches above conv_f32.MAX_FRAMES frames run in equal chunks."""
  if not supports(agent):
    raise NotImplementedError(
        'bf16 HIP torso: deep ResNet on 3/4-channel uint8 frames only (got %r, %r)' %
        (agent.torso_kind, agent.frame_shape))
  from .conv_f32 import _chunked
  fn = (_DeepTorsoInfer if (not torch.is_grad_enabled() and
                            frames.shape[0] <= FUSED_BLOCK_MAX_FRAMES)
        else _DeepTorso)
  return _chunked(fn, frames.contiguous(), deep_param_list(agent))


def linear_relu(x, w, b):
  """Torso FC: relu(x W + b) on bf16 operands, fp32 accumulation.  Without
  autograd (actor inference) it is one hand-written bf16 MFMA GEMM
  (gemm_bf16.hip, bias + ReLU in the epilogue, fp32 out); the differentiable
  per-op path (the fused core's test oracle) keeps torch.addmm."""
  x16 = x.to(torch.bfloat16).contiguous()
  w16 = w.to(torch.bfloat16).contiguous()
  if not (torch.is_grad_enabled() and
          (x.requires_grad or w.requires_grad or b.requires_grad)):
    out = torch.empty(x16.shape[0], w16.shape[1], device=x.device,
                      dtype=torch.float32)
    ext().gemm_bf16(x16, w16, False, False, out,
                    bias=b.detach().float().contiguous(), relu=True)
    return out
  y = torch.addmm(b.to(torch.bfloat16), x16, w16)
  return torch.relu(y).to(torch.float32)
