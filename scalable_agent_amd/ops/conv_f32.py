"""Reference-precision conv torsos on the exact-fp32 MFMA kernels
(csrc/kernels/conv_f32.hip: v_mfma_f32_16x16x4_f32, f32 in / f32 accumulate).

The reference computes its torso in fp32 (experiment.py:153-189: to_float/255,
fp32 cuDNN convs); these kernels reproduce that numerically (one rounding
per product, like an fmaf chain) with every TF-SAME padding, the uint8 /255
scaling and the ReLUs/residual adds fused into the conv loads and epilogues:

  shallow (experiment.py:178-183): 3 x [conv (8x8/4, 4x4/2, 3x3/2 with the
      asymmetric W pad 0/1) + bias + ReLU]
  deep    (experiment.py:156-176): per stage conv3x3 + bias -> maxpool
      3x3/2 SAME (argmax saved) -> 2 x [t = relu(conv(relu(x)) + b1);
      y = conv(t) + b2 + x], final ReLU

Backward: data gradients are the same kernel over the stride-dilated dY with
flipped/transposed weights (ReLU masks and skip adds in the epilogue);
weight+bias gradients are a deterministic two-stage reduction accumulated
straight into the learner's flat gradient buffer (grad_sink).  Frames may
carry any C <= 4 channels (RGB, or Atari-style stacked grayscale).
"""

import torch

from . import grad_sink
from ._ext import ext
from ..models import layers

import os
from ..utils.knobs import measure_env

# debug hook (tools/debug): when a dict, the deep torso backward records its
# intermediate gradients in it
DEBUG_TAPE = None
# Deep-torso stage heads (conv -> max-pool).  By default every head whose
# shape the fused Winograd conv+pool kernel covers (conv_wino.hip
# wino_conv_pool_kernel: the 72x96 torso's three heads; SA_F32_WINO_POOL
# selects) runs conv + pool + argmax in one kernel.  Otherwise: stages
# (0-based) listed here run the direct fused conv+pool kernel (pre-pool map
# only in LDS), the rest conv + maxpool_fwd; and whether the backward gathers
# the pre-pool gradient from (dP, argmax) inside the conv kernels' loads
# instead of materialising it with maxpool_bwd.
FUSED_POOL_STAGES = tuple(int(c) for c in measure_env('SA_F32_FUSED_POOL', '0')
                          if c.isdigit())
# SA_F32_POOL_GATHER=1: every stage; a digit string (e.g. '0'): those stages
_pg = measure_env('SA_F32_POOL_GATHER', '')
POOL_GATHER_STAGES = (0, 1, 2) if _pg == '1' else tuple(
    int(c) for c in _pg if c.isdigit())
POOL_GATHER = bool(POOL_GATHER_STAGES)
# Stage 0 (4-channel frames -> 16): the conv's weight gradient is computed
# straight from (dP, argmax) in scatter form (pool_wgrad_kernel) instead of
# maxpool_bwd + the dense wgrad; SA_F32_POOL_SCATTER=0 restores the latter.
POOL_SCATTER = os.environ.get('SA_F32_POOL_SCATTER', '1') != '0'
# uint8 frames straight into the first conv (x / 255 on the way into LDS)
# instead of one fp32 x/255 image written first: the deep stage-0 kernels
# measured slower on bytes (conv+pool 639 vs 529 + 120 us, scatter wgrad
# 463 vs 229 us: per-pixel byte loads) and the shallow learner step too
# (5.15 vs 5.01 ms), so both default to the fp32 image; kept switchable
# Stage-0 scatter wgrad reading the uint8 frames (coalesced dword rows, exact
# x / 255 table in LDS) instead of the 4-channel fp32 image the forward conv
# reads (the image is then dropped after the forward): opt-in
# (SA_F32_PW_U8=1) - measured slower, 9.47-9.52 vs 9.37 ms per fp32 step
# (the byte expansion in LDS costs more than the image reads it saves)
PW_U8 = measure_env('SA_F32_PW_U8', '0') == '1'
U8_DIRECT = {
    'deep': measure_env('SA_F32_U8_DEEP', '0') == '1',
    'shallow': measure_env('SA_F32_U8_SHALLOW', '0') == '1'}


def supports(agent):
  """Shapes the fp32 kernels cover: both torsos, uint8 frames with C <= 4."""
  c = agent.frame_shape[2]
  return agent.torso_kind in ('deep', 'shallow') and 1 <= c <= 4


def _conv_geom(H, W, k, s):
  return (layers.same_pads(H, k, s)[0], layers.same_pads(W, k, s)[0],
          layers.same_out(H, s), layers.same_out(W, s))


class _ShallowTorsoF32(torch.autograd.Function):

  @staticmethod
  def forward(ctx, frames, *params):
    C = ext()
    # layer 1 reads the uint8 frames itself (x / 255 on the way into LDS),
    # or a 4-channel fp32 x / 255 image (one 16-B load per pixel)
    x = frames.contiguous()
    if not U8_DIRECT['shallow']:
      x = C.cf32_frames_f32(x)
    acts = [x]
    geoms = []
    for i in range(3):
      w, b = params[2 * i], params[2 * i + 1]
      if i == 0 and w.shape[2] != x.shape[3]:
        w = _pad_cin(w, x.shape[3])  # zero rows for the image's pad channel
      k = w.shape[0]
      s = (4, 2, 2)[i]
      H, W = x.shape[1], x.shape[2]
      pt, pl, Ho, Wo = _conv_geom(H, W, k, s)
      x = C.cf32_conv_fwd(x, w, b, s, pt, pl, Ho, Wo, relu_out=True)
      acts.append(x)
      geoms.append((s, pt, pl, H, W))
    ctx.save_for_backward(*acts, *params)
    ctx.geoms = geoms
    return x.reshape(x.shape[0], -1)

  @staticmethod
  def backward(ctx, grad_out):
    C = ext()
    t = ctx.saved_tensors
    acts, params = t[:4], t[4:]
    out = acts[3]
    gv, direct = grad_sink.sinks(params)
    # the torso's trailing ReLUs (layer-3 ReLU and experiment.py:185)
    dy = grad_out.reshape(out.shape).to(torch.float32).clone(
        memory_format=torch.contiguous_format)
    C.cf32_relu_mask_(dy, out)
    for i in reversed(range(3)):
      s, pt, pl, H, W = ctx.geoms[i]
      # layer 0 on an RGB frame staged as 4 channels: the kernel writes the
      # 3-channel weight gradient directly (dw_cin)
      C.cf32_conv_wgrad(acts[i], dy, s, pt, pl, False, gv[2 * i], gv[2 * i + 1])
      if i > 0:
        # input of layer i is the ReLU'd output of layer i-1
        dy = C.cf32_conv_dgrad(dy, params[2 * i], s, pt, pl, H, W, mask=acts[i])
    return (None,) + grad_sink.returned(gv, direct)


class _DeepTorsoF32(torch.autograd.Function):

  @staticmethod
  def forward(ctx, frames, *params):
    C = ext()
    # stage 0 reads a 4-channel fp32 x / 255 image (one 16-B load per pixel
    # in the conv+pool and scatter-wgrad stagers), or the uint8 frames
    x = frames.contiguous()
    if not U8_DIRECT['deep']:
      x = C.cf32_frames_f32(x)
    saved, meta = [], []
    p = 0
    for s in range(3):
      w, b = params[p], params[p + 1]
      p += 2
      if s == 0 and w.shape[2] != x.shape[3]:
        w = _pad_cin(w, x.shape[3])  # zero rows for the image's pad channel
      H, W = x.shape[1], x.shape[2]
      pbh = layers.same_pads(H, 3, 2)[0]
      pbw = layers.same_pads(W, 3, 2)[0]
      fused = (C.cf32_wino_conv_pool_fwd(x, w, b) if x.dtype == torch.float32
               else [])
      if fused:
        # stage 0 (4-channel image -> 16) and stage 1 (16 -> 32) heads
        # with the pool in the Winograd epilogue (the pre-pool map only in
        # LDS); other shapes: the direct conv+pool or conv + maxpool_fwd
        xa, arg = fused
      elif s in FUSED_POOL_STAGES:
        xa, arg = C.cf32_conv_pool_fwd(x, w, b, pbh, pbw)
      else:
        conv = C.cf32_conv_fwd(x, w, b, 1, 1, 1, H, W)
        xa, arg = C.cf32_maxpool_fwd(conv, pbh, pbw)
        del conv
      h, w_ = xa.shape[1], xa.shape[2]
      # stage 0 on the scatter wgrad path: its backward reads the uint8
      # frames, so the fp32 image is not kept alive for it
      keep = (frames if (s == 0 and PW_U8 and POOL_SCATTER and
                         x.dtype == torch.float32 and frames.dtype == torch.uint8 and
                         frames.shape[3] <= 4 and xa.shape[3] == 16)
              else x)
      saved += [keep, arg]
      for blk in range(2):
        w1, b1, w2, b2 = params[p:p + 4]
        p += 4
        last = s == 2 and blk == 1
        # t stored ReLU'd: conv 2 reads it as is, its mask is (t > 0)
        t = C.cf32_conv_fwd(xa, w1, b1, 1, 1, 1, h, w_, relu_in=True,
                            relu_out=True)
        y = C.cf32_conv_fwd(t, w2, b2, 1, 1, 1, h, w_, add=xa, relu_out=last)
        saved += [xa, t]
        xa = y
      meta.append((H, W, h, w_, pbh, pbw))
      x = xa
    ctx.save_for_backward(*saved, x, *params)
    ctx.meta = meta
    ctx.nparams = len(params)
    if DEBUG_TAPE is not None:
      DEBUG_TAPE['saved'] = [t.clone() for t in saved]
    return x.reshape(x.shape[0], -1)

  @staticmethod
  def backward(ctx, grad_out):
    C = ext()
    t = ctx.saved_tensors
    params = t[-ctx.nparams:]
    out = t[-ctx.nparams - 1]
    saved = t[:-ctx.nparams - 1]
    gv, direct = grad_sink.sinks(params)
    dy = grad_out.reshape(out.shape)
    if not (getattr(grad_out, '_sa_scratch', False) and
            dy.dtype == torch.float32 and dy.is_contiguous()):
      # the incoming gradient is masked in place below: copy unless it is
      # the fused core's own scratch dfeats buffer (never a caller's tensor)
      dy = dy.to(torch.float32).clone(memory_format=torch.contiguous_format)
    if not getattr(grad_out, '_sa_relu_masked', False):
      # final ReLU of the torso (the fused fp32 core masks dfeats in its
      # GEMM epilogue already; masking twice would be harmless)
      C.cf32_relu_mask_(dy, out)
    # the ~15 fixed-order weight-gradient slot sums of this backward are
    # queued and launched as ONE kernel at the end (cf32_wgrad_flush)
    C.cf32_wgrad_defer(True)
    try:
      _deep_backward(C, ctx, saved, params, gv, dy)
    finally:
      C.cf32_wgrad_defer(False)
      C.cf32_wgrad_flush()
    return (None,) + grad_sink.returned(gv, direct)


def _deep_backward(C, ctx, saved, params, gv, dy):
  """The stage loop of _DeepTorsoF32.backward (reverse stage order)."""
  for s in reversed(range(3)):
    k = 6 * s
    if DEBUG_TAPE is not None:
      DEBUG_TAPE[('intact', s)] = [bool(torch.equal(a, b)) for a, b in
                                   zip(saved, DEBUG_TAPE['saved'])]
    stage_in, arg = saved[k], saved[k + 1]
    H, W, h, w_, pbh, pbw = ctx.meta[s]
    pb = 10 * s
    for blk in reversed(range(2)):
      xa, tt = saved[k + 2 + 2 * blk], saved[k + 3 + 2 * blk]
      i1 = pb + 2 + 4 * blk
      w1, w2 = params[i1], params[i1 + 2]
      # one pass per conv: its data gradient (masked by the conv's own
      # input, + the skip for the block's first conv) and its weight/bias
      # gradient read dY and the input once (conv_wino.hip fused backward
      # where it covers the shape, else the separate kernels)
      dt = C.cf32_conv_bwd_fused(dy, w2, tt, False, gv[i1 + 2], gv[i1 + 3])
      if DEBUG_TAPE is not None:
        DEBUG_TAPE[('dy', s, blk)] = dy.clone()
        DEBUG_TAPE[('dt', s, blk)] = dt.clone()
      dy = C.cf32_conv_bwd_fused(dt, w1, xa, True, gv[i1], gv[i1 + 1], add=dy)
    # stage 0 on an RGB frame staged as 4 channels: the kernels write
    # the 3-channel weight gradient directly (dw_cin)
    gw = gv[pb]
    scatter = (s == 0 and POOL_SCATTER and stage_in.shape[3] <= 4
               and dy.shape[3] == 16)
    if s in POOL_GATHER_STAGES or scatter:
      # the conv kernels gather the pre-pool gradient from (dP, argmax)
      C.cf32_conv_wgrad(stage_in, dy, 1, 1, 1, False, gw, gv[pb + 1],
                        pool_arg=arg, pool_pbh=pbh, pool_pbw=pbw)
      if s > 0:
        dy = C.cf32_conv_dgrad(dy, params[pb], 1, 1, 1, H, W, pool_arg=arg,
                               pool_pbh=pbh, pool_pbw=pbw)
      continue
    dconv = C.cf32_maxpool_bwd(dy, arg, H, W, pbh, pbw)
    if DEBUG_TAPE is not None:
      DEBUG_TAPE[('dpool', s)] = dy.clone()
      DEBUG_TAPE[('dconv', s)] = dconv.clone()
    if s > 0:
      # stage head (16 -> 32 / 32 -> 32): data + weight gradient in one
      # pass over (dconv, stage input); the input is the previous stage's
      # raw output, so no ReLU mask
      dy = C.cf32_conv_bwd_fused(dconv, params[pb], stage_in, False, gw, gv[pb + 1],
                                 mask=False)
      continue
    C.cf32_conv_wgrad(stage_in, dconv, 1, 1, 1, False, gw, gv[pb + 1])


_ZPAD = {}


def _pad_cin(w, c):
  """HWIO weights zero-padded on the input-channel axis to c channels: one
  concatenation with a cached zero block (a fill + a copy per call before)."""
  shape = w.shape[:2] + (c - w.shape[2],) + w.shape[3:]
  key = (tuple(shape), w.dtype, w.device)
  z = _ZPAD.get(key)
  if z is None:
    z = torch.zeros(shape, dtype=w.dtype, device=w.device)
    # a block first made inside a graph capture holds zeros only once that
    # graph has replayed: cache eagerly made blocks only, and only once their
    # fill has run (other threads may read the cache from other streams)
    if not w.is_cuda:
      _ZPAD[key] = z
    elif not torch.cuda.is_current_stream_capturing():
      torch.cuda.current_stream(w.device).synchronize()
      _ZPAD[key] = z
  return torch.cat([w, z], dim=2)


def shallow_param_list(agent):
  out = []
  for sp in agent.specs:
    out += list(agent._conv_params(sp['name']))
  return out


# Frames per torso launch sequence.  Larger learner batches (e.g. the
# single-learner equivalent of 8 data-parallel ranks: B=256, T=100 = 25856
# frames) run the torso in equal chunks of at most this many frames: the
# Winograd launchers take < 2^22 tiles (9709 frames at 36x48) and every
# tensor must stay inside one 4 GB buffer descriptor (36x48x32 fp32 is
# 221 KB per frame).  Per-frame features are independent of the chunking;
# the weight gradients of the chunks accumulate into the same sinks.  The
# headline batch (3232 frames) is one chunk.
MAX_FRAMES = int(os.environ.get('SA_F32_MAX_FRAMES', '8192'))


def _chunked(fn, frames, params):
  n = frames.shape[0]
  k = -(-n // max(1, MAX_FRAMES))
  if k <= 1:
    return fn.apply(frames, *params)
  step = -(-n // k)
  return torch.cat([fn.apply(frames[i:i + step], *params)
                    for i in range(0, n, step)])


def torso_forward_f32(agent, frames):
  """uint8 frames [N,H,W,C] -> ReLU'd conv features [N, flat] (fp32)."""
  if not supports(agent):
    raise NotImplementedError(
        'fp32 HIP torso: unsupported torso %r / frame shape %r' %
        (agent.torso_kind, agent.frame_shape))
  if frames.dtype != torch.uint8:
    raise TypeError('HIP torso expects uint8 frames, got %s' % frames.dtype)
  frames = frames.contiguous()
  if agent.torso_kind == 'shallow':
    return _chunked(_ShallowTorsoF32, frames, shallow_param_list(agent))
  from .conv import deep_param_list
  params = deep_param_list(agent)
  cache = getattr(agent, '_inference_cache', None)
  if (cache is not None and cache.get('w0pad') is not None and
      not torch.is_grad_enabled() and not U8_DIRECT['deep']):
    # an inference agent's stage-0 weights, zero-padded to the image's 4
    # channels once per weight publish (no concatenation kernel per step)
    params = [cache['w0pad']] + params[1:]
  return _chunked(_DeepTorsoF32, frames, params)


def linear_relu_f32(x, w, b):
  """Torso FC in fp32: relu(x W + b) (library fp32 GEMM: exact f32 on gfx950,
  which has no xf32/TF32 mode)."""
  return torch.relu(torch.addmm(b, x, w))
