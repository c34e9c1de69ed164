"""Fused TF-RMSProp launch (csrc/kernels/rmsprop.hip)."""

from ._ext import ext, check_cuda


def rmsprop_step(params, grads, ms, mom, frames, lr0, total_frames, decay,
                 momentum, epsilon, guard=None):
  """In-place update of the flat buffers; lr decays with the device counter.

  guard: optional int32[2] device tensor (flag, skipped-count): when given,
  a step whose gradients contain a NaN/inf is skipped on the device and
  counted in guard[1]."""
  check_cuda(params, grads, ms, mom, frames)
  ext().rmsprop(params, grads, ms, mom, frames, float(lr0),
                float(total_frames), float(decay), float(momentum),
                float(epsilon), guard)
