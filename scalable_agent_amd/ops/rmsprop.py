"""Fused TF-RMSProp launch (csrc/kernels/rmsprop.hip)."""

from ._ext import ext, check_cuda


def rmsprop_step(params, grads, ms, mom, frames, lr0, total_frames, decay,
                 momentum, epsilon):
  """In-place update of the flat buffers; lr decays with the device counter."""
  check_cuda(params, grads, ms, mom, frames)
  ext().rmsprop(params, grads, ms, mom, frames, float(lr0),
                float(total_frames), float(decay), float(momentum),
                float(epsilon))
