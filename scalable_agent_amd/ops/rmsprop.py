"""Fused TF-RMSProp launch (csrc/kernels/rmsprop.hip)."""

from ._ext import ext, check_cuda


def rmsprop_step(params, grads, ms, mom, frames, lr0, total_frames, decay,
                 momentum, epsilon, guard=None, lstm_err=None):
  """In-place update of the flat buffers; lr decays with the device counter.

  guard: optional int32[4] device tensor (flag, skipped, lstm_timeouts, -):
  when given, a step whose gradients contain a NaN/inf is skipped on the
  device and counted in guard[1].  lstm_err: the recurrence kernels' sticky
  timeout word (ops.lstm.persistent_error_word): a step whose unroll was
  abandoned is skipped too (counted in guard[1] and guard[2]) and the word
  is reset."""
  check_cuda(params, grads, ms, mom, frames)
  ext().rmsprop(params, grads, ms, mom, frames, float(lr0),
                float(total_frames), float(decay), float(momentum),
                float(epsilon), guard, lstm_err)
