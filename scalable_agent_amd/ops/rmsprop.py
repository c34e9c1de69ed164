"""Fused TF-RMSProp launch (csrc/kernels/rmsprop.hip)."""

from ._ext import ext, check_cuda


def rmsprop_step(params, grads, ms, mom, frames, lr0, total_frames, decay,
                 momentum, epsilon, guard=None, lstm_err=None, grad_scale=1.0):
  """In-place update of the flat buffers; lr decays with the device counter.
  grad_scale multiplies the gradient inside the update (1/world: the
  data-parallel mean without a separate pass over the buffer).

  guard: optional int32[4] device tensor (flag, skipped, lstm_timeouts,
  conv_timeouts): when given, a step whose gradients contain a NaN/inf is
  skipped on the device and counted in guard[1].  lstm_err: the device's
  sticky error words (ops.lstm.persistent_error_word, int32[4]): [0] set by
  an abandoned cooperative LSTM unroll, [1] by an expired hand-off wait of
  the fused Winograd backward; such a step is skipped too (counted in
  guard[1] and guard[2] / guard[3]) and the words are reset."""
  check_cuda(params, grads, ms, mom, frames)
  ext().rmsprop(params, grads, ms, mom, frames, float(lr0),
                float(total_frames), float(decay), float(momentum),
                float(epsilon), guard, lstm_err, float(grad_scale))


def poison_on_error(slot, err):
  """DP step guard (before the gradient all-reduce): NaN into `slot` (the
  flat gradient buffer's reserved sentinel element) when this device's
  sticky error words are set, so every rank's finite check skips the step."""
  check_cuda(slot, err)
  ext().err_poison(slot, err)
