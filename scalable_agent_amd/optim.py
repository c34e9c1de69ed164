"""TF-semantics RMSProp on a flat parameter buffer + polynomial LR decay.

Reference: `tf.train.RMSPropOptimizer(lr, decay, momentum, epsilon)` applied by
`ApplyRMSProp` per variable (experiment.py:410-415) [TF-lib semantics]:
    ms  <- ms + (g^2 - ms) * (1 - decay)      # ms slot initialised to 1.0
    mom <- momentum * mom + lr * g / sqrt(ms + epsilon)
    w   <- w - mom
and `tf.train.polynomial_decay(lr0, frames, total_frames, 0)` = linear decay to
zero driven by the env-frame counter (read BEFORE the step's increment,
experiment.py:418-420).

MI355X design: all parameters live in ONE contiguous fp32 buffer (and all
gradients in another), so the optimizer is a single fused HIP launch over the
flat buffer (`ops.rmsprop_step`, K15/K16 of SURVEY.md §2.3) with the learning
rate computed on the device from the frame counter (no host sync, graph
capturable), and the gradient all-reduce is one bucketed RCCL call.
"""

import torch


def polynomial_decay(lr0, frames, total_frames, end_lr=0.0, power=1.0):
  """Works on python numbers or tensors."""
  if torch.is_tensor(frames):
    f = torch.clamp(frames.to(torch.float64), max=float(total_frames))
    return (lr0 - end_lr) * (1 - f / float(total_frames)) ** power + end_lr
  f = min(float(frames), float(total_frames))
  return (lr0 - end_lr) * (1 - f / float(total_frames)) ** power + end_lr


class FlatParams:
  """Re-homes every parameter of `module` into one flat fp32 buffer.

  `module` must already live on its final device.  Parameter `.data` and
  `.grad` become views into `self.params` / `self.grads`.
  """

  ALIGN = 64  # elements; keeps every tensor 256-B aligned for vector loads

  def __init__(self, module):
    # the buffer ends with ALIGN reserved elements that belong to no
    # parameter: `sentinel` (their first) is where the data-parallel step
    # guard writes a NaN that the gradient all-reduce carries to every rank
    # (Learner._apply); the update leaves them at zero
    self.module = module
    self.named = [(n, p) for n, p in module.named_parameters()]
    device = self.named[0][1].device
    offsets = []
    off = 0
    for _, p in self.named:
      offsets.append(off)
      off += (p.numel() + self.ALIGN - 1) // self.ALIGN * self.ALIGN
    self.sentinel = off
    off += self.ALIGN
    self.numel = off
    self.offsets = offsets
    self.params = torch.zeros(off, dtype=torch.float32, device=device)
    self.grads = torch.zeros(off, dtype=torch.float32, device=device)
    for (_, p), o in zip(self.named, offsets):
      n = p.numel()
      self.params[o:o + n].copy_(p.data.reshape(-1).to(torch.float32))
      p.data = self.params[o:o + n].view_as(p)
      p.grad = self.grads[o:o + n].view_as(p)

  def view_of(self, buf, name):
    """View of parameter `name` in a buffer with the flat layout (e.g. the
    RMSProp ms / mom slots)."""
    for (n, p), o in zip(self.named, self.offsets):
      if n == name:
        return buf[o:o + p.numel()].view_as(p)
    raise KeyError(name)

  def zero_grad(self):
    self.grads.zero_()

  def rebind_grads(self):
    """Autograd may replace `.grad`; force it back onto the flat buffer."""
    for (_, p), o in zip(self.named, self.offsets):
      n = p.numel()
      view = self.grads[o:o + n].view_as(p)
      if p.grad is None or p.grad.data_ptr() != view.data_ptr():
        if p.grad is not None:
          view.copy_(p.grad)
        p.grad = view

  def state_dict(self):
    return {n: p.detach().clone() for n, p in self.named}

  def load_state_dict(self, sd):
    for n, p in self.named:
      p.data.copy_(sd[n].to(p.device))


class RMSProp:
  """TF RMSProp over a FlatParams buffer with on-device LR schedule."""

  def __init__(self, flat: FlatParams, learning_rate, decay=0.99, momentum=0.,
               epsilon=0.1, total_frames=int(1e9), use_hip=None,
               skip_nonfinite=True, lstm_err=None, grad_scale=1.0):
    self.flat = flat
    # the step uses grad_scale * grad (data-parallel mean: 1 / world, folded
    # into the update instead of a separate pass over the gradient buffer)
    self.grad_scale = float(grad_scale)
    self.lr0 = float(learning_rate)
    self.decay = float(decay)
    self.momentum = float(momentum)
    self.epsilon = float(epsilon)
    self.total_frames = int(total_frames)
    dev = flat.params.device
    self.ms = torch.ones_like(flat.params)    # TF initialises ms to 1.0
    self.mom = torch.zeros_like(flat.params)
    if use_hip is None:
      use_hip = dev.type == 'cuda'
    self.use_hip = use_hip
    # (flag, skipped steps, lstm timeouts, conv timeouts): a step with NaN/inf
    # gradients, an abandoned cooperative LSTM unroll or an expired conv
    # hand-off wait (lstm_err: the device's sticky error words, [0] the
    # recurrence's, [1] the fused conv backward's) leaves the parameters and
    # slots untouched (SURVEY §5.3 failure detection).
    self.skip_nonfinite = skip_nonfinite
    self.lstm_err = lstm_err if skip_nonfinite else None
    self.guard = torch.zeros(4, dtype=torch.int32, device=dev)

  @property
  def skipped_steps(self):
    return int(self.guard[1].item())

  @property
  def lstm_timeouts(self):
    return int(self.guard[2].item())

  def health(self):
    """(skipped steps, lstm timeouts, conv timeouts) with one device read."""
    g = self.guard.tolist()
    return int(g[1]), int(g[2]), int(g[3])

  def step(self, frames):
    """frames: int64 0-d tensor on the param device (read-only here)."""
    if self.use_hip:
      from . import ops
      ops.rmsprop_step(self.flat.params, self.flat.grads, self.ms, self.mom,
                       frames, self.lr0, self.total_frames, self.decay,
                       self.momentum, self.epsilon,
                       self.guard if self.skip_nonfinite else None,
                       self.lstm_err, self.grad_scale)
      return
    g = self.flat.grads
    if self.grad_scale != 1.0:
      g = g * self.grad_scale
    if self.skip_nonfinite and not bool(torch.isfinite(g).all()):
      self.guard[1] += 1
      return
    lr = polynomial_decay(self.lr0, frames, self.total_frames).to(torch.float32)
    self.ms.add_((g * g - self.ms) * (1 - self.decay))
    self.mom.mul_(self.momentum).add_(lr * g / torch.sqrt(self.ms +
                                                           self.epsilon))
    self.flat.params.sub_(self.mom)

  def current_lr(self, frames):
    return float(polynomial_decay(self.lr0, int(frames), self.total_frames))

  def state_dict(self):
    return {'ms': self.ms.detach().clone(), 'mom': self.mom.detach().clone()}

  def load_state_dict(self, sd):
    # checkpoints written before the sentinel tail existed are ALIGN
    # elements shorter; the tail's slots keep their initial values
    for dst, key in ((self.ms, 'ms'), (self.mom, 'mom')):
      src = sd[key].to(dst.device)
      dst[:src.numel()].copy_(src)
