"""Near-discontinuities of the torso in float64 (test helper).

A max-pool window whose top two values are within fp32 rounding of each
other, or a ReLU input within rounding of 0, can branch differently in fp32
and in the float64 oracle; one such flip moves a whole local gradient and
shows up as a ~1e-3 relative error in every upstream gradient, although each
kernel is exact.  Gradient-parity tests use inputs free of them (asserted).
"""

import torch
import torch.nn.functional as F

from scalable_agent_amd.models import layers


def count(agent, frames, rel=1e-6):
  """Number of pool near-ties / ReLU near-zeros of agent's torso on frames."""
  P = {k: v.detach().double().cpu() for k, v in agent.convnet.items()}
  x = frames.cpu().double() / 255.0
  n = 0

  def relu(z):
    nonlocal n
    a = z.abs()
    n += int(((a > 0) & (a < rel * a.amax().clamp(min=1e-30))).sum())
    return z.clamp(min=0)

  for sp in agent.specs:
    if sp['kind'] == 'conv':
      x = layers.conv2d_same_nhwc(x, P[sp['name'] + '__w'], P[sp['name'] + '__b'], sp['s'])
      if sp['relu_out']:
        x = relu(x)
    elif sp['kind'] == 'pool':
      ph = layers.same_pads(x.shape[1], 3, 2)
      pw = layers.same_pads(x.shape[2], 3, 2)
      xc = F.pad(x.permute(0, 3, 1, 2), (pw[0], pw[1], ph[0], ph[1]), value=float('-inf'))
      win = F.unfold(xc, 3, stride=2)
      win = win.view(win.shape[0], -1, 9, win.shape[2])
      top2 = win.topk(2, dim=2).values
      gap = top2[:, :, 0] - top2[:, :, 1]
      n += int((gap < rel * top2[:, :, 0].abs().clamp(min=1e-3)).sum())
      x = layers.maxpool_same_nhwc(x, 3, 2)
    else:
      block_in = x
      for sub in ('conv_2d', 'conv_2d_1'):
        x = relu(x)
        x = layers.conv2d_same_nhwc(x, P[sp['name'] + '__' + sub + '__w'],
                                    P[sp['name'] + '__' + sub + '__b'], 1)
      x = x + block_in
  relu(x)
  return n
