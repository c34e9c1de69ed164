"""Bisects a crash of hipGraph capture of the pipelined (two-stream) unroll."""
import faulthandler
import sys

import torch

sys.path.insert(0, '.')
faulthandler.enable()

from scalable_agent_amd import flags as flags_lib  # noqa: E402
from scalable_agent_amd import ops  # noqa: E402
from scalable_agent_amd.envs.synthetic import make_synthetic_batch  # noqa
from scalable_agent_amd.learner import Learner, batch_to_device, compute_loss  # noqa
from scalable_agent_amd.models import Agent  # noqa: E402


def log(*a):
  print(*a, flush=True)


def main():
  mode = sys.argv[1]
  ops.load()
  dev = torch.device('cuda', 0)
  f = flags_lib.default_flags(batch_size=4, unroll_length=15)
  b = batch_to_device(make_synthetic_batch(4, 15, (72, 96, 3), 9, seed=7), dev)
  agent = Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=5,
                backend='hip', compute_dtype=torch.bfloat16, pipeline_chunks=4)
  lrn = Learner(agent, f, dev)
  s = torch.cuda.Stream(dev)
  s.wait_stream(torch.cuda.current_stream(dev))

  def body():
    if mode == 'fwd':
      with torch.no_grad():
        return compute_loss(agent, b, f, use_fused=True)
    if mode == 'fwdgrad':
      return compute_loss(agent, b, f, use_fused=True)
    if mode == 'lstm':
      T, B = 16, 4
      x = torch.randn(T, B, 330, device=dev, requires_grad=True)
      done = torch.zeros(T, B, dtype=torch.bool, device=dev)
      side = agent._core_stream(dev)
      main_s = torch.cuda.current_stream(dev)
      side.wait_stream(main_s)
      with torch.cuda.stream(side):
        hs, st = ops.lstm_unroll(x, done, agent.initial_state(B, dev),
                                 agent.lstm_kernel, agent.lstm_bias)
      main_s.wait_stream(side)
      loss = hs.sum()
      loss.backward()
      return loss
    loss = compute_loss(agent, b, f, use_fused=True)
    loss.backward()
    return loss

  with torch.cuda.stream(s):
    for _ in range(2):
      body()
  torch.cuda.current_stream(dev).wait_stream(s)
  torch.cuda.synchronize()
  log('eager ok')
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    log('capturing')
    out = body()
    log('body done')
  log('capture done')
  g.replay()
  torch.cuda.synchronize()
  log('replay ok', float(out))


if __name__ == '__main__':
  main()
