#!/usr/bin/env python3
"""Which torch ops launch kernels in one eager learner step (torch.profiler
with stacks): every aten op with device time, grouped by the Python frame
that called it.  usage: python tools/micro/step_ops.py [fp32|bf16]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
from scalable_agent_amd import flags as flags_lib  # noqa: E402
from scalable_agent_amd.envs.synthetic import make_synthetic_batch  # noqa: E402
from scalable_agent_amd.learner import FlatStaging, Learner  # noqa: E402
from scalable_agent_amd.models import Agent  # noqa: E402

dtype = sys.argv[1] if len(sys.argv) > 1 else 'fp32'
dev = torch.device('cuda')
flags = flags_lib.default_flags(batch_size=32, unroll_length=100, torso='deep', dtype=dtype)
agent = Agent(9, torso='deep', frame_shape=(72, 96, 3), seed=1, backend='hip',
              compute_dtype=torch.bfloat16 if dtype == 'bf16' else torch.float32)
learner = Learner(agent, flags, dev)
hb = make_synthetic_batch(32, 100, (72, 96, 3), 9, seed=3, pin_memory=False)
slot = FlatStaging(hb, dev).load(hb).views
for _ in range(3):
  learner.step(slot)
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
             with_stack=True, record_shapes=True) as prof:
  learner.step(slot)
  torch.cuda.synchronize()
small = ('fill_', 'zero_', 'copy_', 'clone', 'contiguous', 'to', 'add_', 'ones_like',
         'zeros', 'zeros_like', 'mul_', 'where', 'eq', 'ne', '_to_copy')
for e in prof.events():
  if e.device_type != torch.autograd.DeviceType.CPU:
    continue
  name = e.name.replace('aten::', '')
  if name not in small:
    continue
  kids = [k.name for k in e.cpu_children]
  print('%-10s shapes=%s dtypes=%s children=%s' % (
      name, e.input_shapes, getattr(e, 'dtypes', None), kids[:3]))
