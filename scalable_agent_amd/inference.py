"""Batched actor inference on the GPU (the reference's dynamic-batching path,
experiment.py:534-546 + dynamic_batching.py).

`InferenceModel` owns its OWN copy of the agent parameters on the device (a
versioned weight snapshot): the learner publishes new
weights after every update with one device-to-device copy of the flat buffer,
so an inference batch never reads half-updated weights.  Inference runs on a
dedicated HIP stream, concurrently with the learner stream.

`make_batched_infer` wraps it with the C++ dynamic batcher: actor threads call
it with batch-1 numpy arrays; the runner thread executes batches of up to
`max_batch` rows (timeout `timeout_ms`).
"""

import threading

import numpy as np
import torch

from . import dynamic_batching
from .optim import FlatParams
from .structs import StepOutput, StepOutputInfo


class InferenceModel(object):

  def __init__(self, agent, device, use_instruction=True, seed=0):
    self.device = torch.device(device)
    self.agent = agent.to(self.device)
    self.agent.eval()
    self.flat = FlatParams(self.agent)
    self.use_instruction = use_instruction
    self.version = 0
    self._lock = threading.Lock()
    self._stream = (torch.cuda.Stream(self.device)
                    if self.device.type == 'cuda' else None)
    self._gen = torch.Generator(device=self.device).manual_seed(seed)

  def publish(self, flat_params, version=None):
    """Copies the learner's flat parameter buffer into the snapshot."""
    with self._lock:
      if self._stream is not None:
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._stream.wait_event(ev)
        with torch.cuda.stream(self._stream):
          self.flat.params.copy_(flat_params, non_blocking=True)
      else:
        self.flat.params.copy_(flat_params)
      self.version = self.version + 1 if version is None else version

  @torch.no_grad()
  def infer(self, last_action, reward, done, frame, instr_ids, instr_len, c,
            h):
    """Batched numpy in -> numpy out (action, logits, baseline, c, h)."""
    dev = self.device
    with self._lock:
      ctx = (torch.cuda.stream(self._stream) if self._stream is not None
             else _null())
      with ctx:
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(
            dev, non_blocking=True)
        instr = None
        if self.use_instruction and int(np.max(instr_len, initial=0)) > 0:
          instr = (t(instr_ids), t(instr_len))
        env_output = StepOutput(t(reward), StepOutputInfo(None, None),
                                t(done), (t(frame), instr))
        out, (c2, h2) = self.agent.step(t(last_action), env_output,
                                        (t(c), t(h)), generator=self._gen)
        res = [out.action, out.policy_logits, out.baseline, c2, h2]
        res = [r.to('cpu', non_blocking=False) for r in res]
    return tuple(r.numpy() for r in res)


class _null(object):
  def __enter__(self):
    return self

  def __exit__(self, *a):
    return False


def make_batched_infer(model, min_batch=1, max_batch=1024, timeout_ms=100):
  return dynamic_batching.batch_fn_with_options(
      minimum_batch_size=min_batch, maximum_batch_size=max_batch,
      timeout_ms=timeout_ms)(model.infer)
