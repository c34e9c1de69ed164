"""The learner process's stream plan (parallel/streams.py): every stream of
the learner / data-parallel path is created once, in a fixed order, so the
hardware queue each lands on does not depend on how many captures or
measurements ran before it (the measured queue map is
profiles/r6_dp_queues.txt)."""

import os
import re

import torch

from scalable_agent_amd import parallel
from scalable_agent_amd.parallel import streams

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Fake(object):
  made = []

  def __init__(self, device):
    self.device = device
    _Fake.made.append(self)


def test_plan_order_and_reuse():
  streams.reset_stream_plans()
  _Fake.made = []
  try:
    p = parallel.stream_plan('cpu', factory=_Fake)
    # copy and early first: the two pool streams that measured on queues of
    # their own (parallel/streams.py, profiles/r6_dp_queues.txt)
    assert streams.ORDER == ('copy', 'early', 'capture')
    assert [p.copy, p.early, p.capture] == _Fake.made  # creation order
    # a second request (another capture, another measurement) makes nothing
    q = parallel.stream_plan(torch.device('cpu'), factory=_Fake)
    assert q is p and len(_Fake.made) == 3
  finally:
    streams.reset_stream_plans()


def test_learner_path_creates_streams_only_through_the_plan():
  """No stream of the learner step, the bench loop or the training feeder is
  created outside the plan (a stray torch.cuda.Stream() there would move
  every later stream to another hardware queue)."""
  for rel in ('scalable_agent_amd/learner.py', 'bench.py',
              'scalable_agent_amd/experiment.py',
              'scalable_agent_amd/parallel/dist.py'):
    src = open(os.path.join(ROOT, rel)).read()
    assert not re.search(r'torch\.cuda\.Stream\(', src), rel
  src = open(os.path.join(ROOT, 'scalable_agent_amd/learner.py')).read()
  assert 'stream_plan(self.device).capture' in src
  assert 'stream_plan(self.device).early' in src


def test_warmup_collective_without_group_is_a_noop():
  parallel.warmup_collective(torch.device('cpu'))


def test_split_keeps_the_sentinel_in_the_late_bucket():
  """The DP step guard's NaN sentinel is written after the early bucket has
  gone out, so it must sit past the split (GradientSynchronizer.set_split)."""
  import pytest

  class Flat(object):
    numel = 1000
    sentinel = 900
    grads = torch.zeros(1000)

  gs = parallel.GradientSynchronizer(Flat())
  gs.set_split(800)
  assert gs.split == 800
  with pytest.raises(AssertionError):
    gs.set_split(950)
