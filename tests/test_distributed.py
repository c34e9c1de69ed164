"""Data-parallel learners without a cluster: gloo
process group, world size 2, CPU.  N learners x batch B with grad_reduce=sum
must equal one learner with batch N*B under the reference's sum losses."""

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from scalable_agent_amd import flags as flags_lib
from scalable_agent_amd.envs.synthetic import make_synthetic_batch
from scalable_agent_amd.learner import Learner, _map_tensors
from scalable_agent_amd.models import Agent

T, B, SHAPE = 5, 4, (16, 24, 3)


def _free_port():
  s = socket.socket()
  s.bind(('127.0.0.1', 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _slice_batch(batch, lo, hi):
  out = _map_tensors(batch, lambda t: t)
  def sl_time(t):
    return t[:, lo:hi]
  env = out.env_outputs
  return out._replace(
      agent_state=(out.agent_state[0][lo:hi], out.agent_state[1][lo:hi]),
      env_outputs=env._replace(
          reward=sl_time(env.reward), done=sl_time(env.done),
          info=env.info._replace(episode_return=sl_time(env.info.episode_return),
                                 episode_step=sl_time(env.info.episode_step)),
          observation=(sl_time(env.observation[0]), None)),
      agent_outputs=out.agent_outputs._replace(
          action=sl_time(out.agent_outputs.action),
          policy_logits=sl_time(out.agent_outputs.policy_logits),
          baseline=sl_time(out.agent_outputs.baseline)))


def _worker(rank, world, port, result_path, overlap=True, reduce='sum'):
  os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                    MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
  from scalable_agent_amd import parallel
  parallel.init_distributed(backend='gloo')
  torch.manual_seed(0)
  f = flags_lib.default_flags(batch_size=B // world, unroll_length=T,
                              torso='shallow', grad_reduce=reduce,
                              grad_overlap=overlap)
  agent = Agent(9, torso='shallow', frame_shape=SHAPE, seed=rank + 10)
  learner = Learner(agent, f, 'cpu', world_size=world)
  # two-phase backward (early all-reduce of heads/core/FC under the torso
  # backward) exactly when asked
  assert learner._split == overlap
  parallel.broadcast_params(learner.flat.params)   # rank 0's init wins
  full = make_synthetic_batch(B, T, SHAPE, 9, seed=7)
  per = B // world
  learner.step(_slice_batch(full, rank * per, (rank + 1) * per))
  learner.step(_slice_batch(full, rank * per, (rank + 1) * per))
  assert parallel.param_checksum_consistent(learner.flat.params)
  if rank == 0:
    torch.save({'params': learner.flat.params.clone(),
                'frames': int(learner.frames)}, result_path)
  parallel.cleanup()


@pytest.mark.parametrize('overlap', [True, False])
def test_dp_sum_equals_single_learner_with_full_batch(tmp_path, overlap):
  path = str(tmp_path / 'dp.pt')
  mp.spawn(_worker, args=(2, _free_port(), path, overlap), nprocs=2, join=True)
  dp = torch.load(path, weights_only=True)
  # single learner, full batch, same init as rank 0
  torch.manual_seed(0)
  f = flags_lib.default_flags(batch_size=B, unroll_length=T, torso='shallow')
  agent = Agent(9, torso='shallow', frame_shape=SHAPE, seed=10)
  learner = Learner(agent, f, 'cpu')
  full = make_synthetic_batch(B, T, SHAPE, 9, seed=7)
  learner.step(full)
  learner.step(full)
  assert dp['frames'] == int(learner.frames)
  torch.testing.assert_close(dp['params'], learner.flat.params, rtol=1e-4,
                             atol=1e-6)


def test_dp_mean_equals_single_learner_with_grad_scale(tmp_path):
  """--grad_reduce=mean (the 1/world folded into the RMSProp update) over N
  learners x B == one learner with N*B and --grad_scale 1/N: the single-GPU
  stand-in used to pick the data-parallel default
  (profiles/r4_learning_dp_equiv.md)."""
  path = str(tmp_path / 'dp_mean.pt')
  mp.spawn(_worker, args=(2, _free_port(), path, True, 'mean'), nprocs=2,
           join=True)
  dp = torch.load(path, weights_only=True)
  torch.manual_seed(0)
  f = flags_lib.default_flags(batch_size=B, unroll_length=T, torso='shallow',
                              grad_scale=0.5)
  agent = Agent(9, torso='shallow', frame_shape=SHAPE, seed=10)
  learner = Learner(agent, f, 'cpu')
  full = make_synthetic_batch(B, T, SHAPE, 9, seed=7)
  learner.step(full)
  learner.step(full)
  torch.testing.assert_close(dp['params'], learner.flat.params, rtol=1e-4,
                             atol=1e-6)
  # and it is NOT the sum semantics
  f2 = flags_lib.default_flags(batch_size=B, unroll_length=T, torso='shallow')
  ref = Learner(Agent(9, torso='shallow', frame_shape=SHAPE, seed=10), f2, 'cpu')
  ref.step(full)
  ref.step(full)
  assert not torch.allclose(dp['params'], ref.flat.params, rtol=1e-4, atol=1e-6)


def test_default_reduction_is_mean():
  """Data-parallel default (profiles/r4_learning_dp_equiv.md: at the B=256
  single-learner equivalent of 8 ranks the summed gradient does not learn at
  the reference learning rate, the 1/N-scaled one does)."""
  assert flags_lib.default_flags().grad_reduce == 'mean'


def _poison_worker(rank, world, port, result_path):
  os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                    MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
  from scalable_agent_amd import parallel
  parallel.init_distributed(backend='gloo')
  f = flags_lib.default_flags(batch_size=B // world, unroll_length=T,
                              torso='shallow')
  learner = Learner(Agent(9, torso='shallow', frame_shape=SHAPE, seed=10), f,
                    'cpu', world_size=world)
  parallel.broadcast_params(learner.flat.params)
  sync = learner.grad_sync
  real = sync.all_reduce
  state = {'poison': rank == 1}

  def all_reduce():
    # what ops.poison_on_error does on a GPU rank whose error words are set
    if state['poison']:
      learner.flat.grads[learner.flat.sentinel] = float('nan')
      state['poison'] = False
    real()

  sync.all_reduce = all_reduce
  full = make_synthetic_batch(B, T, SHAPE, 9, seed=7)
  per = B // world
  mine = _slice_batch(full, rank * per, (rank + 1) * per)
  p0 = learner.flat.params.clone()
  learner.step(mine)
  skipped_first = torch.equal(learner.flat.params, p0)
  consistent = parallel.param_checksum_consistent(learner.flat.params)
  learner.step(mine)
  torch.save({'skipped_first': skipped_first, 'consistent': consistent,
              'applied_second': not torch.equal(learner.flat.params, p0),
              'consistent2': parallel.param_checksum_consistent(
                  learner.flat.params),
              'skipped': learner.opt.skipped_steps,
              'sentinel': float(learner.flat.params[learner.flat.sentinel])},
             '%s.%d' % (result_path, rank))
  parallel.cleanup()


def test_poisoned_sentinel_skips_the_step_on_every_rank(tmp_path):
  """The DP step guard's transport: a NaN in one rank's gradient sentinel
  reaches every rank through the all-reduce, so all skip the same step and
  the replicas stay identical; the next step applies everywhere."""
  path = str(tmp_path / 'poison.pt')
  mp.spawn(_poison_worker, args=(2, _free_port(), path), nprocs=2, join=True)
  for r in (0, 1):
    rec = torch.load('%s.%d' % (path, r), weights_only=True)
    assert rec['skipped_first'] and rec['consistent']
    assert rec['applied_second'] and rec['consistent2']
    assert rec['skipped'] == 1
    assert rec['sentinel'] == 0.0
