"""Synthetic environment and synthetic trajectory batches.

The image has neither DeepMind Lab nor ViZDoom, so a synthetic env is the
first-class fake backend and the benchmark data source:
random uint8 frames of a configurable shape, random rewards, geometric episode
lengths, an optional instruction string.  Interface = the reference env
protocol (`initial()`, `step(action)`, `close()`, environments.py:66-140).
"""

import numpy as np
import torch

from ..structs import ActorOutput, AgentOutput, StepOutput, StepOutputInfo


LEARNABLE_LEVELS = ('synthetic_cue', 'synthetic_memory')


def _action_index(action, num_actions):
  """Index of `action` in the action set: a scalar index (Doom style) or a
  row of environments.DEFAULT_ACTION_SET (the DMLab-style actor output)."""
  a = np.asarray(action)
  if a.ndim == 0:
    return int(a)
  from ..environments import DEFAULT_ACTION_SET
  for i, row in enumerate(DEFAULT_ACTION_SET[:num_actions]):
    if np.array_equal(a, np.asarray(row)):
      return i
  return -1


class SyntheticEnv(object):
  """Synthetic env with the PyProcessDmLab interface.

  Levels:
    'synthetic' (any other name): random frames from a pool, random rewards,
        geometric episode lengths - the throughput/plumbing level;
    'synthetic_cue': each frame shows one of `num_actions` bright vertical
        bands; acting with that band's index is rewarded +1 on the next step
        (a reactive policy reaches one reward per step, a random one 1/A);
        fixed `episode_length` steps;
    'synthetic_memory': the band is shown only on the episode's first frame,
        later frames are noise; every step whose action matches it is
        rewarded +1 (needs the LSTM to carry the cue).
  """

  def __init__(self, level='synthetic', config=None, num_action_repeats=4,
               seed=1, frame_shape=(72, 96, 3), episode_length=200,
               instruction='', num_actions=9, frame_pool=16):
    config = config or {}
    self._rng = np.random.RandomState(seed)
    self._repeats = num_action_repeats
    self._shape = tuple(frame_shape)
    self._p_done = 1.0 / max(1, episode_length)
    self._episode_length = max(1, int(episode_length))
    self._instruction = instruction
    self.num_actions = num_actions
    self.benchmark_mode = bool(config.get('benchmark_mode', 0))
    self.level = level
    self._kind = level if level in LEARNABLE_LEVELS else 'synthetic'
    # a pool of pre-generated frames keeps the env cheap (throughput tests)
    self._frames = self._rng.randint(
        0, 256, size=(frame_pool,) + self._shape, dtype=np.uint8)
    if self._kind != 'synthetic':
      h, w = self._shape[0], self._shape[1]
      noise = self._rng.randint(0, 48, size=self._shape, dtype=np.uint8)
      self._blank = noise
      self._cues = []
      band = max(1, w // num_actions)
      for k in range(num_actions):
        f = noise.copy()
        f[:, k * band:(k + 1) * band] = 255
        self._cues.append(f)
      self._cue = 0
      self._step_in_episode = 0
    self._t = 0
    self.closed = False

  def _obs(self):
    self._t += 1
    if self._kind == 'synthetic':
      return [self._frames[self._t % len(self._frames)], self._instruction]
    if self._kind == 'synthetic_cue' or self._step_in_episode == 0:
      return [self._cues[self._cue], self._instruction]
    return [self._blank, self._instruction]

  def _new_episode(self):
    self._step_in_episode = 0
    self._cue = self._rng.randint(self.num_actions)

  def initial(self):
    if self._kind != 'synthetic':
      self._new_episode()
    return self._obs()

  def step(self, action):
    if self._kind == 'synthetic':
      reward = np.float32(self._rng.randint(-1, 2) * (self._rng.rand() < 0.1))
      done = np.array(self._rng.rand() < self._p_done)
      return reward, done, self._obs()
    if self.benchmark_mode:
      action = self._rng.randint(self.num_actions)
    a = _action_index(action, self.num_actions)
    reward = np.float32(1.0 if a == self._cue else 0.0)
    self._step_in_episode += 1
    done = self._step_in_episode >= self._episode_length
    if done:
      self._new_episode()
    elif self._kind == 'synthetic_cue':
      self._cue = self._rng.randint(self.num_actions)
    return reward, np.array(done), self._obs()

  def close(self):
    self.closed = True

  @staticmethod
  def _tensor_specs(method_name, unused_kwargs, constructor_kwargs):
    shape = tuple(constructor_kwargs.get('frame_shape', (72, 96, 3)))
    obs = [(shape, np.uint8), ((), object)]
    if method_name == 'initial':
      return obs
    elif method_name == 'step':
      return (((), np.float32), ((), np.bool_), obs)


def make_synthetic_batch(batch_size, unroll_length, frame_shape, num_actions,
                         seed=0, pin_memory=False, device='cpu',
                         done_prob=0.005, core_size=256):
  """A time-major ActorOutput with T+1 steps of synthetic data."""
  g = torch.Generator().manual_seed(seed)
  T1, B = unroll_length + 1, batch_size
  frame = torch.randint(0, 256, (T1, B) + tuple(frame_shape), generator=g,
                        dtype=torch.uint8)
  reward = (torch.randint(-1, 2, (T1, B), generator=g).float() *
            (torch.rand(T1, B, generator=g) < 0.1).float())
  done = torch.rand(T1, B, generator=g) < done_prob
  done[0] = True
  ep_ret = torch.randn(T1, B, generator=g)
  ep_step = torch.randint(0, 1000, (T1, B), generator=g, dtype=torch.int32)
  action = torch.randint(0, num_actions, (T1, B), generator=g,
                         dtype=torch.int64)
  logits = torch.randn(T1, B, num_actions, generator=g)
  baseline = torch.randn(T1, B, generator=g)
  c = torch.randn(B, core_size, generator=g) * 0.1
  h = torch.randn(B, core_size, generator=g) * 0.1
  out = ActorOutput(
      level_name='synthetic', agent_state=(c, h),
      env_outputs=StepOutput(reward, StepOutputInfo(ep_ret, ep_step), done,
                             (frame, None)),
      agent_outputs=AgentOutput(action, logits, baseline))
  if pin_memory or device != 'cpu':
    from ..learner import _map_tensors
    if pin_memory:
      out = _map_tensors(out, lambda t: t.pin_memory())
    if device != 'cpu':
      out = _map_tensors(out, lambda t: t.to(device))
  return out


def add_synthetic_instructions(batch, vocab, seed=0, max_len=16):
  """Adds DMLab-style instruction observations to a time-major batch:
  word ids [T+1, B, max_len] (< vocab, zero past the length) and lengths
  [T+1, B] in 0..max_len (0 = no instruction on that step)."""
  g = torch.Generator().manual_seed(seed)
  T1, B = batch.env_outputs.reward.shape
  ids = torch.randint(1, vocab, (T1, B, max_len), generator=g)
  lengths = torch.randint(0, max_len + 1, (T1, B), generator=g)
  ids = ids * (torch.arange(max_len).view(1, 1, max_len) <
               lengths.unsqueeze(-1))
  eo = batch.env_outputs
  return batch._replace(env_outputs=eo._replace(
      observation=(eo.observation[0], (ids, lengths))))
