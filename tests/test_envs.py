"""Env stack tests: spaces (port of the reference's
algorithms/spaces/tests/test_spaces.py), native image ops vs numpy
references, every generic gym wrapper, algo utils (GAE, discounted sums,
RunningMeanStd), action distributions, MultiEnv (threads and processes),
and the whole Doom stack on the in-tree simulator backend (all 13 env specs,
action conversion, reward shaping, multiplayer standings, bots, multi-agent
aggregation, the IMPALA adaptor).  The UDP-port check ports
utils/tests/test_utils.py."""

import json
import os

import numpy as np
import pytest
import torch

from scalable_agent_amd.algo import algo_utils
from scalable_agent_amd.algo.action_distributions import (
    CategoricalActionDistribution, TupleActionDistribution, calc_num_logits,
    get_action_distribution, sample_actions_log_probs)
from scalable_agent_amd.algo.multi_agent import MultiAgentWrapper
from scalable_agent_amd.algo.multi_env import MultiEnv
from scalable_agent_amd.algo.spaces import Discretized
from scalable_agent_amd.envs import env_wrappers as ew
from scalable_agent_amd.envs import gym_compat as gym
from scalable_agent_amd.envs.synthetic_gym import SyntheticGymEnv
from scalable_agent_amd.utils.png import decode_png


@pytest.fixture(autouse=True)
def _sim_doom(monkeypatch):
  monkeypatch.setenv('SA_DOOM_BACKEND', 'sim')


# --------------------------------------------------------------- spaces

def test_discretized():
  n, lo, hi = 11, -10.0, 10.0
  space = Discretized(n, lo, hi)
  a = space.sample()
  assert 0 <= a < n
  expected, step = lo, (hi - lo) / (n - 1)
  for action in range(n):
    assert space.to_continuous(action) == pytest.approx(expected)
    expected += step


def test_spaces_sample_contains():
  sp = gym.spaces.Tuple((gym.spaces.Discrete(3), gym.spaces.Box(-1, 1, (2,)),
                         Discretized(5, -1, 1)))
  for _ in range(20):
    assert sp.contains(sp.sample())
  assert not gym.spaces.Discrete(3).contains(3)
  box = gym.spaces.Box(0, 255, (4, 4, 3), dtype=np.uint8)
  assert box.sample().dtype == np.uint8 and box.contains(box.sample())
  d = gym.spaces.Dict({'obs': box, 'm': gym.spaces.Box(0, 1, (2,))})
  assert d.contains(d.sample())


# --------------------------------------------------------------- image ops

def test_resize_nearest_area_linear():
  rng = np.random.RandomState(0)
  img = rng.randint(0, 256, (120, 160, 3), dtype=np.uint8)
  near = ew.resize(img, 80, 60, ew.INTER_NEAREST)
  np.testing.assert_array_equal(near, img[::2, ::2])
  area = ew.resize(img, 80, 60, ew.INTER_AREA).astype(np.float64)
  ref = img.reshape(60, 2, 80, 2, 3).astype(np.float64).mean((1, 3))
  assert np.abs(area - ref).max() <= 0.5 + 1e-6
  # non-integer area factor still preserves the mean brightness
  a2 = ew.resize(img, 128, 72, ew.INTER_AREA)
  assert abs(a2.mean() - img.mean()) < 1.0
  lin = ew.resize(img, 320, 240, ew.INTER_LINEAR)
  assert lin.shape == (240, 320, 3)
  assert abs(lin.astype(float).mean() - img.mean()) < 1.0
  gray = ew.rgb_to_gray(img)
  ref = img @ np.array([0.299, 0.587, 0.114])
  assert np.abs(gray - ref).max() <= 1.0


# --------------------------------------------------------------- wrappers

class _CountEnv(gym.Env):
  """Deterministic env: obs = step counter image/vector."""

  def __init__(self, shape=(8, 8), horizon=10, reward=1.0):
    self.observation_space = gym.spaces.Box(0, 255, shape, dtype=np.uint8)
    self.action_space = gym.spaces.Discrete(2)
    self.reward_range = (-1.0, 1.0)
    self._h, self._r, self.t = horizon, reward, 0

  def _obs(self):
    return np.full(self.observation_space.shape, self.t, np.uint8)

  def reset(self):
    self.t = 0
    return self._obs()

  def step(self, action):
    self.t += 1
    return self._obs(), self._r, self.t >= self._h, {}


def test_stack_skip_wrappers():
  env = ew.StackFramesWrapper(_CountEnv(), 3, channel_config='CHW')
  assert env.observation_space.shape == (3, 8, 8)
  o = env.reset()
  assert o.shape == (3, 8, 8) and o.max() == 0
  o, *_ = env.step(0)
  np.testing.assert_array_equal(o[:, 0, 0], [0, 0, 1])
  env = ew.StackFramesWrapper(_CountEnv(), 2, channel_config='HWC')
  assert env.reset().shape == (8, 8, 2)
  env = ew.SkipFramesWrapper(_CountEnv(horizon=5), 4)
  env.reset()
  o, r, d, info = env.step(0)
  assert (o[0, 0], r, d, info['num_frames']) == (4, 4.0, False, 4)
  o, r, d, info = env.step(0)
  assert (o[0, 0], r, d, info['num_frames']) == (5, 1.0, True, 1)
  env = ew.SkipAndStackFramesWrapper(_CountEnv(), 2, 3, 'CHW')
  env.reset()
  o, r, _, info = env.step(1)
  np.testing.assert_array_equal(o[:, 0, 0], [0, 1, 2])
  assert r == 2.0 and info['num_frames'] == 2


def test_normalize_crop_scale_clip_wrappers():
  base = _CountEnv(shape=(4,))
  base.observation_space = gym.spaces.Box(0.0, 10.0, (4,))
  env = ew.NormalizeWrapper(base)
  base.reset = lambda: np.full(4, 10.0)
  np.testing.assert_allclose(env.reset(), 1.0)
  env = ew.VerticalCropWrapper(_CountEnv(shape=(10, 4, 3)), 6)
  assert env.observation_space.shape == (6, 4, 3)
  assert env.reset().shape == (6, 4, 3)
  env = ew.RewardScalingWrapper(_CountEnv(reward=2.0), 0.5)
  env.reset()
  assert env.step(0)[1] == 1.0 and env.reward_range == (-0.5, 0.5)
  env = ew.ClipRewardWrapper(_CountEnv(reward=9.0))
  env.reset()
  assert env.step(0)[1] == 5.0


def test_resize_wrapper_and_chw():
  env = ew.ResizeWrapper(_CountEnv(shape=(120, 160, 3)), 80, 60,
                         grayscale=True, add_channel_dim=True)
  assert env.observation_space.shape == (60, 80, 1)
  assert env.reset().shape == (60, 80, 1)
  env = ew.PixelFormatChwWrapper(ew.ResizeWrapper(
      _CountEnv(shape=(120, 160, 3)), 80, 60, grayscale=False))
  assert env.observation_space.shape == (3, 60, 80)
  assert env.reset().shape == (3, 60, 80)
  with pytest.raises(Exception, match='already in CHW'):
    ew.PixelFormatChwWrapper(_CountEnv(shape=(3, 60, 80)))


def test_time_limit_and_remaining_time():
  env = ew.TimeLimitWrapper(_CountEnv(horizon=100), limit=3)
  rt = ew.RemainingTimeWrapper(env)
  o = rt.reset()
  assert o['timer'] == 0
  for i in range(3):
    o, _, d, info = rt.step(0)
  assert d and info[ew.TimeLimitWrapper.terminated_by_timer]
  assert o['timer'] == pytest.approx(1.0)
  with pytest.raises(Exception, match='TimeLimitWrapper'):
    ew.RemainingTimeWrapper(_CountEnv())


def test_recording_wrapper(tmp_path):
  env = ew.RecordingWrapper(_CountEnv(shape=(6, 5, 3), horizon=3),
                            str(tmp_path), player_id=1)
  for _ in range(2):
    env.reset()
    done = False
    while not done:
      _, _, done, _ = env.step(np.int64(1))
  env.close()
  root = os.path.join(str(tmp_path), os.listdir(str(tmp_path))[0])
  dirs = sorted(os.listdir(root))
  assert dirs == ['ep_000_p1_r3.00', 'ep_001_p1_r3.00']
  ep = os.path.join(root, dirs[0])
  assert json.load(open(os.path.join(ep, 'actions.json'))) == [1, 1, 1]
  img = decode_png(open(os.path.join(ep, '00002.png'), 'rb').read())
  assert img.shape == (6, 5, 3) and img.max() == 3


# --------------------------------------------------------------- algo utils

def test_discounted_sum_and_gae():
  rng = np.random.RandomState(1)
  T, N, g, lam = 7, 3, 0.9, 0.8
  r = rng.randn(T, N).astype(np.float32)
  d = (rng.rand(T, N) < 0.3).astype(np.float32)
  v = rng.randn(T + 1, N).astype(np.float32)
  adv, ret = algo_utils.calculate_gae(r, d, v, g, lam)
  # naive reference
  adv_ref = np.zeros((T, N))
  ret_ref = np.zeros((T, N))
  for n in range(N):
    for t in range(T):
      a, R, disc_a, disc_r = 0.0, 0.0, 1.0, 1.0
      for k in range(t, T):
        delta = r[k, n] + (1 - d[k, n]) * g * v[k + 1, n] - v[k, n]
        a += disc_a * delta
        R += disc_r * r[k, n]
        if d[k, n]:
          break
        disc_a *= g * lam
        disc_r *= g
      else:
        R += disc_r * v[T, n]
      adv_ref[t, n], ret_ref[t, n] = a, R
  np.testing.assert_allclose(adv, adv_ref, rtol=1e-5, atol=1e-5)
  np.testing.assert_allclose(ret, ret_ref, rtol=1e-5, atol=1e-5)
  assert algo_utils.num_env_steps([{'num_frames': 4}, {}]) == 5


def test_running_mean_std():
  rng = np.random.RandomState(0)
  rms = algo_utils.RunningMeanStd(shape=(3,))
  data = [rng.randn(50, 3) * 2 + 1 for _ in range(4)]
  for x in data:
    rms.update(x)
  allx = np.concatenate(data)
  np.testing.assert_allclose(rms.mean, allx.mean(0), rtol=1e-3)
  np.testing.assert_allclose(rms.var, allx.var(0), rtol=1e-3)


def test_action_distributions():
  torch.manual_seed(0)
  space = gym.spaces.Tuple((gym.spaces.Discrete(3), Discretized(5, -1, 1)))
  assert calc_num_logits(space) == 8
  logits = torch.randn(6, 8)
  dist = get_action_distribution(space, logits)
  assert isinstance(dist, TupleActionDistribution)
  actions, lp = sample_actions_log_probs(dist)
  assert actions.shape == (6, 2)
  ref = (torch.log_softmax(logits[:, :3], 1).gather(1, actions[:, :1]) +
         torch.log_softmax(logits[:, 3:], 1).gather(1, actions[:, 1:]))
  torch.testing.assert_close(lp, ref.squeeze(1))
  torch.testing.assert_close(dist.log_prob(actions), lp)
  ent = dist.entropy()
  p1, p2 = torch.softmax(logits[:, :3], 1), torch.softmax(logits[:, 3:], 1)
  ref_ent = -(p1 * p1.log()).sum(1) - (p2 * p2.log()).sum(1)
  torch.testing.assert_close(ent, ref_ent)
  assert torch.all(dist.kl_divergence(dist).abs() < 1e-6)
  cat = CategoricalActionDistribution(torch.zeros(2, 4))
  assert torch.all(cat.kl_prior().abs() < 1e-6)
  masked = TupleActionDistribution(space, logits, mask=[0])
  torch.testing.assert_close(masked.distributions[1].probs,
                             torch.full((6, 5), 0.2))


# --------------------------------------------------------------- MultiEnv

@pytest.mark.parametrize('use_mp', [False, True])
def test_multi_env(use_mp):
  make = lambda cfg: SyntheticGymEnv(12, 16, episode_length=5)
  me = MultiEnv(4, 2, make, stats_episodes=4, use_multiprocessing=use_mp)
  try:
    obs = me.reset()
    assert len(obs) == 4 and obs[0].shape == (12, 16, 3)
    for _ in range(12):
      obs, rew, dones, infos = me.step([1, 2, 3, 4])
    assert me.stats_num_episodes() >= 8
    assert me.calc_avg_episode_lengths(4) == pytest.approx(20.0, rel=0.6)
    o, r, d = me.predict([[0, 1], [0, 1], [0, 1], [0, 1]])
    assert len(o) == 4 and len(o[0]) == 2
    _, _, dones, _ = me.step([0] * 4, reset=[True, False, False, False])
    assert len(me.info()) == 4
  finally:
    me.close()


def test_multi_agent_wrapper():
  env = MultiAgentWrapper(_CountEnv(horizon=2))
  assert env.num_agents == 1
  assert len(env.reset()) == 1
  obs, rew, done, info = env.step([0])
  obs, rew, done, info = env.step([0])
  assert done == [True] and obs[0].max() == 0  # auto-reset


def test_udp_port():
  from scalable_agent_amd.utils.network import is_udp_port_available
  is_udp_port_available(50301)


# --------------------------------------------------------------- Doom (sim)

def _doom_cfg(name, **overrides):
  from scalable_agent_amd.envs.arguments import default_cfg
  cfg = default_cfg(env=name)
  for k, v in overrides.items():
    setattr(cfg, k, v)
  return cfg


def test_doom_specs_build_and_step():
  from scalable_agent_amd.envs.create_env import create_env
  from scalable_agent_amd.envs.doom.doom_utils import DOOM_ENVS
  for spec in DOOM_ENVS:
    if spec.num_agents > 1:
      continue
    env = create_env(spec.name, cfg=_doom_cfg(spec.name))
    obs = env.reset()
    img = obs['obs'] if isinstance(obs, dict) else obs
    assert img.shape == (3, 72, 128), spec.name
    for _ in range(5):
      obs, r, d, info = env.step(env.action_space.sample())
      assert info['num_frames'] == 4
    if isinstance(obs, dict):
      assert obs['measurements'].shape == (23,)
    env.close()


def test_doom_convert_actions():
  from scalable_agent_amd.envs.doom.action_space import \
      doom_action_space_full_discretized
  from scalable_agent_amd.envs.doom.doom_gym import VizdoomEnv
  env = VizdoomEnv(doom_action_space_full_discretized(with_use=True),
                   'freedm.cfg')
  flat = env._convert_actions((1, 2, 3, 1, 0, 1, 20))
  # fwd/back, right/left, 7 weapon slots, attack, speed, use, turn delta
  assert flat == [1, 0, 0, 1, 0, 0, 1, 0, 0, 0, 0, 1, 0, 1, 12.5]
  assert len(flat) == 15
  assert env.variable_indices['HEALTH'] == 5


def test_doom_reward_shaping_and_stats():
  from scalable_agent_amd.envs.doom.wrappers.multiplayer_stats import \
      MultiplayerStatsWrapper
  from scalable_agent_amd.envs.doom.wrappers.reward_shaping import (
      REWARD_SHAPING_DEATHMATCH_V0, DoomRewardShapingWrapper,
      true_reward_frags)

  class Scripted(gym.Env):
    def __init__(self, infos):
      self.infos = list(infos)
      self.observation_space = gym.spaces.Box(0, 255, (4, 4, 3), np.uint8)
      self.action_space = gym.spaces.Discrete(2)

    def reset(self):
      return np.zeros((4, 4, 3), np.uint8)

    def step(self, a):
      info = dict(self.infos.pop(0))
      return self.reset(), 0.0, not self.infos, info

  base = dict(FRAGCOUNT=0, DEATHCOUNT=0, HEALTH=100, DEAD=0,
              SELECTED_WEAPON=2, SELECTED_WEAPON_AMMO=10, PLAYER_COUNT=3,
              PLAYER_NUMBER=1, PLAYER1_FRAGCOUNT=0, PLAYER2_FRAGCOUNT=1,
              PLAYER3_FRAGCOUNT=0)
  infos = [dict(base), dict(base), dict(base, FRAGCOUNT=1, HEALTH=90,
                                        PLAYER1_FRAGCOUNT=2),
           dict(base, FRAGCOUNT=2, PLAYER1_FRAGCOUNT=2)]
  env = DoomRewardShapingWrapper(MultiplayerStatsWrapper(Scripted(infos)),
                                 REWARD_SHAPING_DEATHMATCH_V0,
                                 true_reward_frags)
  env.reset()
  rews = [env.step(0)[1] for _ in range(3)]
  # step 1: respawn step, no shaping; step 2: no deltas; step 3: +1 frag and
  # -10 health.  Selected-weapon bonus needs 5 steady steps (not yet).
  assert rews[0] == 0.0 and rews[1] == 0.0
  assert rews[2] == pytest.approx(1.0 - 10 * 0.003)
  _, _, done, info = env.step(0)
  assert done and info['true_reward'] == 2
  assert info['FINAL_PLACE'] == 1 and info['LEADER_GAP'] == -1


def test_bot_difficulty_wrapper():
  from scalable_agent_amd.envs.doom.wrappers.bot_difficulty import \
      BotDifficultyWrapper
  env = BotDifficultyWrapper(_CountEnv(horizon=1), 20)
  env._analyze_standings({'FINAL_PLACE': 1, 'LEADER_GAP': -2})
  assert env._curr_difficulty == 30
  env._analyze_standings({'FINAL_PLACE': 4, 'PLAYER_COUNT': 4})
  assert env._curr_difficulty == 20
  assert not BotDifficultyWrapper(_CountEnv(), 150)._adaptive_curriculum


def test_doom_multiagent_aggregator():
  from scalable_agent_amd.envs.doom.doom_utils import make_doom_env
  from scalable_agent_amd.envs.env_utils import create_multi_env
  cfg = _doom_cfg('doom_duel', env_frameskip=2, res_w=32, res_h=24)
  make = lambda env_config: make_doom_env('doom_duel', cfg=cfg,
                                          env_config=env_config)
  me = create_multi_env(4, 1, make, stats_episodes=2,
                        use_multiprocessing=False)
  try:
    assert me.num_agents == 2 and me._num_actors() == 4
    obs = me.reset()
    assert len(obs) == 4 and obs[0]['obs'].shape == (3, 24, 32)
    for _ in range(3):
      obs, rew, dones, infos = me.step([me.action_space.sample()
                                        for _ in range(4)])
    assert len(rew) == 4 and infos[0]['num_frames'] == 2
  finally:
    me.close()


def test_impala_doom_adaptor():
  from scalable_agent_amd.envs.doom import PyProcessDoom
  env = PyProcessDoom('doom_benchmark', {}, 4, 1)
  frame, instr = env.initial()
  assert frame.shape == (72, 128, 3) and frame.dtype == np.uint8
  assert instr == ''
  reward, done, (frame, instr) = env.step(3)
  assert reward.dtype == np.float32 and frame.shape == (72, 128, 3)
  env.close()


def test_doom_backend_error_without_vizdoom(monkeypatch):
  from scalable_agent_amd.envs.doom.doom_gym import doom_backend
  monkeypatch.setenv('SA_DOOM_BACKEND', 'auto')
  try:
    import vizdoom  # noqa: F401
    pytest.skip('vizdoom installed')
  except ImportError:
    pass
  with pytest.raises(ImportError, match='SA_DOOM_BACKEND=sim'):
    doom_backend()
