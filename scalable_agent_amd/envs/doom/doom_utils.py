"""Doom env specs and factories (reference envs/doom/doom_utils.py:18-268).

`DOOM_ENVS` lists the 15 named environments (scenario cfg, action space,
reward scale, default timeout, agents/bots, respawn delay, extra wrappers).
`make_doom_env(name, cfg=...)` builds the wrapper chain:

  VizdoomEnv | VizdoomEnvMultiplayer
  -> [RecordingWrapper] -> MultiplayerStatsWrapper -> [BotDifficultyWrapper]
  -> SetResolutionWrapper -> [ResizeWrapper to cfg.res_w x cfg.res_h]
  -> [TimeLimitWrapper] -> [PixelFormatChwWrapper] -> extra wrappers
  -> [RewardScalingWrapper]

and routes specs with several agents or bots through the multiplayer
factory (MultiAgentEnv for >1 agents, a single hosting player otherwise).
"""

from ..env_wrappers import (PixelFormatChwWrapper, RecordingWrapper,
                            ResizeWrapper, RewardScalingWrapper,
                            TimeLimitWrapper)
from ..gym_compat import Discrete
from ...utils.utils import log
from .action_space import (doom_action_space, doom_action_space_basic,
                           doom_action_space_discretized_no_weap,
                           doom_action_space_full_discretized)
from .doom_gym import VizdoomEnv
from .wrappers.additional_input import DoomAdditionalInput
from .wrappers.bot_difficulty import BotDifficultyWrapper
from .wrappers.multiplayer_stats import MultiplayerStatsWrapper
from .wrappers.observation_space import SetResolutionWrapper, resolutions
from .wrappers.reward_shaping import (REWARD_SHAPING_BATTLE,
                                      REWARD_SHAPING_DEATHMATCH_V0,
                                      REWARD_SHAPING_DEATHMATCH_V1,
                                      DoomRewardShapingWrapper,
                                      true_reward_final_position,
                                      true_reward_frags)
from .wrappers.scenario_wrappers.gathering_reward_shaping import \
    DoomGatheringRewardShaping


class DoomSpec(object):

  def __init__(self, name, env_spec_file, action_space, reward_scaling=1.0,
               default_timeout=-1, num_agents=1, num_bots=0, respawn_delay=0,
               extra_wrappers=None):
    self.name = name
    self.env_spec_file = env_spec_file
    self.action_space = action_space
    self.reward_scaling = reward_scaling
    self.default_timeout = default_timeout
    self.num_agents = num_agents      # 1 = single player
    self.num_bots = num_bots          # CLI --num_bots overrides
    self.respawn_delay = respawn_delay
    self.extra_wrappers = extra_wrappers  # [(wrapper_cls, kwargs)]


ADDITIONAL_INPUT = (DoomAdditionalInput, {})
BATTLE_REWARD_SHAPING = (DoomRewardShapingWrapper, dict(
    reward_shaping_scheme=REWARD_SHAPING_BATTLE, true_reward_func=None))
BOTS_REWARD_SHAPING = (DoomRewardShapingWrapper, dict(
    reward_shaping_scheme=REWARD_SHAPING_DEATHMATCH_V0,
    true_reward_func=true_reward_frags))
DEATHMATCH_REWARD_SHAPING = (DoomRewardShapingWrapper, dict(
    reward_shaping_scheme=REWARD_SHAPING_DEATHMATCH_V1,
    true_reward_func=true_reward_final_position))

_DM = [ADDITIONAL_INPUT, DEATHMATCH_REWARD_SHAPING]

DOOM_ENVS = [
    DoomSpec('doom_basic', 'basic.cfg', Discrete(1 + 3), 0.01, 300),
    DoomSpec('doom_corridor', 'deadly_corridor.cfg', Discrete(1 + 7), 0.01,
             2100),
    DoomSpec('doom_gathering', 'health_gathering.cfg', Discrete(1 + 3), 0.01,
             2100),
    DoomSpec('doom_two_colors_easy', 'two_colors_easy.cfg',
             doom_action_space_basic(),
             extra_wrappers=[(DoomGatheringRewardShaping, {})]),
    DoomSpec('doom_two_colors_hard', 'two_colors_hard.cfg',
             doom_action_space_basic(),
             extra_wrappers=[(DoomGatheringRewardShaping, {})]),
    DoomSpec('doom_dm', 'cig.cfg', doom_action_space(), 1.0, int(1e9),
             num_agents=8, extra_wrappers=_DM),
    DoomSpec('doom_dwango5', 'dwango5_dm.cfg', doom_action_space(), 1.0,
             int(1e9), num_agents=8, extra_wrappers=_DM),
    # single-player envs of the paper
    DoomSpec('doom_battle', 'battle_continuous_turning.cfg',
             doom_action_space_discretized_no_weap(), 1.0, 2100,
             extra_wrappers=[ADDITIONAL_INPUT, BATTLE_REWARD_SHAPING]),
    DoomSpec('doom_battle2', 'battle2_continuous_turning.cfg',
             doom_action_space_discretized_no_weap(), 1.0, 2100,
             extra_wrappers=[ADDITIONAL_INPUT, BATTLE_REWARD_SHAPING]),
    # one agent against bots
    DoomSpec('doom_deathmatch_bots', 'dwango5_dm_continuous_weap.cfg',
             doom_action_space_full_discretized(), 1.0, int(1e9),
             num_agents=1, num_bots=7,
             extra_wrappers=[ADDITIONAL_INPUT, BOTS_REWARD_SHAPING]),
    # self-play / PBT
    DoomSpec('doom_duel', 'ssl2.cfg',
             doom_action_space_full_discretized(with_use=True), 1.0,
             int(1e9), num_agents=2, num_bots=0, respawn_delay=2,
             extra_wrappers=_DM),
    DoomSpec('doom_deathmatch_full', 'freedm.cfg',
             doom_action_space_full_discretized(with_use=True), 1.0,
             int(1e9), num_agents=4, num_bots=4, respawn_delay=2,
             extra_wrappers=_DM),
    # throughput benchmark: doom_battle map, simple 9-way discrete actions,
    # no extra inputs; 128x72 frames from 160x120, frameskip 4
    DoomSpec('doom_benchmark', 'battle.cfg', Discrete(1 + 8), 1.0, 2100),
]


def doom_env_by_name(name):
  for spec in DOOM_ENVS:
    if spec.name == name:
      return spec
  raise Exception('Unknown Doom env')


def _cfg(cfg, key, default=None):
  if cfg is None:
    return default
  if isinstance(cfg, dict):
    return cfg.get(key, default)
  return getattr(cfg, key, default)


def make_doom_env_impl(doom_spec, cfg=None, env_config=None, skip_frames=None,
                       episode_horizon=None, player_id=None, num_agents=None,
                       max_num_players=None, num_bots=0,
                       custom_resolution=None, **kwargs):
  del kwargs
  skip_frames = skip_frames if skip_frames is not None else \
      _cfg(cfg, 'env_frameskip', 4)
  fps = _cfg(cfg, 'fps')
  async_mode = fps == 0
  backend = _cfg(cfg, 'doom_backend')
  backend = None if backend == 'auto' else backend
  if player_id is None:
    env = VizdoomEnv(doom_spec.action_space, doom_spec.env_spec_file,
                     skip_frames=skip_frames, async_mode=async_mode,
                     backend=backend)
  else:
    from .multiplayer.doom_multiagent import VizdoomEnvMultiplayer  # pylint: disable=import-outside-toplevel
    env = VizdoomEnvMultiplayer(
        doom_spec.action_space, doom_spec.env_spec_file, player_id=player_id,
        num_agents=num_agents, max_num_players=max_num_players,
        num_bots=num_bots, skip_frames=skip_frames, async_mode=async_mode,
        respawn_delay=doom_spec.respawn_delay, backend=backend)

  record_to = _cfg(cfg, 'record_to')
  should_record = env_config is None or (
      env_config.worker_index == 0 and env_config.vector_index == 0 and
      (player_id is None or player_id <= 1))
  if record_to is not None and should_record:
    env = RecordingWrapper(env, record_to, player_id)

  env = MultiplayerStatsWrapper(env)
  if num_bots > 0:
    env = BotDifficultyWrapper(env, _cfg(cfg, 'start_bot_difficulty'))

  resolution = custom_resolution
  if resolution is None:
    resolution = '256x144' if _cfg(cfg, 'wide_aspect_ratio', True) \
        else '160x120'
  assert resolution in resolutions
  env = SetResolutionWrapper(env, resolution)

  res_w, res_h = _cfg(cfg, 'res_w', 128), _cfg(cfg, 'res_h', 72)
  h, w, _ = env.observation_space.shape
  if w != res_w or h != res_h:
    env = ResizeWrapper(env, res_w, res_h, grayscale=False)
  log.info('Doom resolution: %s, resize resolution: %r', resolution,
           (res_w, res_h))

  timeout = doom_spec.default_timeout
  if episode_horizon is not None and episode_horizon > 0:
    timeout = episode_horizon
  if timeout > 0:
    env = TimeLimitWrapper(env, limit=timeout, random_variation_steps=0)

  if _cfg(cfg, 'pixel_format', 'HWC') == 'CHW':
    env = PixelFormatChwWrapper(env)

  for wrapper_cls, wrapper_kwargs in doom_spec.extra_wrappers or []:
    env = wrapper_cls(env, **wrapper_kwargs)

  if doom_spec.reward_scaling != 1.0:
    env = RewardScalingWrapper(env, doom_spec.reward_scaling)
  return env


def make_doom_multiplayer_env(doom_spec, cfg=None, env_config=None, **kwargs):
  skip_frames = _cfg(cfg, 'env_frameskip', 4)
  cli_bots = _cfg(cfg, 'num_bots', -1)
  num_bots = doom_spec.num_bots if cli_bots < 0 else cli_bots
  cli_agents = _cfg(cfg, 'num_agents', -1)
  num_agents = doom_spec.num_agents if cli_agents <= 0 else cli_agents
  max_num_players = num_agents + _cfg(cfg, 'num_humans', 0)
  is_multiagent = num_agents > 1

  def make_env_func(player_id):
    return make_doom_env_impl(
        doom_spec, cfg=cfg, player_id=player_id, num_agents=num_agents,
        max_num_players=max_num_players, num_bots=num_bots,
        # multi-agent frame skipping is done by the wrapper
        skip_frames=1 if is_multiagent else skip_frames,
        env_config=env_config, **kwargs)

  if is_multiagent:
    from .multiplayer.doom_multiagent_wrapper import MultiAgentEnv  # pylint: disable=import-outside-toplevel
    return MultiAgentEnv(num_agents=num_agents, make_env_func=make_env_func,
                         env_config=env_config, skip_frames=skip_frames)
  from .multiplayer.doom_multiagent_wrapper import init_multiplayer_env  # pylint: disable=import-outside-toplevel
  return init_multiplayer_env(make_env_func, player_id=0,
                              env_config=env_config)


def make_doom_env(env_name, **kwargs):
  spec = doom_env_by_name(env_name)
  if spec.num_agents > 1 or spec.num_bots > 0:
    return make_doom_multiplayer_env(spec, **kwargs)
  return make_doom_env_impl(spec, **kwargs)
