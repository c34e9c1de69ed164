"""Atari env specs and factory (reference envs/atari/atari_utils.py):
NoFrameskip-v4 games, 84x84 grayscale (nearest), skip 4 + stack 4 (CHW).
Needs gym with the ALE; raises a clear ImportError otherwise."""

from ..env_wrappers import ResizeWrapper, SkipAndStackFramesWrapper

ATARI_W = ATARI_H = 84


class AtariSpec(object):

  def __init__(self, name, env_id, default_timeout=None):
    self.name = name
    self.env_id = env_id
    self.default_timeout = default_timeout
    self.has_timer = False


ATARI_ENVS = [
    AtariSpec('atari_montezuma', 'MontezumaRevengeNoFrameskip-v4',
              default_timeout=18000),
    AtariSpec('atari_pong', 'PongNoFrameskip-v4'),
    AtariSpec('atari_qbert', 'QbertNoFrameskip-v4'),
    AtariSpec('atari_breakout', 'BreakoutNoFrameskip-v4'),
    AtariSpec('atari_spaceinvaders', 'SpaceInvadersNoFrameskip-v4'),
    AtariSpec('atari_asteroids', 'AsteroidsNoFrameskip-v4'),
    AtariSpec('atari_gravitar', 'GravitarNoFrameskip-v4'),
    AtariSpec('atari_mspacman', 'MsPacmanNoFrameskip-v4'),
    AtariSpec('atari_seaquest', 'SeaquestNoFrameskip-v4'),
]


def atari_env_by_name(name):
  for spec in ATARI_ENVS:
    if spec.name == name:
      return spec
  raise Exception('Unknown Atari env')


def make_atari_env(env_name, cfg, **kwargs):
  del kwargs
  spec = atari_env_by_name(env_name)
  try:
    import gym  # pylint: disable=import-outside-toplevel
  except ImportError as e:
    raise ImportError('Atari envs need gym with the Arcade Learning '
                      'Environment installed') from e
  env = gym.make(spec.env_id)
  if spec.default_timeout is not None:
    env._max_episode_steps = spec.default_timeout
  assert 'NoFrameskip' in env.spec.id
  env = ResizeWrapper(env, ATARI_W, ATARI_H, grayscale=True,
                      add_channel_dim=False, area_interpolation=False)
  skip = cfg.env_frameskip if cfg.env_frameskip is not None else 4
  return SkipAndStackFramesWrapper(env, skip_frames=skip, stack_frames=4,
                                   channel_config='CHW')
