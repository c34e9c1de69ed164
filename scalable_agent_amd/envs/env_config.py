"""Env-specific CLI arguments and per-env default overrides (reference
envs/env_config.py:1-24).  The reference's MiniGrid branch targets a module
it does not ship and is not replicated."""


def env_override_defaults(env, parser):
  if env.startswith('doom'):
    from .doom.doom_params import doom_override_defaults  # pylint: disable=import-outside-toplevel
    doom_override_defaults(env, parser)
  elif env.startswith('dmlab'):
    from .dmlab.dmlab_params import dmlab_override_defaults  # pylint: disable=import-outside-toplevel
    dmlab_override_defaults(env, parser)
  elif env.startswith('atari'):
    from .atari.atari_params import atari_override_defaults  # pylint: disable=import-outside-toplevel
    atari_override_defaults(env, parser)


def add_env_args(env, parser):
  p = parser
  p.add_argument('--env_frameskip', default=None, type=int,
                 help='Action repeat; None = the environment default')
  p.add_argument('--pixel_format', default='CHW', type=str,
                 help='CHW (PyTorch convention) or HWC')
  if env.startswith('doom'):
    from .doom.doom_params import add_doom_env_args  # pylint: disable=import-outside-toplevel
    add_doom_env_args(env, parser)
