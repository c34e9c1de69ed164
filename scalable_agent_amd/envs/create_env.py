"""Env dispatcher by name prefix (reference envs/create_env.py):
doom_* -> ViZDoom, atari_* -> ALE via gym, dmlab_* -> DeepMind Lab gym env,
synthetic_* -> in-tree synthetic gym env (no simulator needed)."""


def create_env(env, **kwargs):
  if env.startswith('doom_'):
    from .doom.doom_utils import make_doom_env  # pylint: disable=import-outside-toplevel
    return make_doom_env(env, **kwargs)
  if env.startswith('atari_'):
    from .atari.atari_utils import make_atari_env  # pylint: disable=import-outside-toplevel
    return make_atari_env(env, **kwargs)
  if env.startswith('dmlab_'):
    from .dmlab.dmlab_utils import make_dmlab_env  # pylint: disable=import-outside-toplevel
    return make_dmlab_env(env, **kwargs)
  if env.startswith('synthetic_'):
    from .synthetic_gym import make_synthetic_gym_env  # pylint: disable=import-outside-toplevel
    return make_synthetic_gym_env(env, **kwargs)
  raise Exception('Unsupported env {0}'.format(env))
