"""Atari defaults (reference envs/atari/atari_params.py)."""


def atari_override_defaults(env, parser):
  del env
  parser.set_defaults(encoder='convnet_simple', hidden_size=512,
                      obs_subtract_mean=128.0, obs_scale=128.0, gamma=0.99,
                      reward_clip=1.0, env_frameskip=4, prior_loss_coeff=0.01)
