"""Doom-specific CLI arguments and defaults (reference
envs/doom/doom_params.py:5-27)."""

from ...utils.utils import str2bool


def doom_override_defaults(env, parser):
  del env
  parser.set_defaults(encoder='convnet_simple', hidden_size=512,
                      obs_subtract_mean=128.0, obs_scale=128.0,
                      env_frameskip=4)


def add_doom_env_args(env, parser):
  del env
  p = parser
  p.add_argument('--num_agents', default=-1, type=int,
                 help='Number of agents (fewer than players lets humans '
                 'join); -1 = the env default')
  p.add_argument('--num_humans', default=0, type=int,
                 help='Human players joining the match')
  p.add_argument('--num_bots', default=-1, type=int,
                 help='Classic (non-neural) bots; -1 = the env default')
  p.add_argument('--start_bot_difficulty', default=None, type=int,
                 help='Initial bot difficulty (useful for evaluation)')
  p.add_argument('--res_w', default=128, type=int,
                 help='Game frame width after resize')
  p.add_argument('--res_h', default=72, type=int,
                 help='Game frame height after resize')
  p.add_argument('--wide_aspect_ratio', default=True, type=str2bool,
                 help='Render wide aspect ratio (better FOV, slower)')
  p.add_argument('--doom_backend', default='auto', type=str,
                 choices=['auto', 'vizdoom', 'sim'],
                 help="'sim' = in-tree simulator test double")
