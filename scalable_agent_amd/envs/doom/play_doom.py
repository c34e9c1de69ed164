"""Human play against bots (reference envs/doom/play_doom.py; needs pynput
and a display).  The reference names `doom_freedm`, which is not one of its
specs; `doom_deathmatch_full` (freedm.cfg) is used."""

import sys

from ..arguments import default_cfg
from .doom_gym import VizdoomEnv
from .doom_utils import doom_env_by_name, make_doom_multiplayer_env


def main(env_name='doom_deathmatch_full'):
  cfg = default_cfg(env=env_name)
  cfg.num_agents = 1
  cfg.num_bots = 7
  env = make_doom_multiplayer_env(doom_env_by_name(env_name), cfg=cfg,
                                  custom_resolution='1280x720')
  return VizdoomEnv.play_human_mode(env, skip_frames=2, num_actions=15)


if __name__ == '__main__':
  sys.exit(main())
