"""Replays a recorded ViZDoom demo (.lmp) and dumps its frames as PNGs
(reference envs/doom/doom_play_demo.py)."""

import argparse
import os
import shutil
import sys

from ..arguments import default_cfg
from ...utils.png import write_png
from ...utils.utils import log
from .doom_utils import make_doom_env


def main(argv=None):
  parser = argparse.ArgumentParser()
  parser.add_argument('--env', type=str, required=True)
  parser.add_argument('--demo_path', type=str, required=True)
  args = parser.parse_args(argv)
  env = make_doom_env(args.env, cfg=default_cfg(env=args.env),
                      custom_resolution='1920x1080')
  env.unwrapped.mode = 'replay'
  env.unwrapped.initialize()
  game = env.unwrapped.game
  game.replay_episode(args.demo_path)
  frames_dir = args.demo_path + '_frames'
  if os.path.exists(frames_dir):
    shutil.rmtree(frames_dir)
  os.makedirs(frames_dir)
  frame_id = 0
  while not game.is_episode_finished():
    game.advance_action()
    img = env.render(mode='rgb_array')
    if img is not None:
      write_png(os.path.join(frames_dir, '%05d.png' % frame_id), img)
    frame_id += 1
    log.debug('Reward %.3f at frame %d', game.get_last_reward(), frame_id)
  game.close()
  return 0


if __name__ == '__main__':
  sys.exit(main())
