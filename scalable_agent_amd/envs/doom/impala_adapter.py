"""IMPALA adaptor for VizDoom (reference environments_doom.py:12-97).

Always creates `doom_benchmark` (ignoring level/seed/repeats like the
reference), renders 128x72 RGB HWC frames, instruction ''.  The initial reset
is serialised across processes with a file lock (ViZDoom instances fight over
shared resources at start-up).
"""

import numpy as np

DOOM_W = 128
DOOM_H = 72

# use the same number of actions as dmlab
DOOM_ACTION_SET = (
    0,  # MOVE_FORWARD
    1,  # MOVE_BACKWARD
    2,  # MOVE_RIGHT
    3,  # MOVE_LEFT
    4,  # TURN_RIGHT
    5,  # TURN_LEFT
    6,  # ATTACK
    7,  # SPEED
    8,  # USE
)

DOOM_LOCK_PATH = '/tmp/doom_impala_lock'


class PyProcessDoom(object):
  """VizDoom wrapper following the IMPALA env protocol."""

  def __init__(self, level, config, num_action_repeats, seed,
               runfiles_path=None, level_cache=None):
    from filelock import FileLock, Timeout
    from ...envs.create_env import create_env
    from ...envs.arguments import default_cfg
    env_name = 'doom_benchmark'
    cfg = default_cfg(env=env_name)
    cfg.pixel_format = 'HWC'
    cfg.res_w = DOOM_W
    cfg.res_h = DOOM_H
    cfg.wide_aspect_ratio = False
    self._env = create_env(env_name, cfg=cfg)
    lock = FileLock(DOOM_LOCK_PATH)
    attempt = 0
    while True:
      attempt += 1
      try:
        with lock.acquire(timeout=10):
          self._env.reset()
          break
      except Timeout:
        print('Another instance holds the doom lock, attempt:', attempt)

  def initial(self):
    obs = self._env.reset()
    return [obs, '']

  def step(self, action):
    obs, rew, done, _ = self._env.step(action)
    done = np.array(done)
    if done:
      obs = self._env.reset()
    return np.array(rew, dtype=np.float32), done, [obs, '']

  def close(self):
    self._env.close()
