"""Screen-resolution selection (reference envs/doom/wrappers/
observation_space.py): must run before the first reset."""

from ...gym_compat import Dict, Error, Wrapper

resolutions = ['160x120', '200x125', '200x150', '256x144', '256x160',
               '256x192', '320x180', '320x200', '320x240', '320x256',
               '400x225', '400x250', '400x300', '512x288', '512x320',
               '512x384', '640x360', '640x400', '640x480', '800x450',
               '800x500', '800x600', '1024x576', '1024x640', '1024x768',
               '1280x720', '1280x800', '1280x960', '1280x1024', '1400x787',
               '1400x875', '1400x1050', '1600x900', '1600x1000', '1600x1200',
               '1920x1080']


class SetResolutionWrapper(Wrapper):

  def __init__(self, env, target_resolution):
    super().__init__(env)
    if target_resolution not in resolutions:
      raise Error('Error - The specified resolution "%s" is not supported by '
                  'Vizdoom.' % target_resolution)
    orig = self.observation_space
    w, h = (int(p) for p in target_resolution.lower().split('x'))
    u = self.unwrapped
    u.screen_w, u.screen_h = w, h
    u.screen_resolution = getattr(u._backend.ScreenResolution,
                                  'RES_%dX%d' % (w, h))
    u.calc_observation_space()
    if isinstance(orig, Dict):
      new = Dict({k: u.observation_space for k in orig.spaces})
    else:
      new = u.observation_space
    self.observation_space = u.observation_space = new

  def reset(self):
    return self.env.reset()

  def step(self, action):
    return self.env.step(action)
