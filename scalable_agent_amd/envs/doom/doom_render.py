"""Frame grids / display helpers for Doom (reference envs/doom/
doom_render.py)."""

import numpy as np

from ..env_wrappers import INTER_LINEAR, resize


def cvt_doom_obs(obs, w=1200, h=675):
  """CHW or HWC frame -> HWC RGB at display size."""
  if obs.shape[0] <= 4:
    obs = np.transpose(obs, (1, 2, 0))
  return resize(np.ascontiguousarray(obs), w, h, INTER_LINEAR)


def concat_grid(obs, max_horizontal=3):
  """Tiles frames into a grid (3 per row, padded with black frames)."""
  obs = [cvt_doom_obs(o) for o in obs]
  horizontal = min(max_horizontal, len(obs))
  while len(obs) % horizontal != 0:
    obs.append(np.zeros_like(obs[0]))
  rows = [np.concatenate(obs[i:i + horizontal], axis=1)
          for i in range(0, len(obs), horizontal)]
  return np.concatenate(rows, axis=0)


def show_image(title, img):
  """Displays an RGB frame when a GUI toolkit is available; otherwise the
  frame is only returned by render() (headless boxes)."""
  try:
    import cv2  # pylint: disable=import-outside-toplevel
  except ImportError:
    return False
  cv2.imshow(title, img[:, :, ::-1])
  cv2.waitKey(1)
  return True
