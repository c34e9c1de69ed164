"""Episode GIF encoding (reference utils/gifs.py uses an ffmpeg pipe).

ffmpeg may be absent: falls back to writing the raw frames as .npy."""

import os
import shutil
import subprocess

import numpy as np


def encode_gif(frames, fps=30, path=None):
  frames = np.asarray(frames, np.uint8)
  h, w, c = frames[0].shape
  if shutil.which('ffmpeg') is None:
    if path:
      np.save(os.path.splitext(path)[0] + '.npy', frames)
    return None
  pxfmt = {1: 'gray', 3: 'rgb24'}[c]
  cmd = ['ffmpeg', '-y', '-f', 'rawvideo', '-vcodec', 'rawvideo', '-r',
         '%.02f' % fps, '-s', '%dx%d' % (w, h), '-pix_fmt', pxfmt, '-i', '-',
         '-filter_complex', '[0:v]split[x][z];[z]palettegen[y];[x][y]paletteuse',
         '-r', '%.02f' % fps, '-f', 'gif', '-']
  proc = subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                          stderr=subprocess.PIPE)
  out, err = proc.communicate(frames.tobytes())
  if proc.returncode:
    raise IOError(err.decode('utf8'))
  if path:
    with open(path, 'wb') as f:
      f.write(out)
  return out
