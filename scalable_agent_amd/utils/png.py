"""Dependency-free PNG encoder/decoder for uint8 frames (episode recording;
the reference uses cv2.imwrite, envs/env_wrappers.py:472-476)."""

import struct
import zlib

import numpy as np


def _chunk(tag, data):
  body = tag + data
  return struct.pack('>I', len(data)) + body + struct.pack(
      '>I', zlib.crc32(body) & 0xffffffff)


def encode_png(img, level=6):
  """img: [H,W] gray or [H,W,3|4] uint8 -> PNG bytes."""
  img = np.ascontiguousarray(img, dtype=np.uint8)
  if img.ndim == 2:
    img = img[:, :, None]
  h, w, c = img.shape
  color_type = {1: 0, 3: 2, 4: 6}[c]
  raw = np.concatenate([np.zeros((h, 1), np.uint8), img.reshape(h, w * c)],
                       axis=1)  # filter byte 0 (None) per row
  header = struct.pack('>IIBBBBB', w, h, 8, color_type, 0, 0, 0)
  return (b'\x89PNG\r\n\x1a\n' + _chunk(b'IHDR', header) +
          _chunk(b'IDAT', zlib.compress(raw.tobytes(), level)) +
          _chunk(b'IEND', b''))


def write_png(path, img, level=6):
  with open(path, 'wb') as f:
    f.write(encode_png(img, level))


def decode_png(data):
  """Decodes PNGs written by `encode_png` (8-bit, filter 0 rows only)."""
  assert data[:8] == b'\x89PNG\r\n\x1a\n', 'not a PNG'
  pos, idat, hdr = 8, b'', None
  while pos < len(data):
    (n,) = struct.unpack('>I', data[pos:pos + 4])
    tag = data[pos + 4:pos + 8]
    body = data[pos + 8:pos + 8 + n]
    if tag == b'IHDR':
      hdr = struct.unpack('>IIBBBBB', body)
    elif tag == b'IDAT':
      idat += body
    pos += 12 + n
  w, h, _, color_type = hdr[:4]
  c = {0: 1, 2: 3, 6: 4}[color_type]
  raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, w * c + 1)
  if np.any(raw[:, 0] != 0):
    raise ValueError('only filter type 0 is supported')
  img = raw[:, 1:].reshape(h, w, c)
  return img[:, :, 0] if c == 1 else img
