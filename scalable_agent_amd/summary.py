"""Self-contained TensorBoard event writer (no tensorflow/tensorboard needed).

Writes `events.out.tfevents.<time>.<host>` files: TFRecord framing
(length, masked CRC32C, payload, masked CRC32C) around hand-encoded `Event`
protos carrying `Summary` scalar and histogram values, so the reference's tags
(`learning_rate`, `total_loss`, `action` histogram, `<level>/episode_return`,
`<level>/episode_frames`, `dmlab30/training_no_cap`, `dmlab30/training_cap_100`;
experiment.py:423-425, 644-663) load in a stock TensorBoard.  Every record is
mirrored to `summaries.jsonl` for tooling without protobuf.
"""

import json
import os
import socket
import struct
import threading
import time

import numpy as np

# ------------------------------------------------------------------ crc32c
_CRC_TABLE = []
for _i in range(256):
  _c = _i
  for _ in range(8):
    _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
  _CRC_TABLE.append(_c)


def _crc32c_py(data):
  crc = 0xFFFFFFFF
  for b in data:
    crc = _CRC_TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
  return crc ^ 0xFFFFFFFF


def _native_crc():
  try:
    from .runtime import native
    return getattr(native.load(), 'crc32c', None)
  except Exception:  # pylint: disable=broad-except
    return None


_CRC_NATIVE = _native_crc()


def crc32c(data):
  """CRC-32C; the native slicing-by-8 version when the runtime is built."""
  if _CRC_NATIVE is not None:
    return _CRC_NATIVE(memoryview(bytes(data) if not isinstance(
        data, (bytes, bytearray, memoryview)) else data).cast('B'))
  return _crc32c_py(data)


def masked_crc32c(data):
  crc = crc32c(data)
  return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ------------------------------------------------------------------ protobuf
def _varint(v):
  out = bytearray()
  v &= (1 << 64) - 1
  while True:
    b = v & 0x7F
    v >>= 7
    if v:
      out.append(b | 0x80)
    else:
      out.append(b)
      return bytes(out)


def _key(field, wire):
  return _varint((field << 3) | wire)


def _f_double(field, v):
  return _key(field, 1) + struct.pack('<d', float(v))


def _f_float(field, v):
  return _key(field, 5) + struct.pack('<f', float(v))


def _f_int(field, v):
  return _key(field, 0) + _varint(int(v))


def _f_bytes(field, b):
  return _key(field, 2) + _varint(len(b)) + b


def _f_packed_doubles(field, vals):
  payload = b''.join(struct.pack('<d', float(v)) for v in vals)
  return _f_bytes(field, payload)


def _histogram_proto(values, bins=30):
  values = np.asarray(values, dtype=np.float64).reshape(-1)
  if values.size == 0:
    values = np.zeros(1)
  counts, edges = np.histogram(values, bins=bins)
  return (_f_double(1, values.min()) + _f_double(2, values.max()) +
          _f_double(3, values.size) + _f_double(4, values.sum()) +
          _f_double(5, np.square(values).sum()) +
          _f_packed_doubles(6, edges[1:]) + _f_packed_doubles(7, counts))


def _event(wall_time, step, summary=None, file_version=None):
  b = _f_double(1, wall_time) + _f_int(2, step)
  if file_version is not None:
    b += _f_bytes(3, file_version.encode())
  if summary is not None:
    b += _f_bytes(5, summary)
  return b


class SummaryWriter(object):
  """Thread-safe scalar/histogram writer (tf.summary.FileWriter analogue)."""

  def __init__(self, logdir, filename_suffix=''):
    os.makedirs(logdir, exist_ok=True)
    self.logdir = logdir
    fname = 'events.out.tfevents.%010d.%s%s' % (int(time.time()),
                                                 socket.gethostname(),
                                                 filename_suffix)
    self.path = os.path.join(logdir, fname)
    self._f = open(self.path, 'ab')
    self._jsonl = open(os.path.join(logdir, 'summaries.jsonl'), 'a')
    self._lock = threading.Lock()
    self._write_record(_event(time.time(), 0, file_version='brain.Event:2'))

  def _write_record(self, data):
    header = struct.pack('<Q', len(data))
    rec = (header + struct.pack('<I', masked_crc32c(header)) + data +
           struct.pack('<I', masked_crc32c(data)))
    self._f.write(rec)

  def add_scalars(self, values, step):
    """values: dict tag -> float."""
    summ = b''
    for tag, v in values.items():
      summ += _f_bytes(1, _f_bytes(1, str(tag).encode()) + _f_float(2, v))
    with self._lock:
      self._write_record(_event(time.time(), step, summary=summ))
      self._jsonl.write(json.dumps({'step': int(step), 'time': time.time(),
                                    **{k: float(v) for k, v in values.items()}})
                        + '\n')

  def add_scalar(self, tag, value, step):
    self.add_scalars({tag: value}, step)

  def add_histogram(self, tag, values, step, bins=30):
    value = _f_bytes(1, str(tag).encode()) + _f_bytes(5, _histogram_proto(
        values, bins))
    with self._lock:
      self._write_record(_event(time.time(), step, summary=_f_bytes(1, value)))

  def flush(self):
    with self._lock:
      self._f.flush()
      self._jsonl.flush()

  def close(self):
    self.flush()
    self._f.close()
    self._jsonl.close()


def read_events(path):
  """Parses an event file written by SummaryWriter -> list of (step, {tag: v}).

  Minimal decoder used by the tests (scalars only), validating both CRCs.
  """
  out = []
  with open(path, 'rb') as f:
    data = f.read()
  pos = 0
  while pos < len(data):
    (n,) = struct.unpack_from('<Q', data, pos)
    (hcrc,) = struct.unpack_from('<I', data, pos + 8)
    assert hcrc == masked_crc32c(data[pos:pos + 8]), 'header crc'
    payload = data[pos + 12:pos + 12 + n]
    (pcrc,) = struct.unpack_from('<I', data, pos + 12 + n)
    assert pcrc == masked_crc32c(payload), 'payload crc'
    pos += 16 + n
    out.append(_decode_event(payload))
  return out


def _read_varint(b, i):
  shift = v = 0
  while True:
    c = b[i]
    i += 1
    v |= (c & 0x7F) << shift
    shift += 7
    if not c & 0x80:
      return v, i


def _fields(b):
  i = 0
  while i < len(b):
    key, i = _read_varint(b, i)
    field, wire = key >> 3, key & 7
    if wire == 0:
      v, i = _read_varint(b, i)
    elif wire == 1:
      v = struct.unpack_from('<d', b, i)[0]
      i += 8
    elif wire == 5:
      v = struct.unpack_from('<f', b, i)[0]
      i += 4
    elif wire == 2:
      n, i = _read_varint(b, i)
      v = b[i:i + n]
      i += n
    else:
      raise ValueError('wire type %d' % wire)
    yield field, v


def _decode_event(b):
  step = 0
  scalars = {}
  for field, v in _fields(b):
    if field == 2:
      step = v
    elif field == 5:
      for f2, val in _fields(v):
        if f2 == 1:
          tag, simple = None, None
          for f3, x in _fields(val):
            if f3 == 1:
              tag = x.decode()
            elif f3 == 2:
              simple = x
          if tag is not None and simple is not None:
            scalars[tag] = simple
  return step, scalars
