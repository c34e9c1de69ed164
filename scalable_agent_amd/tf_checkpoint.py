"""TensorFlow checkpoint import/export without TensorFlow (SURVEY.md §5.4,
§7.4 "Variable naming").

The reference trains under `tf.train.MonitoredTrainingSession`, whose Saver
writes V2 checkpoints: `model.ckpt-<frames>.index` (a LevelDB-format table
mapping variable names to BundleEntryProto records) plus
`model.ckpt-<frames>.data-00000-of-00001` (raw little-endian tensor bytes),
and a `checkpoint` text file naming the latest prefix (experiment.py:608-616).
This module reads and writes that format directly:

  * SSTable: prefix-compressed data blocks with restart arrays, an index
    block of BlockHandles, a 48-byte footer with the table magic, and a
    5-byte trailer (compression type + masked crc32c) after every block;
  * BundleHeaderProto under the empty key, BundleEntryProto per variable
    (dtype, shape, shard, offset, size, masked crc32c of the bytes), decoded
    with a minimal protobuf wire-format parser.

`import_tf_checkpoint` loads the agent weights (reference variable names,
`Agent.tf_variable_names`), the RMSProp slots (`<var>/RMSProp` = ms,
`<var>/RMSProp_1` = mom) and `num_environment_frames` into a Learner;
`export_tf_checkpoint` writes the same layout from one.  No TensorFlow is
installed here, so compatibility with TF-written files is pinned only by the
format description above (parity unpinned); the round trip is tested.
"""

import glob
import os
import re
import struct

import numpy as np

from .summary import crc32c, masked_crc32c

_MAGIC = 0xdb4775248b80fb57
# DataType enum (tensorflow/core/framework/types.proto) <-> numpy
_DT = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16,
       6: np.int8, 9: np.int64, 10: np.bool_, 19: np.float16}
_DT_OF = {np.dtype(v): k for k, v in _DT.items()}


# ----------------------------------------------------------------- varints
def _varint(buf, pos):
  shift = result = 0
  while True:
    b = buf[pos]
    pos += 1
    result |= (b & 0x7F) << shift
    if not b & 0x80:
      return result, pos
    shift += 7


def _put_varint(v):
  out = bytearray()
  while True:
    b = v & 0x7F
    v >>= 7
    if v:
      out.append(b | 0x80)
    else:
      out.append(b)
      return bytes(out)


def _unmask(m):
  rot = (m - 0xa282ead8) & 0xFFFFFFFF
  return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ---------------------------------------------------------------- protobuf
def _fields(buf):
  """Yields (field_number, wire_type, value) of a serialized message."""
  pos = 0
  while pos < len(buf):
    key, pos = _varint(buf, pos)
    num, wt = key >> 3, key & 7
    if wt == 0:
      v, pos = _varint(buf, pos)
    elif wt == 1:
      v = struct.unpack_from('<Q', buf, pos)[0]
      pos += 8
    elif wt == 2:
      n, pos = _varint(buf, pos)
      v = bytes(buf[pos:pos + n])
      pos += n
    elif wt == 5:
      v = struct.unpack_from('<I', buf, pos)[0]
      pos += 4
    else:
      raise ValueError('unsupported protobuf wire type %d' % wt)
    yield num, wt, v


def _parse_entry(buf):
  e = {'dtype': 1, 'shape': [], 'shard_id': 0, 'offset': 0, 'size': 0,
       'crc32c': None, 'slices': False}
  for num, _, v in _fields(buf):
    if num == 1:
      e['dtype'] = v
    elif num == 2:
      for dn, _, dv in _fields(v):
        if dn == 2:  # Dim
          size = 0
          for sn, _, sv in _fields(dv):
            if sn == 1:
              size = sv
          e['shape'].append(size)
    elif num == 3:
      e['shard_id'] = v
    elif num == 4:
      e['offset'] = v
    elif num == 5:
      e['size'] = v
    elif num == 6:
      e['crc32c'] = v
    elif num == 7:
      e['slices'] = True
  return e


def _field_varint(num, v):
  return _put_varint(num << 3) + _put_varint(v)


def _field_bytes(num, b):
  return _put_varint((num << 3) | 2) + _put_varint(len(b)) + b


def _entry_bytes(dtype, shape, offset, size, crc):
  dims = b''.join(_field_bytes(2, _field_varint(1, d)) for d in shape)
  out = _field_varint(1, dtype) + _field_bytes(2, dims)
  out += _field_varint(4, offset) if offset else b''
  out += _field_varint(5, size)
  out += _put_varint((6 << 3) | 5) + struct.pack('<I', crc)
  return out


def _header_bytes(num_shards=1):
  # num_shards, endianness LITTLE (0, default), version {producer: 1}
  return _field_varint(1, num_shards) + _field_bytes(3, _field_varint(1, 1))


# ------------------------------------------------------------------ sstable
def _read_block(data, offset, size):
  block = data[offset:offset + size]
  ctype = data[offset + size]
  if ctype != 0:
    raise ValueError('compressed checkpoint index blocks are not supported')
  want = struct.unpack_from('<I', data, offset + size + 1)[0]
  if masked_crc32c(bytes(block) + bytes([ctype])) != want:
    raise ValueError('checkpoint index block checksum mismatch')
  return block


def _block_entries(block):
  n_restarts = struct.unpack_from('<I', block, len(block) - 4)[0]
  end = len(block) - 4 - 4 * n_restarts
  pos, key = 0, b''
  while pos < end:
    shared, pos = _varint(block, pos)
    non_shared, pos = _varint(block, pos)
    vlen, pos = _varint(block, pos)
    key = key[:shared] + bytes(block[pos:pos + non_shared])
    pos += non_shared
    yield key, bytes(block[pos:pos + vlen])
    pos += vlen


def _read_table(data):
  if len(data) < 48:
    raise ValueError('not a checkpoint index (too short)')
  footer = data[-48:]
  if struct.unpack_from('<Q', footer, 40)[0] != _MAGIC:
    raise ValueError('not a checkpoint index (bad table magic)')
  pos = 0
  _, pos = _varint(footer, pos)   # metaindex offset
  _, pos = _varint(footer, pos)   # metaindex size
  ioff, pos = _varint(footer, pos)
  isize, pos = _varint(footer, pos)
  out = {}
  for _, handle in _block_entries(_read_block(data, ioff, isize)):
    boff, p = _varint(handle, 0)
    bsize, _ = _varint(handle, p)
    for k, v in _block_entries(_read_block(data, boff, bsize)):
      out[k] = v
  return out


def _block_bytes(items, restart_interval=16):
  out, restarts, prev = bytearray(), [], b''
  for i, (k, v) in enumerate(items):
    if i % restart_interval == 0:
      restarts.append(len(out))
      shared = 0
    else:
      shared = 0
      while (shared < min(len(prev), len(k)) and prev[shared] == k[shared]):
        shared += 1
    out += _put_varint(shared) + _put_varint(len(k) - shared) + \
        _put_varint(len(v)) + k[shared:] + v
    prev = k
  if not restarts:
    restarts = [0]
  for r in restarts:
    out += struct.pack('<I', r)
  out += struct.pack('<I', len(restarts))
  return bytes(out)


def _write_table(items, block_entries=64):
  """items: sorted (key, value) pairs -> table bytes."""
  out = bytearray()
  index = []

  def put_block(b):
    off = len(out)
    out.extend(b)
    out.append(0)
    out.extend(struct.pack('<I', masked_crc32c(b + b'\x00')))
    return off, len(b)

  for i in range(0, len(items), block_entries):
    chunk = items[i:i + block_entries]
    off, size = put_block(_block_bytes(chunk))
    index.append((chunk[-1][0], _put_varint(off) + _put_varint(size)))
  meta_off, meta_size = put_block(_block_bytes([]))
  idx_off, idx_size = put_block(_block_bytes(index, restart_interval=1))
  footer = (_put_varint(meta_off) + _put_varint(meta_size) +
            _put_varint(idx_off) + _put_varint(idx_size))
  footer += b'\x00' * (40 - len(footer)) + struct.pack('<Q', _MAGIC)
  out.extend(footer)
  return bytes(out)


# ------------------------------------------------------------------ bundles
def read_checkpoint(prefix):
  """-> {variable name: numpy array} of a V2 checkpoint `prefix`."""
  with open(prefix + '.index', 'rb') as f:
    table = _read_table(memoryview(f.read()))
  header = table.pop(b'', None)
  num_shards = 1
  if header is not None:
    for num, _, v in _fields(header):
      if num == 1:
        num_shards = v
  shards = {}
  out = {}
  for key, val in sorted(table.items()):
    e = _parse_entry(val)
    if e['slices']:
      raise ValueError('partitioned variable %s is not supported' % key)
    dt = _DT.get(e['dtype'])
    if dt is None:
      raise ValueError('unsupported dtype %d for %s' % (e['dtype'], key))
    sid = e['shard_id']
    if sid not in shards:
      path = '%s.data-%05d-of-%05d' % (prefix, sid, num_shards)
      shards[sid] = np.memmap(path, dtype=np.uint8, mode='r')
    raw = bytes(shards[sid][e['offset']:e['offset'] + e['size']])
    if e['crc32c'] is not None and _unmask(e['crc32c']) != crc32c(raw):
      raise ValueError('checksum mismatch for %s' % key)
    out[key.decode('utf-8')] = np.frombuffer(raw, dtype=dt).reshape(
        e['shape']).copy()
  return out


def write_checkpoint(prefix, tensors):
  """Writes {name: array} as a single-shard V2 checkpoint at `prefix`."""
  os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
  items, data = [(b'', _header_bytes())], bytearray()
  for name in sorted(tensors):
    a = np.require(np.asarray(tensors[name]), requirements="C")
    dt = _DT_OF.get(a.dtype)
    if dt is None:
      raise ValueError('unsupported dtype %s for %s' % (a.dtype, name))
    raw = a.astype(a.dtype.newbyteorder('<'), copy=False).tobytes()
    items.append((name.encode('utf-8'),
                  _entry_bytes(dt, list(a.shape), len(data), len(raw),
                               masked_crc32c(raw))))
    data.extend(raw)
  items.sort(key=lambda kv: kv[0])
  with open(prefix + '.data-00000-of-00001', 'wb') as f:
    f.write(bytes(data))
  with open(prefix + '.index', 'wb') as f:
    f.write(_write_table(items))


def latest_checkpoint(logdir):
  """The prefix named by `logdir/checkpoint` (model_checkpoint_path)."""
  path = os.path.join(logdir, 'checkpoint')
  if not os.path.exists(path):
    return None
  m = re.search(r'^model_checkpoint_path:\s*"([^"]+)"', open(path).read(),
                re.M)
  if not m:
    return None
  p = m.group(1)
  return p if os.path.isabs(p) else os.path.join(logdir, p)


# ------------------------------------------------------------ agent mapping
def import_tf_checkpoint(prefix_or_logdir, learner=None, agent=None):
  """Loads reference-named variables into `learner` (weights, RMSProp ms /
  mom slots, frame counter) or just `agent`.  Returns the frame count (or
  None when the checkpoint has no `num_environment_frames`)."""
  import torch
  prefix = prefix_or_logdir
  if os.path.isdir(prefix):
    prefix = latest_checkpoint(prefix)
    if prefix is None:
      raise FileNotFoundError('no checkpoint file in %s' % prefix_or_logdir)
  t = read_checkpoint(prefix)
  agent = agent if agent is not None else learner.agent
  names = agent.tf_variable_names()
  missing = [names[n] for n, _ in agent.named_parameters()
             if names[n] not in t]
  if missing:
    raise KeyError('checkpoint %s lacks %s' % (prefix, missing[:5]))
  with torch.no_grad():
    for n, p in agent.named_parameters():
      src = torch.from_numpy(t[names[n]]).to(p.dtype)
      if tuple(src.shape) != tuple(p.shape):
        raise ValueError('%s: checkpoint shape %s != %s' % (
            names[n], tuple(src.shape), tuple(p.shape)))
      p.copy_(src.to(p.device))
  if learner is None:
    return None
  flat = learner.flat
  with torch.no_grad():
    for n, p in flat.named:
      for slot, buf in (('RMSProp', learner.opt.ms),
                        ('RMSProp_1', learner.opt.mom)):
        key = names[n] + '/' + slot
        if key in t:
          v = flat.view_of(buf, n)
          v.copy_(torch.from_numpy(t[key]).to(v.dtype).view_as(v).to(v.device))
  frames = None
  if 'num_environment_frames' in t:
    frames = int(np.asarray(t['num_environment_frames']).reshape(()))
    learner.frames.fill_(frames)
  return frames


def list_tf_checkpoints(logdir):
  """[(frames, prefix)] of the complete model.ckpt-N in logdir, oldest first."""
  out = []
  for idx in glob.glob(os.path.join(logdir, 'model.ckpt-*.index')):
    m = re.search(r'model\.ckpt-(\d+)\.index$', idx)
    prefix = idx[:-len('.index')]
    if m and os.path.exists(prefix + '.data-00000-of-00001'):
      out.append((int(m.group(1)), prefix))
  return sorted(out)


def export_tf_checkpoint(logdir, learner, keep=None, extra=None):
  """Writes `logdir/model.ckpt-<frames>` (+ `checkpoint`) in the reference's
  variable layout (weights, RMSProp `ms`/`mom` slots as `<var>/RMSProp` and
  `<var>/RMSProp_1`, `num_environment_frames`; reference experiment.py:
  608-616); `extra` {name: array} adds further tensors (PopArt statistics).
  The shards are written under temporary names and renamed (data, then
  index), then the `checkpoint` file is replaced atomically; with `keep`,
  older model.ckpt-N beyond the newest `keep` are removed.  Returns the
  prefix."""
  frames = int(learner.frames.item())
  names = learner.agent.tf_variable_names()
  t = {}
  for n, p in learner.flat.named:
    t[names[n]] = p.detach().float().cpu().numpy()
    t[names[n] + '/RMSProp'] = learner.flat.view_of(
        learner.opt.ms, n).detach().float().cpu().numpy()
    t[names[n] + '/RMSProp_1'] = learner.flat.view_of(
        learner.opt.mom, n).detach().float().cpu().numpy()
  t['num_environment_frames'] = np.asarray(frames, np.int64)
  for k, v in (extra or {}).items():
    t[k] = np.asarray(v)
  name = 'model.ckpt-%d' % frames
  prefix = os.path.join(logdir, name)
  tmp = os.path.join(logdir, '.tmp-' + name)
  write_checkpoint(tmp, t)
  for suffix in ('.data-00000-of-00001', '.index'):
    with open(tmp + suffix, 'rb') as f:
      os.fsync(f.fileno())
    os.replace(tmp + suffix, prefix + suffix)
  ckpts = list_tf_checkpoints(logdir)
  if keep:
    for _, old in ckpts[:-keep]:
      for suffix in ('.index', '.data-00000-of-00001'):
        try:
          os.remove(old + suffix)
        except OSError:
          pass
    ckpts = ckpts[-keep:]
  idx_tmp = os.path.join(logdir, 'checkpoint.tmp')
  with open(idx_tmp, 'w') as f:
    f.write('model_checkpoint_path: "%s"\n' % name)
    for _, p in ckpts:
      f.write('all_model_checkpoint_paths: "%s"\n' % os.path.basename(p))
  os.replace(idx_tmp, os.path.join(logdir, 'checkpoint'))
  return prefix
