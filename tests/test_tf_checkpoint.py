"""TF V2 checkpoint bundle reader/writer (scalable_agent_amd/tf_checkpoint.py).

No TensorFlow in this image and no TF checkpoint in the reference tree, so
TF-compatibility is parity unpinned: these tests pin the format pieces that
are fully specified (SSTable blocks/footer/trailers, masked CRC-32C, the
BundleEntryProto wire format) and the learner import/export round trip."""

import os
import struct

import numpy as np
import pytest
import torch

from scalable_agent_amd import flags as flags_lib
from scalable_agent_amd import tf_checkpoint as tfc
from scalable_agent_amd.learner import Learner
from scalable_agent_amd.models import Agent
from scalable_agent_amd.summary import crc32c, masked_crc32c


def test_crc32c_known_vectors():
  assert crc32c(b'123456789') == 0xE3069283
  assert crc32c(b'') == 0
  assert crc32c(bytes(32)) == 0x8A9136AA
  m = masked_crc32c(b'abc')
  assert tfc._unmask(m) == crc32c(b'abc')


def test_roundtrip_many_vars_and_dtypes(tmp_path):
  rng = np.random.RandomState(0)
  t = {'a/w': rng.randn(3, 4).astype(np.float32),
       'a/b': rng.randn(4).astype(np.float64),
       'steps': np.asarray(123456789012, np.int64),
       'mask': rng.rand(5) > 0.5,
       'img': rng.randint(0, 255, (2, 3, 3)).astype(np.uint8)}
  # > 64 entries: several data blocks, prefix-compressed keys, restarts
  for i in range(150):
    t['agent/convnet/res_%03d/conv_2d/w' % i] = rng.randn(2, 2).astype(np.float32)
  prefix = str(tmp_path / 'model.ckpt-7')
  tfc.write_checkpoint(prefix, t)
  got = tfc.read_checkpoint(prefix)
  assert sorted(got) == sorted(t)
  for k in t:
    assert got[k].dtype == np.asarray(t[k]).dtype and got[k].shape == np.shape(t[k])
    np.testing.assert_array_equal(got[k], t[k])
  # footer magic and the first block's trailer checksum
  data = open(prefix + '.index', 'rb').read()
  assert struct.unpack('<Q', data[-8:])[0] == 0xdb4775248b80fb57


def test_corruption_is_detected(tmp_path):
  prefix = str(tmp_path / 'm')
  tfc.write_checkpoint(prefix, {'x': np.arange(10, dtype=np.float32)})
  raw = bytearray(open(prefix + '.data-00000-of-00001', 'rb').read())
  raw[5] ^= 0xFF
  open(prefix + '.data-00000-of-00001', 'wb').write(bytes(raw))
  with pytest.raises(ValueError, match='checksum'):
    tfc.read_checkpoint(prefix)


def test_learner_export_import(tmp_path):
  flags = flags_lib.parse_flags(['--batch_size=2', '--unroll_length=3'])
  torch.manual_seed(0)
  a = Learner(Agent(9, torso='shallow'), flags, 'cpu')
  a.opt.ms.uniform_(1.0, 2.0)
  a.opt.mom.uniform_(-1.0, 1.0)
  a.frames.fill_(4242)
  prefix = tfc.export_tf_checkpoint(str(tmp_path), a)
  assert os.path.basename(prefix) == 'model.ckpt-4242'
  t = tfc.read_checkpoint(prefix)
  assert 'agent/lstm_cell/kernel' in t and 'agent/lstm_cell/kernel/RMSProp_1' in t
  torch.manual_seed(1)
  b = Learner(Agent(9, torso='shallow'), flags, 'cpu')
  frames = tfc.import_tf_checkpoint(str(tmp_path), learner=b)
  assert frames == 4242 and int(b.frames.item()) == 4242
  assert torch.equal(a.flat.params, b.flat.params)
  for (n, _) in a.flat.named:
    assert torch.equal(a.flat.view_of(a.opt.ms, n), b.flat.view_of(b.opt.ms, n))
    assert torch.equal(a.flat.view_of(a.opt.mom, n), b.flat.view_of(b.opt.mom, n))
  with pytest.raises(ValueError, match='shape'):
    tfc.import_tf_checkpoint(prefix, agent=Agent(5, torso='shallow'))


def test_experiment_starts_from_tf_checkpoint(tmp_path):
  """--import_tf_checkpoint: a fresh logdir starts from a reference-layout
  checkpoint (weights + frame counter)."""
  from scalable_agent_amd import checkpoint as ckpt_lib
  from scalable_agent_amd import experiment
  flags = flags_lib.parse_flags(['--batch_size=2', '--unroll_length=3'])
  torch.manual_seed(3)
  src = Learner(Agent(9, torso='shallow', frame_shape=(72, 96, 3)), flags,
                'cpu')
  src.frames.fill_(1200)
  tf_dir = tmp_path / 'tf'
  os.makedirs(tf_dir)
  tfc.export_tf_checkpoint(str(tf_dir), src)
  logdir = tmp_path / 'run'
  argv = ['--level_name=synthetic', '--num_actors=1', '--batch_size=1',
          '--unroll_length=4', '--max_learner_steps=1', '--device=cpu',
          '--logdir=%s' % logdir, '--import_tf_checkpoint=%s' % tf_dir,
          '--total_environment_frames=100000000']
  experiment.main(argv)
  state = ckpt_lib.load_state(ckpt_lib.latest_checkpoint(str(logdir)))
  assert state['num_environment_frames'] == 1200 + 4 * 1 * 4
