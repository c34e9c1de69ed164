"""GPU -> NUMA node affinity from sysfs (parallel/affinity.py), against a
fake sysfs tree: KFD topology GPU nodes in HIP order, PCI numa_node, node
cpulists, *_VISIBLE_DEVICES renumbering; the real pin is applied only when
the node's CPUs overlap this process's affinity."""

import os

from scalable_agent_amd.parallel import affinity


def _fake_sysfs(root, gpus):
  """gpus: list of (bus, numa_node); node0 = cpus 0-3, node1 = cpus 4-7."""
  topo = root / 'class/kfd/kfd/topology/nodes'
  (topo / '0').mkdir(parents=True)
  (topo / '0' / 'properties').write_text('simd_count 0\nlocation_id 0\n')
  for i, (bus, node) in enumerate(gpus):
    d = topo / str(i + 1)
    d.mkdir()
    d.joinpath('properties').write_text(
        'cpu_cores_count 0\nsimd_count 1024\nlocation_id %d\ndomain 0\n' %
        (bus << 8))
    pci = root / 'bus/pci/devices' / ('0000:%02x:00.0' % bus)
    pci.mkdir(parents=True)
    pci.joinpath('numa_node').write_text('%d\n' % node)
  for n, cl in ((0, '0-3'), (1, '4-7')):
    nd = root / ('devices/system/node/node%d' % n)
    nd.mkdir(parents=True)
    nd.joinpath('cpulist').write_text(cl + '\n')


def test_mapping(tmp_path):
  _fake_sysfs(tmp_path, [(0x05, 0), (0x15, 0), (0x85, 1), (0x95, 1)])
  root = str(tmp_path)
  assert affinity.gpu_pci_addresses(root)[2] == '0000:85:00.0'
  assert [affinity.gpu_numa_node(i, root, env={}) for i in range(4)] == [0, 0, 1, 1]
  # HIP_VISIBLE_DEVICES=3,0: logical 0 is physical 3
  env = {'HIP_VISIBLE_DEVICES': '3,0'}
  assert affinity.gpu_numa_node(0, root, env) == 1
  assert affinity.gpu_numa_node(1, root, env) == 0
  assert affinity.gpu_numa_node(7, root, env={}) is None
  node, cpus = affinity.pin_to_gpu_numa(2, root, env={}, apply=False)
  assert node == 1 and cpus == [4, 5, 6, 7]
  assert affinity.parse_cpulist('0-2,5,8-9') == {0, 1, 2, 5, 8, 9}


def test_pin_is_a_noop_without_topology(tmp_path):
  before = os.sched_getaffinity(0)
  assert affinity.pin_to_gpu_numa(0, str(tmp_path)) is None
  assert os.sched_getaffinity(0) == before


def test_pin_applies_in_process(tmp_path):
  import multiprocessing as mp
  _fake_sysfs(tmp_path, [(0x05, 0), (0x85, 1)])
  ctx = mp.get_context('fork')
  q = ctx.Queue()

  def child():
    r = affinity.pin_to_gpu_numa(0, str(tmp_path), env={})
    q.put((r, sorted(os.sched_getaffinity(0))))

  p = ctx.Process(target=child)
  p.start()
  p.join(30)
  r, aff = q.get(timeout=5)
  avail = sorted(os.sched_getaffinity(0) & {0, 1, 2, 3})
  if avail and avail != sorted(os.sched_getaffinity(0)):
    assert r[0] == 0 and aff == avail


def test_visible_masks_like_the_runtime():
  # HIP honours HIP_VISIBLE_DEVICES OR CUDA_VISIBLE_DEVICES (HIP first), not
  # both; ROCR_VISIBLE_DEVICES maps the HIP-level index to a physical one
  vi = affinity.visible_index
  assert vi(0, {'HIP_VISIBLE_DEVICES': '1,0', 'CUDA_VISIBLE_DEVICES': '1,0'}) == 1
  assert vi(1, {'HIP_VISIBLE_DEVICES': '1,0', 'CUDA_VISIBLE_DEVICES': '1,0'}) == 0
  assert vi(0, {'CUDA_VISIBLE_DEVICES': '2,3'}) == 2
  assert vi(0, {'HIP_VISIBLE_DEVICES': '1', 'ROCR_VISIBLE_DEVICES': '4,6'}) == 6
  assert vi(1, {'ROCR_VISIBLE_DEVICES': '4,6'}) == 6
  assert vi(3, {}) == 3


def test_auto_pin_only_when_ranks_cover_every_socket(tmp_path):
  _fake_sysfs(tmp_path, [(0x05, 0), (0x85, 1)])
  root = str(tmp_path)
  assert affinity.numa_node_count(root) == 2
  assert not affinity.auto_pin_wanted(1, root)   # lone rank: actors keep both sockets
  assert affinity.auto_pin_wanted(2, root)
  assert affinity.auto_pin_wanted(8, root)
  assert affinity.numa_node_count(str(tmp_path / 'missing')) == 1
  assert not affinity.auto_pin_wanted(8, str(tmp_path / 'missing'))


def test_auto_pin_needs_the_gpus_on_every_socket(tmp_path):
  # two ranks whose GPUs both hang off socket 0: pinning would idle socket 1
  _fake_sysfs(tmp_path, [(0x05, 0), (0x15, 0), (0x85, 1)])
  root = str(tmp_path)
  assert not affinity.auto_pin_wanted(2, root, env={})
  assert affinity.auto_pin_wanted(3, root, env={})
  # the visible mask decides which physical GPUs the ranks get
  assert affinity.auto_pin_wanted(2, root, env={'HIP_VISIBLE_DEVICES': '0,2'})


def test_visible_gpu_count(tmp_path):
  _fake_sysfs(tmp_path, [(0x05, 0), (0x15, 0), (0x85, 1), (0x95, 1)])
  root = str(tmp_path)
  assert affinity.visible_gpu_count(root, env={}) == 4
  assert affinity.visible_gpu_count(root, env={'HIP_VISIBLE_DEVICES': '1,3'}) == 2
  assert affinity.visible_gpu_count(root, env={'ROCR_VISIBLE_DEVICES': '2'}) == 1
  assert affinity.visible_gpu_count(root, env={'CUDA_VISIBLE_DEVICES': '0,7'}) == 1
  assert affinity.visible_gpu_count(str(tmp_path / 'missing'), env={}) is None
  # a UUID mask is not counted here (unknown): the caller defers to HIP
  assert affinity.visible_gpu_count(
      root, env={'ROCR_VISIBLE_DEVICES': 'GPU-1f2e3d4c5b6a7988'}) is None
  assert affinity.visible_gpu_count(
      root, env={'HIP_VISIBLE_DEVICES': '0,GPU-1f2e3d4c5b6a7988'}) is None
