"""CPU/NUMA affinity of a learner rank to its GPU's NUMA node.

On a 2-socket 8 x MI355X node each GPU hangs off one socket.  A rank whose
learner thread, H2D feeder and pinned trajectory slabs live on the other
socket pays a cross-socket hop on every ~67 MB/step batch copy and on every
kernel launch.  `pin_to_gpu_numa` restricts the calling process (and every
process it forks afterwards: actor groups, env workers) to the CPUs of the
NUMA node of the rank's GPU (under `--numa_affinity auto` only when the
node's ranks cover every socket, `auto_pin_wanted`), in process and without
re-executing anything, so it must run BEFORE the first pinned allocation and before the actor
processes are forked (the slabs' pages are first-touched by those
processes).

The GPU -> NUMA node mapping is read from sysfs only (no HIP call, so it can
run before the GPU is initialised): the KFD topology lists GPU nodes in HIP
enumeration order with their PCI location; /sys/bus/pci/devices/<bdf>/
numa_node gives the node and /sys/devices/system/node/node<N>/cpulist its
CPUs.  HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES
renumber the devices like the runtime does.  Every failure is a no-op.
"""

import logging
import os

log = logging.getLogger('scalable_agent_amd')


def _read(path):
  try:
    with open(path) as f:
      return f.read()
  except OSError:
    return None


def parse_cpulist(text):
  """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11}."""
  out = set()
  for part in (text or '').strip().split(','):
    if not part:
      continue
    if '-' in part:
      a, b = part.split('-')
      out.update(range(int(a), int(b) + 1))
    else:
      out.add(int(part))
  return out


def gpu_pci_addresses(root='/sys'):
  """PCI addresses ('0000:05:00.0') of the GPUs in HIP enumeration order
  (KFD topology GPU nodes, i.e. nodes with SIMDs)."""
  base = os.path.join(root, 'class/kfd/kfd/topology/nodes')
  try:
    nodes = sorted(os.listdir(base), key=int)
  except (OSError, ValueError):
    return []
  out = []
  for n in nodes:
    props = _read(os.path.join(base, n, 'properties')) or ''
    kv = {}
    for line in props.splitlines():
      parts = line.split()
      if len(parts) == 2:
        kv[parts[0]] = parts[1]
    if int(kv.get('simd_count', '0')) <= 0:
      continue  # a CPU node
    loc = int(kv.get('location_id', '0'))
    dom = int(kv.get('domain', '0'))
    bus, dev, fn = (loc >> 8) & 0xff, (loc >> 3) & 0x1f, loc & 0x7
    out.append('%04x:%02x:%02x.%x' % (dom, bus, dev, fn))
  return out


def visible_index(local_rank, env=None):
  """Physical GPU index of logical device `local_rank` under the
  *_VISIBLE_DEVICES masks, applied like the runtime does: the HIP-level
  mask (HIP_VISIBLE_DEVICES, or CUDA_VISIBLE_DEVICES when HIP's is unset -
  HIP honours only one of them) indexes the devices ROCr exposes, and
  ROCR_VISIBLE_DEVICES (applied first, at the ROCr level) maps those to
  physical devices."""
  env = os.environ if env is None else env

  def ids(var):
    spec = env.get(var)
    if not spec:
      return None
    return [int(x) for x in spec.split(',') if x.strip().isdigit()]

  idx = local_rank
  hip = ids('HIP_VISIBLE_DEVICES')
  if hip is None:
    hip = ids('CUDA_VISIBLE_DEVICES')
  if hip is not None and idx < len(hip):
    idx = hip[idx]
  rocr = ids('ROCR_VISIBLE_DEVICES')
  if rocr is not None and idx < len(rocr):
    idx = rocr[idx]
  return idx


def cpu_numa_nodes(root='/sys'):
  """Ids of the NUMA nodes that have CPUs (empty when unknown)."""
  base = os.path.join(root, 'devices/system/node')
  try:
    names = [n for n in os.listdir(base)
             if n.startswith('node') and n[4:].isdigit()]
  except OSError:
    return set()
  return {int(name[4:]) for name in names
          if parse_cpulist(_read(os.path.join(base, name, 'cpulist')))}


def numa_node_count(root='/sys'):
  """Number of NUMA nodes with CPUs (1 when unknown)."""
  return max(1, len(cpu_numa_nodes(root)))


def visible_gpu_count(root='/sys', env=None):
  """GPUs this process may use, from sysfs and the *_VISIBLE_DEVICES masks
  only (no HIP call); None when the KFD topology is unreadable."""
  env = os.environ if env is None else env
  phys = len(gpu_pci_addresses(root))
  if phys == 0 and not os.path.isdir(os.path.join(
      root, 'class/kfd/kfd/topology/nodes')):
    return None
  n = phys
  for var in ('ROCR_VISIBLE_DEVICES',
              'HIP_VISIBLE_DEVICES' if env.get('HIP_VISIBLE_DEVICES')
              else 'CUDA_VISIBLE_DEVICES'):
    spec = env.get(var)
    if spec is None:
      continue
    toks = [x.strip() for x in spec.split(',') if x.strip()]
    if not all(x.isdigit() for x in toks):
      # a UUID mask (GPU-<uuid>) or anything else that is not plain
      # ordinals: unknown here, the caller defers to the HIP device count
      return None
    ids = [int(x) for x in toks]
    n = len([i for i in ids if i < n])
  return n


def auto_pin_wanted(local_world, root='/sys', env=None):
  """'auto' NUMA pinning policy: pin a rank (and the actor / env processes
  it forks, which inherit the mask) to its GPU's node only when the GPUs of
  the node's ranks together sit on every NUMA node that has CPUs.  A single
  rank on a 2-socket box, or two ranks whose GPUs both hang off socket 0,
  would otherwise confine every CPU-bound actor to half of the machine."""
  cpu_nodes = cpu_numa_nodes(root)
  if len(cpu_nodes) <= 1:
    return False
  gpu_nodes = {gpu_numa_node(r, root, env) for r in range(local_world)}
  return cpu_nodes <= gpu_nodes


def gpu_numa_node(local_rank, root='/sys', env=None):
  """NUMA node of logical GPU `local_rank`, or None when unknown."""
  addrs = gpu_pci_addresses(root)
  phys = visible_index(local_rank, env)
  if phys >= len(addrs):
    return None
  txt = _read(os.path.join(root, 'bus/pci/devices', addrs[phys], 'numa_node'))
  try:
    node = int(txt)
  except (TypeError, ValueError):
    return None
  return node if node >= 0 else None


def pin_to_gpu_numa(local_rank, root='/sys', env=None, apply=True):
  """Restricts this process's CPU affinity to its GPU's NUMA node.

  -> (node, sorted cpu list) when applied, None otherwise (unknown node,
  single-node machine, or no overlap with the current affinity)."""
  node = gpu_numa_node(local_rank, root, env)
  if node is None:
    return None
  cpus = parse_cpulist(_read(os.path.join(
      root, 'devices/system/node/node%d/cpulist' % node)))
  try:
    current = os.sched_getaffinity(0)
  except AttributeError:
    return None
  target = cpus & current if apply else cpus
  if not target or (apply and target == current):
    return None
  if apply:
    try:
      os.sched_setaffinity(0, target)
    except OSError as e:
      log.warning('NUMA pinning to node %d failed: %s', node, e)
      return None
    log.info('rank-local GPU %d on NUMA node %d: pinned to %d CPUs',
             local_rank, node, len(target))
  return node, sorted(target)
