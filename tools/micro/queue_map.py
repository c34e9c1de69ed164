"""Which hardware queue HIP gives each stream (parallel/streams.py design).

  rocprofv3 --kernel-trace -d OUT -o run -- python3 tools/micro/queue_map.py [MODE]
  python3 tools/micro/queue_map.py --parse OUT/run_results.db

MODE: 'pool' (default) five torch pool streams used in creation order;
'rev' the same streams used in reverse order; 'prio' normal and
high-priority pool streams.  Each stream runs one fill of its own dtype;
--parse prints (queue_id, stream_id) per marker.
"""

import collections
import sqlite3
import sys

DTYPES = ['bool', 'int8', 'int16', 'int32', 'int64', 'float16', 'bfloat16',
          'float64']
KERNEL_T = {'bool': 'bool', 'int8': 'signed char', 'int16': 'short',
            'int32': 'int', 'int64': 'long', 'float16': 'c10::Half',
            'bfloat16': 'c10::BFloat16', 'float64': 'double'}


def probe(mode):
  import torch
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(dev)
  torch.empty(1, device=dev).fill_(0)  # the default stream first
  names = ['default']
  streams = [torch.cuda.current_stream(dev)]
  if mode == 'prio':
    for i in range(3):
      streams.append(torch.cuda.Stream(dev))
      names.append('normal%d' % i)
    for i in range(3):
      streams.append(torch.cuda.Stream(dev, priority=-1))
      names.append('high%d' % i)
  else:
    for i in range(6):
      streams.append(torch.cuda.Stream(dev))
      names.append('pool%d' % i)
  order = list(range(len(streams)))
  if mode == 'rev':
    order = [0] + order[:0:-1]
  for i in order:
    with torch.cuda.stream(streams[i]):
      torch.empty(1 << 12, dtype=getattr(torch, DTYPES[i]), device=dev).fill_(1)
  torch.cuda.synchronize()
  for i in order:
    print('%-8s uses %s (first-use position %d)' % (names[i], DTYPES[i],
                                                     order.index(i)))


def parse(path):
  c = sqlite3.connect(path)
  seen = collections.OrderedDict()
  for name, q, s in c.execute('select name, queue_id, stream_id from kernels '
                              'order by start'):
    for dt in DTYPES:
      if 'FillFunctor<%s>' % KERNEL_T[dt] in name:
        seen.setdefault(dt, set()).add((q, s))
  for dt, qs in seen.items():
    print('%-9s (queue, stream) %s' % (dt, sorted(qs)))


if __name__ == '__main__':
  if len(sys.argv) > 2 and sys.argv[1] == '--parse':
    parse(sys.argv[2])
  else:
    probe(sys.argv[1] if len(sys.argv) > 1 else 'pool')
