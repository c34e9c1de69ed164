#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 kernel trace (rocpd .db).

usage: timeline.py <run_results.db> [step_index_from_end=2] [--list]

Steps are delimited by the fused V-trace+loss kernel (one per learner step).
For the chosen step (window from one V-trace launch to the next) it prints the
wall span, the summed kernel time (> span means kernels overlapped), the busy
time (union of kernel intervals), the idle gaps, and per-kernel-family
busy/overlap numbers by HW queue.  --list prints every kernel of the window.
"""
import collections
import sqlite3
import sys


def short(name):
  name = name.replace('(anonymous namespace)::', '')
  for key in ('lstm_fwd_step', 'lstm_bwd_step', 'conv1_pool_fwd',
              'conv1_pool_bwd', 'conv_pool_fwd', 'pool_conv_bwd',
              'res_conv_fwd', 'res_conv_bwd', 'vtrace_loss', 'rmsprop',
              'Cijk', 'copyBuffer', 'fillBuffer'):
    if key in name:
      if key.startswith('res_conv') or key.startswith('conv_pool') or \
          key.startswith('pool_conv'):
        tmpl = name[name.find('<'):name.find('>') + 1]
        return key + tmpl
      return key
  if 'at::native' in name:
    i = name.find('at::native::')
    return 'torch:' + name[i + 12:i + 50]
  return name[:50]


def union(iv):
  iv = sorted(iv)
  tot, cur_s, cur_e = 0, None, None
  for s, e in iv:
    if cur_e is None or s > cur_e:
      if cur_e is not None:
        tot += cur_e - cur_s
      cur_s, cur_e = s, e
    else:
      cur_e = max(cur_e, e)
  if cur_e is not None:
    tot += cur_e - cur_s
  return tot


def main():
  path = sys.argv[1]
  back = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2][0] != '-' else 2
  c = sqlite3.connect(path)
  rows = list(c.execute('select name, start, end, queue_id, stream_id from '
                        'kernels order by start'))
  marks = [r[1] for r in rows if 'vtrace_loss' in r[0] or 'learner_head_fwd' in r[0]]
  if len(marks) < back + 1:
    raise SystemExit('not enough steps')
  t0, t1 = marks[-back - 1], marks[-back]
  win = [r for r in rows if t0 <= r[1] < t1]
  span = t1 - t0
  ksum = sum(r[2] - r[1] for r in win)
  busy = union([(r[1], r[2]) for r in win])
  print('step window %.3f ms: kernel sum %.3f ms, busy (union) %.3f ms, '
        'idle %.3f ms, %d kernels' % (span / 1e6, ksum / 1e6, busy / 1e6,
                                      (span - busy) / 1e6, len(win)))
  fam = collections.OrderedDict()
  for r in win:
    k = short(r[0])
    d = fam.setdefault(k, [0, 0, set()])
    d[0] += 1
    d[1] += r[2] - r[1]
    d[2].add(r[3])
  print('%8s %6s %9s  %s' % ('ms', 'calls', 'queues', 'family'))
  for k, (n, t, q) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
    print('%8.3f %6d %9s  %s' % (t / 1e6, n, ','.join(map(str, sorted(q))), k))
  if '--list' in sys.argv:
    for r in win:
      print('%9.1f %8.1f q%-3d %s' % ((r[1] - t0) / 1e3, (r[2] - r[1]) / 1e3,
                                     r[3], short(r[0])))


if __name__ == '__main__':
  main()
