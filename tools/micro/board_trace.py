#!/usr/bin/env python3
"""Where an inference-board launch's time goes (profiles/r6_e2e.md).

  python3 tools/micro/board_trace.py RUN_RESULTS.db [OUT.txt]

Reads a rocprofv3 --kernel-trace --memory-copy-trace database of an
`experiment.py` run with the inference board, finds the board's launches by
their last kernel (actor_head_sample_kernel: the fused heads + sampler ends
every inference graph) on the inference queue, and prints for the steady
state (the middle half of the launches): launches per second, the mean time
from one launch's first kernel to its sampler's end, the GPU-busy part of it,
the kernels of one launch (name, us) and the copies on the queue.
"""
import collections
import sqlite3
import sys


def main():
  db, out = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else None)
  c = sqlite3.connect(db)
  rows = list(c.execute('select name, queue_id, start, end from kernels '
                        'order by start'))
  samp = [r for r in rows if 'actor_head_sample' in r[0]]
  if not samp:
    raise SystemExit('no actor_head_sample_kernel in the trace')
  q = collections.Counter(r[1] for r in samp).most_common(1)[0][0]
  inf = [r for r in rows if r[1] == q]
  ends = [r[3] for r in samp if r[1] == q]
  # launches: the kernels of the inference queue between two sampler ends
  launches, cur = [], []
  ei = 0
  for r in inf:
    cur.append(r)
    if 'actor_head_sample' in r[0]:
      launches.append(cur)
      cur = []
  n = len(launches)
  mid = launches[n // 4: 3 * n // 4] or launches
  span = (mid[-1][-1][3] - mid[0][0][2]) / 1e9
  lines = ['# tools/micro/board_trace.py %s' % db,
           'inference queue %d: %d launches, steady state (middle half) %d '
           'launches in %.3f s = %.0f launches/s' % (q, n, len(mid), span,
                                                    len(mid) / span)]
  first_to_end = [(l[-1][3] - l[0][2]) / 1e3 for l in mid]
  busy = [sum(r[3] - r[2] for r in l) / 1e3 for l in mid]
  gaps = [(mid[i + 1][0][2] - mid[i][-1][3]) / 1e3 for i in range(len(mid) - 1)]
  med = lambda v: sorted(v)[len(v) // 2]
  lines.append('per launch (median): %d kernels, first kernel -> sampler end '
               '%.1f us, kernel time %.1f us, gap to the next launch %.1f us'
               % (med([len(l) for l in mid]), med(first_to_end), med(busy),
                  med(gaps)))
  fam = collections.OrderedDict()
  for l in mid:
    for r in l:
      k = r[0].split('(')[0][-70:]
      d = fam.setdefault(k, [0, 0.0])
      d[0] += 1
      d[1] += (r[3] - r[2]) / 1e3
  lines.append('%10s %8s  kernel (per launch, steady state)' % ('us', 'calls'))
  for k, (cnt, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
    lines.append('%10.1f %8.2f  %s' % (t / len(mid), cnt / len(mid), k))
  # one steady-state launch in order: start offset, duration, gap before
  one = mid[len(mid) // 2]
  lines.append('one launch (offset us, duration us, gap before us, kernel):')
  prev = None
  for r in one:
    lines.append('%8.1f %7.1f %7.1f  %s' % (
        (r[2] - one[0][2]) / 1e3, (r[3] - r[2]) / 1e3,
        0.0 if prev is None else (r[2] - prev) / 1e3, r[0][:90]))
    prev = r[3]
  try:
    cps = list(c.execute('select start, end, size from memory_copies'))
    # the copies of that launch's window (offsets from its first kernel)
    w0, w1 = one[0][2], one[-1][3]
    lines.append('copies in that window (offset us, duration us, bytes):')
    for x in sorted(cps):
      if w0 <= x[0] <= w1:
        lines.append('%8.1f %7.1f %10d' % ((x[0] - w0) / 1e3,
                                            (x[1] - x[0]) / 1e3, x[2] or 0))
    t0, t1 = mid[0][0][2], mid[-1][-1][3]
    cps = [x for x in cps if t0 <= x[0] <= t1]
    if cps:
      lines.append('memory copies in the window: %d, %.1f MB, median %.1f us'
                   % (len(cps), sum(x[2] or 0 for x in cps) / 1e6,
                      med([(x[1] - x[0]) / 1e3 for x in cps])))
  except sqlite3.Error as e:
    lines.append('memory copies: %s' % e)
  text = '\n'.join(lines)
  print(text)
  if out:
    open(out, 'w').write(text + '\n')


if __name__ == '__main__':
  main()
