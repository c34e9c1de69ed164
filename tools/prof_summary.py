#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel CSV: per-kernel time per learner step."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print('total kernel time %.3f ms over %g steps = %.3f ms/step (%d kernels)'
      % (tot / 1e6, steps, tot / 1e6 / steps, len(rows)))
print('%10s %8s %10s %6s  %s' % ('ms/step', 'calls', 'us/call', '%', 'kernel'))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:top]:
  t = float(r['TotalDurationNs'])
  c = int(r['Calls'])
  name = r['Name'].replace('(anonymous namespace)::', '')
  print('%10.3f %8d %10.1f %6.1f  %s' % (t / 1e6 / steps, c, t / 1e3 / c,
                                        100 * t / tot, name[:110]))
