#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace: per-kernel time per learner step.

usage: prof_summary.py <run_results.db | kernel_stats.csv> [steps|auto] [top]

`auto` divides by the number of fused V-trace-loss launches (exactly one per
learner step), so warmup/capture steps are accounted for.
"""
import csv
import sqlite3
import sys


def load(path):
  """-> list of (name, calls, total_ns, vgpr, lds, grid, wg)."""
  if path.endswith('.db'):
    c = sqlite3.connect(path)
    q = ('select name, count(*), sum(duration), max(vgpr_count), '
         'max(accum_vgpr_count), max(lds_size), max(grid_x*grid_y*grid_z), '
         'max(workgroup_x*workgroup_y*workgroup_z) from kernels group by name')
    return [(r[0], r[1], float(r[2]), '%d+%d' % (r[3], r[4]), r[5], r[6],
             r[7]) for r in c.execute(q)]
  rows = list(csv.DictReader(open(path)))
  return [(r['Name'], int(r['Calls']), float(r['TotalDurationNs']), '', '',
           '', '') for r in rows]


def main():
  path = sys.argv[1]
  rows = load(path)
  steps_arg = sys.argv[2] if len(sys.argv) > 2 else 'auto'
  top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
  if steps_arg == 'auto':
    steps = max([r[1] for r in rows if 'vtrace_loss_kernel' in r[0] or 'learner_head_fwd' in r[0]] or [1])
  else:
    steps = float(steps_arg)
  tot = sum(r[2] for r in rows)
  print('total kernel time %.3f ms over %g steps = %.3f ms/step (%d kernels)'
        % (tot / 1e6, steps, tot / 1e6 / steps, len(rows)))
  print('%9s %7s %9s %6s %8s %7s %9s %5s  %s' % (
      'ms/step', 'calls', 'us/call', '%', 'vgpr+a', 'lds', 'grid', 'wg',
      'kernel'))
  for name, calls, t, vgpr, lds, grid, wg in sorted(rows,
                                                    key=lambda r: -r[2])[:top]:
    name = name.replace('(anonymous namespace)::', '')
    print('%9.3f %7d %9.1f %6.1f %8s %7s %9s %5s  %s' % (
        t / 1e6 / steps, calls, t / 1e3 / calls, 100 * t / tot, vgpr, lds,
        grid, wg, name[:120]))


if __name__ == '__main__':
  main()
