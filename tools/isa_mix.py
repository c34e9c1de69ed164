#!/usr/bin/env python3
"""Static instruction mix per basic block of one kernel in a gfx950 .s file
(hipcc -S --cuda-device-only).  Loop blocks (those that branch back to
themselves or to an earlier block) are marked '*'.
usage: isa_mix.py file.s <kernel-substring> [--all]"""
import collections
import re
import sys


def kind(op):
  if op.startswith('v_mfma'):
    return 'mfma'
  if op.startswith('ds_'):
    return 'ds'
  if op.startswith(('global_', 'buffer_', 'flat_')):
    return 'vmem'
  if op.startswith('v_'):
    return 'valu'
  if op.startswith('s_'):
    return 'salu'
  return 'other'


def main():
  path, sub = sys.argv[1], sys.argv[2]
  lines = open(path).read().split('\n')
  start = next(i for i, l in enumerate(lines)
               if re.match(r'^_Z\S*:', l) and sub in l)
  end = next(i for i in range(start, len(lines))
             if lines[i].startswith('.Lfunc_end'))
  print(lines[start].split(':')[0])
  blocks, cur, order = [], None, {}
  for l in lines[start + 1:end + 1]:
    t = l.strip()
    m = re.match(r'^(\.LBB\w+):', t)
    if m:
      cur = [m.group(1), collections.Counter(), []]
      order[m.group(1)] = len(blocks)
      blocks.append(cur)
      continue
    if cur is None:
      cur = ['entry', collections.Counter(), []]
      blocks.append(cur)
    if not t or t.startswith(('.', ';')):
      continue
    op = t.split()[0]
    cur[1][kind(op)] += 1
    if op.startswith(('s_cbranch', 's_branch')):
      cur[2].append(t.split()[-1])
  tot = collections.Counter()
  for i, (name, c, br) in enumerate(blocks):
    tot.update(c)
    loop = any(order.get(b, 1 << 30) <= i for b in br)
    if loop or '--all' in sys.argv:
      print('%s %-14s %s' % ('*' if loop else ' ', name,
                             ' '.join('%s=%d' % kv for kv in sorted(c.items()))))
  print('total', ' '.join('%s=%d' % kv for kv in sorted(tot.items())))


if __name__ == '__main__':
  main()
