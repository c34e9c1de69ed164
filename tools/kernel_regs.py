#!/usr/bin/env python3
"""Register/LDS/spill summary of every kernel in a gfx950 .s file
(hipcc -S --cuda-device-only).  usage: kernel_regs.py file.s [filter]"""
import re
import subprocess
import sys


def main():
  text = open(sys.argv[1]).read()
  filt = sys.argv[2] if len(sys.argv) > 2 else ''
  meta = text[text.find('amdhsa.kernels:'):]
  for blk in re.split(r'\n  - ', meta)[1:]:
    get = lambda k: (re.search(r'\.%s:\s+(\S+)' % k, blk) or [None, '?'])[1]
    name = get('name')
    dn = subprocess.run(['c++filt', name], capture_output=True,
                        text=True).stdout.strip()
    dn = dn.replace('(anonymous namespace)::', '')
    if filt in dn:
      print('vgpr %4s agpr %4s spill %3s sgpr %3s lds %6s  %s' % (
          get('vgpr_count'), get('agpr_count'), get('vgpr_spill_count'),
          get('sgpr_count'), get('group_segment_fixed_size'), dn[:100]))


if __name__ == '__main__':
  main()
