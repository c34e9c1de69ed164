#!/usr/bin/env python3
"""Per-kernel PMC table from rocprofv3 --pmc csv dirs (sums over dispatches,
prints ratios per wave-cycle / per instruction).
usage: pmc_table.py dir1 [dir2 ...] [--filter sa::]"""
import collections
import csv
import glob
import sys


def load(dirs, filt):
  agg = collections.defaultdict(lambda: collections.defaultdict(float))
  disp = collections.defaultdict(set)
  for d in dirs:
    for f in glob.glob(d + '/*counter_collection.csv'):
      for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '')
        k = k.split('(')[0].replace('void ', '').replace('sa::conv::', '')
        if filt not in r['Kernel_Name']:
          continue
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        disp[k].add((d, r['Dispatch_Id']))
  return agg, disp


def main():
  args = [a for a in sys.argv[1:] if not a.startswith('--')]
  filt = 'sa::'
  for a in sys.argv[1:]:
    if a.startswith('--filter='):
      filt = a.split('=', 1)[1]
  agg, disp = load(args, filt)
  cols = [('busy', 'SQ_ACTIVE_INST_ANY', 'SQ_WAVE_CYCLES'),
          ('wait', 'SQ_WAIT_ANY', 'SQ_WAVE_CYCLES'),
          ('wInst', 'SQ_WAIT_INST_ANY', 'SQ_WAVE_CYCLES'),
          ('wLDS', 'SQ_WAIT_INST_LDS', 'SQ_WAVE_CYCLES'),
          ('aVALU', 'SQ_ACTIVE_INST_VALU', 'SQ_WAVE_CYCLES'),
          ('aLDS', 'SQ_ACTIVE_INST_LDS', 'SQ_WAVE_CYCLES'),
          ('aVMEM', 'SQ_ACTIVE_INST_VMEM', 'SQ_WAVE_CYCLES'),
          ('valu/mfma', 'SQ_INSTS_VALU', 'SQ_INSTS_MFMA'),
          ('lds/mfma', 'SQ_INSTS_LDS', 'SQ_INSTS_MFMA'),
          ('conf/lds', 'SQ_LDS_BANK_CONFLICT', 'SQ_INSTS_LDS'),
          ('waves', 'SQ_LEVEL_WAVES', 'SQ_BUSY_CYCLES'),
          ('mfmaB', 'SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_BUSY_CYCLES')]
  print('%-44s' % 'kernel' + ''.join('%10s' % c[0] for c in cols) +
        '%10s%10s' % ('fetchMB', 'writeMB'))
  for k in sorted(agg):
    d = agg[k]
    row = '%-44s' % k[:44]
    for _, a, b in cols:
      row += '%10.2f' % (d[a] / d[b]) if d.get(a) and d.get(b) else '%10s' % '-'
    n = max(1, len([x for x in disp[k] if 'pmc3' in x[0]]))
    row += '%10.0f' % (d.get('FETCH_SIZE', 0) / n / 1024) if d.get(
        'FETCH_SIZE') else '%10s' % '-'
    n = max(1, len([x for x in disp[k] if 'pmc4' in x[0]]))
    row += '%10.0f' % (d.get('WRITE_SIZE', 0) / n / 1024) if d.get(
        'WRITE_SIZE') else '%10s' % '-'
    print(row)


if __name__ == '__main__':
  main()
