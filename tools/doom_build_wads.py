#!/usr/bin/env python3
"""Writes this framework's Doom scenario WADs (envs/doom/scenario_maps.py)
into a directory, e.g. to ship them next to the .cfg files or to point
SA_DOOM_SCENARIOS_DIR at them.

  python tools/doom_build_wads.py OUT_DIR [--acc /path/to/acc] [--only basic.wad ...]

--acc: ZDoom's ACS compiler; each map's SCRIPTS lump is then compiled into a
BEHAVIOR lump, which real ViZDoom needs to run the scenario rules (without
it the maps load and only the .cfg rewards apply).  The in-tree simulator
backend needs no BEHAVIOR.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scalable_agent_amd.envs.doom import scenario_maps, wad  # noqa: E402


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('out_dir')
  ap.add_argument('--acc', default=None)
  ap.add_argument('--only', nargs='*', default=None)
  a = ap.parse_args()
  for path in scenario_maps.build_all(a.out_dir, acc=a.acc, names=a.only):
    lumps = wad.read_wad(path)
    maps = wad.map_names(lumps)
    print('%-24s %7d bytes  maps %s%s' % (
        os.path.basename(path), os.path.getsize(path), ','.join(maps),
        '  +BEHAVIOR' if any(n == 'BEHAVIOR' for n, _ in lumps) else ''))


if __name__ == '__main__':
  main()
