#!/usr/bin/env python3
"""Host CPU profile of an end-to-end run, by process role.

  python tools/micro/cpu_sampler.py OUT.txt -- python experiment.py ...

Starts the command as a child (its own process group), samples the CPU time
of every process in its tree every `--every` seconds with psutil and writes,
per role, the CPU time used and the average number of CPUs busy:

  learner     the command's own process (learner loop, feeder, board server)
  group       processes whose children are env processes (actor groups)
  env         env supervisors and env workers (leaf processes)
  other       anything else (compile workers, tools)

plus the cgroup CPU quota when one is visible (cpu.max), the number of
processes per role and the run's wall time.  The command's exit code is
returned.  Used for profiles/r6_e2e.md (what bounds the
end-to-end actor throughput).
"""

import os
import signal
import subprocess
import sys
import time

import psutil


def _quota():
  for path in ('/sys/fs/cgroup/cpu.max',):
    try:
      q, p = open(path).read().split()[:2]
      if q != 'max':
        return float(q) / float(p)
    except (OSError, ValueError):
      pass
  try:
    q = int(open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us').read())
    p = int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
    if q > 0:
      return q / p
  except (OSError, ValueError):
    pass
  return None


def _role(proc, root_pid, kids_of):
  if proc.pid == root_pid:
    return 'learner'
  # an actor group has many children (its envs); an env supervisor has one
  # (its worker); an env worker none
  return 'group' if len(kids_of.get(proc.pid, ())) >= 2 else 'env'


def main():
  if '--' not in sys.argv:
    raise SystemExit(__doc__)
  i = sys.argv.index('--')
  out = sys.argv[1]
  every = 1.0
  cmd = sys.argv[i + 1:]
  t0 = time.time()
  child = subprocess.Popen(cmd, start_new_session=True)
  root = psutil.Process(child.pid)
  cpu = {}      # pid -> last (user + system) seconds
  role_of = {}  # pid -> role
  used = {}     # role -> cpu seconds
  peak = {}     # role -> max processes seen at once
  try:
    while child.poll() is None:
      try:
        procs = [root] + root.children(recursive=True)
      except psutil.Error:
        procs = [root]
      kids_of = {}
      for p in procs:
        try:
          kids_of.setdefault(p.ppid(), []).append(p.pid)
        except psutil.Error:
          pass
      count = {}
      for p in procs:
        try:
          t = p.cpu_times()
        except psutil.Error:
          continue
        s = t.user + t.system
        r = role_of.get(p.pid)
        if r is None or r == 'env':
          r = role_of[p.pid] = _role(p, child.pid, kids_of)
        used[r] = used.get(r, 0.0) + s - cpu.get(p.pid, 0.0)
        cpu[p.pid] = s
        count[r] = count.get(r, 0) + 1
      for r, n in count.items():
        peak[r] = max(peak.get(r, 0), n)
      time.sleep(every)
  except KeyboardInterrupt:
    os.killpg(child.pid, signal.SIGTERM)
  rc = child.wait()
  wall = time.time() - t0
  lines = ['# tools/micro/cpu_sampler.py: %s' % ' '.join(cmd),
           'wall %.1f s, cgroup CPU quota %s, os.cpu_count %d' % (
               wall, _quota(), os.cpu_count()),
           '%-8s %8s %10s %10s' % ('role', 'procs', 'cpu s', 'avg CPUs')]
  for r in ('learner', 'group', 'env', 'other'):
    if r in used:
      lines.append('%-8s %8d %10.1f %10.2f' % (r, peak.get(r, 0), used[r],
                                              used[r] / wall))
  tot = sum(used.values())
  lines.append('%-8s %8d %10.1f %10.2f' % ('total', sum(peak.values()), tot,
                                          tot / wall))
  with open(out, 'w') as f:
    f.write('\n'.join(lines) + '\n')
  print('\n'.join(lines), flush=True)
  return rc


if __name__ == '__main__':
  sys.exit(main())
