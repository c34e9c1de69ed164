"""Host runtime under ThreadSanitizer and AddressSanitizer/UBSan.

SURVEY.md §5.2 (race detection): the reference relies on Clang thread-safety
annotations (dynamic_batching.cc Mutex/GUARDED_BY) only.  Here the C++ batcher
and the shared-memory ring also run a multi-threaded stress driver
(csrc/tests/runtime_stress.cc) compiled with -fsanitize=thread and with
-fsanitize=address,undefined; any data race, heap misuse or UB aborts the
binary with a sanitizer report.  Host code only (no GPU sanitizers on this
pool).
"""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'csrc')
SOURCES = [os.path.join(CSRC, 'tests', 'runtime_stress.cc'),
           os.path.join(CSRC, 'batcher', 'batcher.cc'),
           os.path.join(CSRC, 'envpool', 'shm_ring.cc')]


def _clang():
  for c in ('/opt/rocm/lib/llvm/bin/clang++', shutil.which('clang++')):
    if c and os.path.exists(c):
      return c
  return None


@pytest.mark.parametrize('san', ['thread', 'address,undefined'])
def test_runtime_stress_sanitized(san, tmp_path):
  cxx = _clang()
  if cxx is None:
    pytest.skip('clang++ not available')
  exe = str(tmp_path / ('stress_' + san.split(',')[0]))
  cmd = [cxx, '-std=c++17', '-O1', '-g', '-fsanitize=' + san,
         '-fno-omit-frame-pointer', '-fno-sanitize-recover=all', '-pthread',
         '-I', CSRC] + SOURCES + ['-o', exe, '-lrt']
  r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
  assert r.returncode == 0, r.stderr[-4000:]
  env = dict(os.environ)
  env['TSAN_OPTIONS'] = 'halt_on_error=1'
  env['ASAN_OPTIONS'] = 'detect_leaks=1'
  r = subprocess.run([exe, '100'], capture_output=True, text=True,
                     timeout=300, env=env)
  assert r.returncode == 0, (r.stdout + r.stderr)[-6000:]
  assert 'runtime stress ok' in r.stdout
