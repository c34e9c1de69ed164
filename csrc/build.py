#!/usr/bin/env python3
"""Builds the in-tree native extensions (no hipify, no torch JIT cache).

  * scalable_agent_amd/_C.so        gfx950 HIP kernels + torch bindings
                                    (csrc/kernels/*.hip, csrc/*.cpp)
  * scalable_agent_amd/runtime/_native.so
                                    host-only C++17 runtime: dynamic batcher,
                                    trajectory ring, env-pool primitives
                                    (csrc/batcher/, csrc/envpool/) via pybind11

hipcc cross-compiles gfx950 without a GPU.  Objects are rebuilt when the
source or any header in csrc/ changes.  Usage: python csrc/build.py [-j N]
[--force] [--only C|native] [--sanitize thread|address] (sanitizers apply to
the host-only runtime, the HIP code is never built with GPU sanitizers).
"""

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'csrc')
BUILD = os.path.join(ROOT, 'build')
PKG = os.path.join(ROOT, 'scalable_agent_amd')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('SA_OFFLOAD_ARCH', 'gfx950')


def _torch_paths():
  import torch
  import torch.utils.cpp_extension as ce
  inc = ce.include_paths(device_type='cuda')
  lib = os.path.join(os.path.dirname(torch.__file__), 'lib')
  abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
  return inc, lib, abi


def _pybind_inc():
  import pybind11
  return pybind11.get_include()


def _headers_digest(dirs):
  h = hashlib.sha1()
  for d in dirs:
    for p in sorted(glob.glob(os.path.join(d, '**', '*.h'), recursive=True)):
      with open(p, 'rb') as f:
        h.update(p.encode())
        h.update(f.read())
  return h.hexdigest()[:12]


def _run(cmd):
  r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                     text=True)
  if r.returncode != 0:
    raise RuntimeError('command failed:\n%s\n%s' % (' '.join(cmd), r.stdout))
  return r.stdout


def _compile_all(jobs, workers):
  todo = [(src, obj, cmd) for src, obj, cmd in jobs
          if not (os.path.exists(obj) and
                  os.path.getmtime(obj) >= os.path.getmtime(src))]
  if not todo:
    return
  with cf.ThreadPoolExecutor(max_workers=workers) as ex:
    futs = {ex.submit(_run, cmd): src for src, _, cmd in todo}
    for f in cf.as_completed(futs):
      f.result()
      print('  compiled', os.path.relpath(futs[f], ROOT), flush=True)


def build_hip(workers=8, force=False, extra_flags=(), out=None):
  inc, lib, abi = _torch_paths()
  py_inc = sysconfig.get_paths()['include']
  digest = _headers_digest([CSRC])
  if extra_flags:
    digest += '-' + hashlib.sha1(' '.join(extra_flags).encode()).hexdigest()[:8]
  objdir = os.path.join(BUILD, 'hip-%s' % digest)
  os.makedirs(objdir, exist_ok=True)
  if force:
    for o in glob.glob(os.path.join(objdir, '*.o')):
      os.remove(o)
  common = ['-O3', '-std=c++17', '-fPIC', '-I' + CSRC] + list(extra_flags)
  jobs = []
  for src in sorted(glob.glob(os.path.join(CSRC, 'kernels', '*.hip'))):
    obj = os.path.join(objdir, os.path.basename(src) + '.o')
    cmd = [HIPCC, '-c', src, '-o', obj, '--offload-arch=' + ARCH,
           '-munsafe-fp-atomics'] + common
    jobs.append((src, obj, cmd))
  torch_flags = ['-DTORCH_EXTENSION_NAME=_C', '-DTORCH_API_INCLUDE_EXTENSION_H',
                 '-D_GLIBCXX_USE_CXX11_ABI=%d' % abi, '-DUSE_ROCM=1',
                 '-D__HIP_PLATFORM_AMD__=1', '-I' + py_inc] + [
                     '-I' + p for p in inc]
  for src in sorted(glob.glob(os.path.join(CSRC, '*.cpp'))):
    obj = os.path.join(objdir, os.path.basename(src) + '.o')
    cmd = [HIPCC, '-c', src, '-o', obj] + common + torch_flags + [
        '-Wno-unused-parameter', '-Wno-deprecated-declarations']
    jobs.append((src, obj, cmd))
  _compile_all(jobs, workers)
  out = out or os.path.join(PKG, '_C.so')
  objs = [o for _, o, _ in jobs]
  if (force or not os.path.exists(out) or
      max(os.path.getmtime(o) for o in objs) > os.path.getmtime(out)):
    # link to a temporary name and rename: a concurrent reader (a gpurun
    # snapshot, an importing process) never sees a half-written library
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    tmp_out = out + '.tmp'
    cmd = [HIPCC, '-shared', '-fPIC', '-o', tmp_out] + objs + [
        '--offload-arch=' + ARCH, '-L' + lib, '-Wl,-rpath,' + lib,
        '-lc10', '-lc10_hip', '-ltorch', '-ltorch_cpu', '-ltorch_hip',
        '-ltorch_python', '-lamdhip64']
    _run(cmd)
    os.replace(tmp_out, out)
    print('  linked', os.path.relpath(out, ROOT), flush=True)
  return out


def build_native(workers=8, force=False, sanitize=None):
  py_inc = sysconfig.get_paths()['include']
  digest = _headers_digest([CSRC]) + ('-' + sanitize if sanitize else '')
  objdir = os.path.join(BUILD, 'native-%s' % digest)
  os.makedirs(objdir, exist_ok=True)
  cxx = os.environ.get('CXX', '/opt/rocm/lib/llvm/bin/clang++')
  if not os.path.exists(cxx):
    cxx = 'g++'
  flags = ['-O2', '-g', '-std=c++17', '-fPIC', '-I' + CSRC, '-I' + py_inc,
           '-I' + _pybind_inc(), '-Wall', '-Wextra', '-pthread',
           '-fvisibility=hidden']
  if 'clang' in cxx:
    flags += ['-Wthread-safety', '-Werror=thread-safety']
  if sanitize:
    flags += ['-fsanitize=%s' % sanitize, '-fno-omit-frame-pointer', '-O1']
  srcs = sorted(glob.glob(os.path.join(CSRC, 'batcher', '*.cc')) +
                glob.glob(os.path.join(CSRC, 'envpool', '*.cc')))
  jobs = []
  for src in srcs:
    obj = os.path.join(objdir, os.path.basename(src) + '.o')
    jobs.append((src, obj, [cxx, '-c', src, '-o', obj] + flags))
  if force:
    for _, o, _ in jobs:
      if os.path.exists(o):
        os.remove(o)
  _compile_all(jobs, workers)
  # Sanitizer builds keep the module name `_native` (PyInit__native) and live
  # in their own directory; runtime/native.py loads them by path.
  outdir = os.path.join(PKG, 'runtime') if not sanitize else \
      os.path.join(BUILD, 'san_' + sanitize)
  os.makedirs(outdir, exist_ok=True)
  out = os.path.join(outdir, '_native.so')
  objs = [o for _, o, _ in jobs]
  if (force or not os.path.exists(out) or
      max(os.path.getmtime(o) for o in objs) > os.path.getmtime(out)):
    tmp_out = out + '.tmp'  # atomic replace, as build_hip
    cmd = [cxx, '-shared', '-o', tmp_out] + objs + ['-pthread', '-lrt']
    if sanitize:
      cmd += ['-fsanitize=%s' % sanitize]
    _run(cmd)
    os.replace(tmp_out, out)
    print('  linked', os.path.relpath(out, ROOT), flush=True)
  return out


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('-j', type=int, default=min(8, os.cpu_count() or 4))
  ap.add_argument('--force', action='store_true')
  ap.add_argument('--only', choices=['C', 'native'], default=None)
  ap.add_argument('--sanitize', choices=['thread', 'address'], default=None)
  ap.add_argument('--define', action='append', default=[],
                  help='experiment builds: -D NAME=VAL for the HIP extension '
                       '(objects in their own build dir); use with --out')
  ap.add_argument('--flag', action='append', default=[],
                  help='experiment builds: an extra compiler flag for the HIP '
                       'extension (e.g. --flag=-mllvm --flag=-amdgpu-...); use '
                       'with --out')
  ap.add_argument('--out', default=None,
                  help='HIP extension output path (experiment builds, loaded '
                       'with SA_EXT_PATH)')
  args = ap.parse_args()
  if (args.define or args.flag) and not args.out:
    ap.error('--define / --flag need --out (the in-tree _C.so stays the '
             'default build)')
  if args.only in (None, 'native') and not (args.define or args.flag):
    build_native(args.j, args.force, args.sanitize)
  if args.only in (None, 'C') and not args.sanitize:
    build_hip(args.j, args.force,
              extra_flags=['-D' + d for d in args.define] + list(args.flag),
              out=args.out)


if __name__ == '__main__':
  sys.exit(main())
