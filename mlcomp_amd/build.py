"""Build the native parts of mlcomp_amd in-tree.

* ``libmlcomp_kernels.so`` - every ``csrc/kernels/*.hip`` compiled for gfx950 with hipcc
  (extern "C" launchers, loaded with ctypes by :mod:`mlcomp_amd.ops._lib`); links RCCL and
  no vendor GEMM / conv library.
* ``libmlcomp_kernels_blaslt.so`` - its bench-only A/B twin: the same kernel objects, with
  ``csrc/bench/blaslt.hip`` (timed per-shape hipBLASLt selection) in place of
  ``dense_entry.hip``; loaded only through ``MLC_KERNEL_LIB`` by comparison scripts / tests.
* ``mlcomp-broker`` - the C++17 epoll task-queue daemon (``csrc/broker``), the native
  replacement for the reference's vendored redis-server (`mlcomp/bin/redis-server`,
  launched at `mlcomp/server/__main__.py:66-79`).
* ``libmlcomp_runtime.so`` - host-side C++ runtime (``csrc/runtime``): the memory-mapped
  record files and the threaded batch gatherer of the native input pipeline
  (:mod:`mlcomp_amd.train.records`); ``mlcomp-records-selftest-<san>`` is its
  ThreadSanitizer / AddressSanitizer self-test.

Outputs live under ``mlcomp_amd/_native/`` so they travel with the repo snapshot.
Compilation is incremental (mtime based) and parallel.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'mlcomp_amd', '_native')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('MLC_OFFLOAD_ARCH', 'gfx950')

KERNEL_LIB = os.path.join(OUT, 'libmlcomp_kernels.so')
BLASLT_LIB = os.path.join(OUT, 'libmlcomp_kernels_blaslt.so')
BROKER_BIN = os.path.join(OUT, 'mlcomp-broker')
RUNTIME_LIB = os.path.join(OUT, 'libmlcomp_runtime.so')


def _newer(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError('command failed: ' + ' '.join(cmd) + '\n' + r.stdout + r.stderr)
    return r


def build_kernels(verbose=False, jobs=None):
    os.makedirs(OUT, exist_ok=True)
    bench = sorted(glob.glob(os.path.join(ROOT, 'csrc', 'bench', '*.hip')))
    srcs = sorted(glob.glob(os.path.join(ROOT, 'csrc', 'kernels', '*.hip'))) + bench
    headers = glob.glob(os.path.join(ROOT, 'csrc', 'kernels', '*.h'))
    objdir = os.path.join(OUT, 'obj')
    os.makedirs(objdir, exist_ok=True)
    flags = ['-O3', '-std=c++17', '-fPIC', f'--offload-arch={ARCH}', '-Wno-unused-result',
             '-munsafe-fp-atomics', '-I', os.path.join(ROOT, 'csrc', 'kernels')]
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + '.o')
        objs.append(o)
        if _newer(o, [s] + headers):
            todo.append((s, o))
    jobs = jobs or min(8, max(1, len(todo)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_run, [HIPCC] + flags + ['-c', s, '-o', o]) for s, o in todo]
        for f in futs:
            f.result()
    bench_objs = [os.path.join(objdir, os.path.basename(s) + '.o') for s in bench]
    entry = os.path.join(objdir, 'dense_entry.hip.o')
    prod = [o for o in objs if o not in bench_objs]
    if todo or _newer(KERNEL_LIB, prod):
        _run([HIPCC, '-shared', '-fPIC', f'--offload-arch={ARCH}', '-o', KERNEL_LIB] + prod
             + ['-L/opt/rocm/lib', '-lrccl', '-Wl,-rpath,/opt/rocm/lib'])
    twin = [o for o in prod if o != entry] + bench_objs
    if bench_objs and (todo or _newer(BLASLT_LIB, twin)):
        _run([HIPCC, '-shared', '-fPIC', f'--offload-arch={ARCH}', '-o', BLASLT_LIB] + twin
             + ['-L/opt/rocm/lib', '-lrccl', '-lhipblaslt', '-Wl,-rpath,/opt/rocm/lib'])
    if verbose:
        print(f'[build] kernels: {len(todo)} rebuilt -> {KERNEL_LIB} (+ bench twin {os.path.basename(BLASLT_LIB)})')
    return KERNEL_LIB


SANITIZERS = {'asan': ['-fsanitize=address,undefined', '-fno-omit-frame-pointer', '-fno-sanitize-recover=all'],
              'tsan': ['-fsanitize=thread']}


def _link_atomic(cmd, out, srcs):
    """Build into a private temp name, then rename over ``out``: a process that is running
    (or loading) the old file keeps its inode, so concurrent test workers never see a
    half-written binary ("Text file busy" / truncated ELF)."""
    tmp = f'{out}.tmp{os.getpid()}'
    try:
        _run(cmd + [tmp] + srcs)
        os.replace(tmp, out)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)


def build_broker(verbose=False, sanitize=None):
    """The C++ broker daemon; ``sanitize='asan'`` (AddressSanitizer + UBSan, any report
    aborts) or ``'tsan'`` builds an instrumented twin ``mlcomp-broker-<san>`` for the
    sanitizer tests; host code only."""
    os.makedirs(OUT, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(ROOT, 'csrc', 'broker', '*.cpp')))
    hdrs = glob.glob(os.path.join(ROOT, 'csrc', 'broker', '*.h'))
    if not srcs:
        return None
    out = BROKER_BIN if not sanitize else f'{BROKER_BIN}-{sanitize}'
    if _newer(out, srcs + hdrs):
        cxx = shutil.which('g++') or 'c++'
        flags = ['-O2'] if not sanitize else ['-O1', '-g'] + SANITIZERS[sanitize]
        _link_atomic([cxx] + flags + ['-std=c++17', '-pthread', '-Wall', '-o'], out, srcs)
    if verbose:
        print(f'[build] broker -> {out}')
    return out


def _runtime_srcs():
    return sorted(s for s in glob.glob(os.path.join(ROOT, 'csrc', 'runtime', '*.cpp'))
                  if not s.endswith('_selftest.cpp'))


def build_runtime(verbose=False):
    os.makedirs(OUT, exist_ok=True)
    srcs = _runtime_srcs()
    hdrs = glob.glob(os.path.join(ROOT, 'csrc', 'runtime', '*.h'))
    if not srcs:
        return None
    if _newer(RUNTIME_LIB, srcs + hdrs):
        cxx = shutil.which('g++') or 'c++'
        _link_atomic([cxx, '-O3', '-std=c++17', '-pthread', '-fPIC', '-shared', '-Wall', '-o'], RUNTIME_LIB, srcs)
    if verbose:
        print(f'[build] runtime -> {RUNTIME_LIB}')
    return RUNTIME_LIB


def build_runtime_selftest(sanitize='tsan', verbose=False):
    """The record loader's self-test driver linked with an instrumented copy of the
    runtime sources (``tsan``: ThreadSanitizer, ``asan``: AddressSanitizer + UBSan)."""
    os.makedirs(OUT, exist_ok=True)
    main = os.path.join(ROOT, 'csrc', 'runtime', 'records_selftest.cpp')
    srcs = _runtime_srcs() + [main]
    out = os.path.join(OUT, f'mlcomp-records-selftest-{sanitize}')
    if _newer(out, srcs + glob.glob(os.path.join(ROOT, 'csrc', 'runtime', '*.h'))):
        cxx = shutil.which('g++') or 'c++'
        _link_atomic([cxx, '-O1', '-g', '-std=c++17', '-pthread', '-Wall'] + SANITIZERS[sanitize] + ['-o'], out, srcs)
    if verbose:
        print(f'[build] runtime selftest -> {out}')
    return out


def build_all(verbose=True):
    build_kernels(verbose)
    build_broker(verbose)
    build_runtime(verbose)


if __name__ == '__main__':
    build_all(verbose=True)
    sys.exit(0)
