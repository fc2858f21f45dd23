"""The ctypes signatures in mlcomp_amd.ops._lib must match the C launchers exactly
(parsed from csrc/kernels/*.hip), and every launcher must be exported by the built .so."""
import glob
import os
import re

from mlcomp_amd.ops import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_TYPES = {'int': 'i32', 'long': 'i64', 'float': 'f32', 'uint32_t': 'u32'}


def _parse():
    decls = {}
    for f in glob.glob(os.path.join(ROOT, 'csrc', 'kernels', '*.hip')):
        src = open(f).read()
        for m in re.finditer(r'MLC_EXPORT\s+(?:int|long|void\*|void|const char\*)\s+(\w+)\s*\(([^)]*)\)', src):
            args = [a.strip() for a in m.group(2).replace('\n', ' ').split(',') if a.strip()]
            kinds = []
            for a in args:
                if '*' in a or a.startswith('hipStream_t') or a.startswith('void'):
                    kinds.append('vp')
                else:
                    kinds.append(_TYPES[a.split()[0]])
            decls[m.group(1)] = kinds
    return decls


def test_signatures_match():
    decls = _parse()
    names = {_lib.vp: 'vp', _lib.i32: 'i32', _lib.i64: 'i64', _lib.f32: 'f32', _lib.u32: 'u32'}
    assert set(decls) == set(_lib._SIGS), set(decls) ^ set(_lib._SIGS)
    for name, kinds in decls.items():
        got = [names[t] for t in _lib._SIGS[name]]
        assert got == kinds, (name, got, kinds)


def test_library_exports():
    from mlcomp_amd.build import build_kernels
    import ctypes
    path = build_kernels()
    lib = ctypes.CDLL(path)
    for name in _lib._SIGS:
        assert hasattr(lib, name), name


def test_det_copies_floor_matches_kernels():
    """mlc_set_deterministic raises ncopy to >= 32 (batchnorm.hip NSTAT); the Python side
    must size its partial-sum buffers with the same floor."""
    import subprocess
    import sys
    out = subprocess.run([sys.executable, '-c', 'from mlcomp_amd.ops import _lib, functional as F; '
                          'print(_lib.DET_COPIES, F.NSTAT)'],
                         env=dict(os.environ, MLC_DETERMINISTIC='1', MLC_DET_COPIES='8'),
                         capture_output=True, text=True, check=True)
    assert out.stdout.split() == ['32', '32'], out.stdout


def test_production_library_links_no_vendor_gemm():
    """libmlcomp_kernels.so needs RCCL and the HIP runtime, never hipBLASLt / rocBLAS /
    MIOpen (the library A/B path lives in the bench-only twin, csrc/bench/blaslt.hip)."""
    import shutil
    import subprocess
    from mlcomp_amd.build import BLASLT_LIB, build_kernels
    path = build_kernels()
    tool = shutil.which('readelf') or '/opt/rocm/lib/llvm/bin/llvm-readelf'
    needed = subprocess.run([tool, '-d', path], capture_output=True, text=True, check=True).stdout
    libs = [ln.split('[')[1].split(']')[0] for ln in needed.splitlines() if 'NEEDED' in ln]
    assert any('rccl' in n for n in libs), libs
    assert not [n for n in libs if any(v in n for v in ('blas', 'MIOpen', 'miopen'))], libs
    twin = subprocess.run([tool, '-d', BLASLT_LIB], capture_output=True, text=True, check=True).stdout
    assert 'hipblaslt' in twin
