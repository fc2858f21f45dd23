"""Per-shape native / hipBLASLt selection for the dense GEMMs (csrc/bench/blaslt.hip), in the
BENCH-ONLY twin library libmlcomp_kernels_blaslt.so: both forced modes and the timed auto
mode match an fp32 reference for every form the models use (bias forward, residual-addend
input gradient, weight + bias gradient accumulated into fp32), and a HIP graph captured
after the eager warm-up replays the choice warm-up made.

The production library has no library path (dense_entry.hip): mlc_blaslt_mode refuses to
turn it on.  The twin is loaded through MLC_KERNEL_LIB, so when this module runs inside the
GPU suite (production library loaded) the library-path tests run in ONE child process."""
import ctypes
import os
import subprocess
import sys

import pytest
import torch

from mlcomp_amd.ops import _lib
from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.ops import transformer as Tx

pytestmark = pytest.mark.gpu
TWIN = os.environ.get('MLC_KERNEL_LIB', '').endswith('_blaslt.so')


def test_production_library_refuses_the_library_path():
    if TWIN:
        pytest.skip('running inside the twin-library child')
    assert _lib.load().mlc_blaslt_mode(1) == -1
    assert _lib.load().mlc_blaslt_mode(-1) == 0


def test_twin_library_selection_in_child():
    if TWIN:
        pytest.skip('already the child')
    from mlcomp_amd.build import BLASLT_LIB
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MLC_KERNEL_LIB=BLASLT_LIB, PYTHONPATH=root)
    r = subprocess.run([sys.executable, '-m', 'pytest', os.path.abspath(__file__), '-x', '-q', '-m', 'gpu',
                        '-p', 'no:cacheprovider'], env=env, cwd=root, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.fixture
def lib():
    if not TWIN:
        pytest.skip('library-path tests run in the twin-library child')
    lib = _lib.load()
    old = lib.mlc_blaslt_mode(-1)
    yield lib
    lib.mlc_blaslt_mode(old)


def _r(*s):
    return torch.rand(*s, device='cuda').sub(0.5).to(torch.bfloat16)


def _rel(a, b):
    return float((a.float() - b).abs().max() / b.abs().max())


@pytest.mark.parametrize('mode', [0, 1, 2])
@pytest.mark.parametrize('M,N,K', [(1024, 768, 768), (512, 2304, 768), (256, 768, 3072)])
def test_dense_forms_match_fp32(lib, mode, M, N, K):
    lib.mlc_blaslt_mode(mode)
    x, w, dy, add = _r(M, K), _r(N, K), _r(M, N), _r(M, K)
    b = torch.randn(N, device='cuda') * 0.1
    y, _ = Tx.dense_fwd(x, w, b)
    assert _rel(y, x.float() @ w.float().t() + b) < 1e-2
    dx = Tx.dense_dgrad(dy, w, addend=add)
    assert _rel(dx, dy.float() @ w.float() + add.float()) < 1e-2
    dw = torch.full((N, K), 0.5, device='cuda')
    db = torch.full((N,), 0.25, device='cuda')
    Fn.linear_wgrad_bias(dy, x, dw, db)
    assert _rel(dw, dy.float().t() @ x.float() + 0.5) < 1e-2
    assert _rel(db, dy.float().sum(0) + 0.25) < 1e-2


def test_auto_choices_are_recorded_and_graph_replays_them(lib):
    M, N, K = 4096, 2304, 768
    x, w = _r(M, K), _r(N, K)
    b = torch.randn(N, device='cuda') * 0.1
    lib.mlc_blaslt_mode(0)
    y_native = Tx.dense_fwd(x, w, b)[0].clone()
    lib.mlc_blaslt_mode(1)
    y_lib = Tx.dense_fwd(x, w, b)[0].clone()
    lib.mlc_blaslt_mode(2)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        y_auto = Tx.dense_fwd(x, w, b)[0].clone()        # eager: times both, caches the winner
    torch.cuda.synchronize()
    buf = (ctypes.c_int * 100)()
    n = lib.mlc_blaslt_choices(buf, 10)
    rows = [list(buf[10 * i:10 * i + 10]) for i in range(n)]
    row = [r for r in rows if r[:4] == [0, M, N, K]]
    assert row, rows
    pick = row[0][7]
    assert torch.equal(y_auto, y_lib if pick >= 0 else y_native)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y_g = Tx.dense_fwd(x, w, b)[0]
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y_g, y_auto)
    assert _rel(y_g, x.float() @ w.float().t() + b) < 1e-2
