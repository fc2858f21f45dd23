"""Out-of-bounds write detector for the native kernels: every CUDA tensor created through
torch.empty / empty_like / zeros / zeros_like (Python level) is carved out of a larger
buffer with sentinel-filled guard zones on both sides; after every native call the guards
of all live tensors are checked.  The first call that changes a guard is reported with
the guarded tensor's shape and the stack that allocated it.

    python scripts/debug/oob_guard.py efficientnet-b0 [steps]
"""
import math
import sys
import traceback
import weakref

import torch

sys.path[:0] = ['.', 'tests']
G = 2048   # guard elements per side
SENT = {torch.float32: -7777.0, torch.bfloat16: -7776.0, torch.float16: -7776.0, torch.int64: -7777,
        torch.int32: -7777, torch.uint8: 77, torch.int8: -77, torch.bool: None}
_empty, _empty_like, _zeros, _zeros_like = torch.empty, torch.empty_like, torch.zeros, torch.zeros_like
live = []


def _shape(size):
    if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)):
        return tuple(size[0])
    return tuple(size)


def _guarded(shape, dtype, device, zero, kw=None):
    kw = dict(kw or {})
    rg = kw.pop('requires_grad', False)
    if kw:
        return None
    dtype = dtype or torch.get_default_dtype()
    if SENT.get(dtype) is None:
        return None
    n = int(math.prod(shape)) if shape else 1
    base = _empty(n + 2 * G, dtype=dtype, device=device)
    base.fill_(SENT[dtype])
    t = base[G:G + n]
    if zero:
        t.zero_()
    t = t.view(shape)
    if rg:
        t.requires_grad_()
    live.append((weakref.ref(t), base[:G], base[G + n:], shape, dtype,
                 ''.join(traceback.format_stack(limit=7)[:-2])))
    return t


def _is_cuda(device):
    return device is not None and torch.device(device).type == 'cuda'


def empty(*size, dtype=None, device=None, **kw):
    if _is_cuda(device) and not kw.get('memory_format'):
        t = _guarded(_shape(size), dtype, device, False, kw)
        if t is not None:
            return t
    return _empty(*size, dtype=dtype, device=device, **kw)


def zeros(*size, dtype=None, device=None, **kw):
    if _is_cuda(device):
        t = _guarded(_shape(size), dtype, device, True, kw)
        if t is not None:
            return t
    return _zeros(*size, dtype=dtype, device=device, **kw)


def empty_like(x, dtype=None, device=None, **kw):
    dev = device or x.device
    if _is_cuda(dev) and x.is_contiguous() and not kw.get('memory_format'):
        t = _guarded(tuple(x.shape), dtype or x.dtype, dev, False, kw)
        if t is not None:
            return t
    return _empty_like(x, dtype=dtype, device=device, **kw)


def zeros_like(x, dtype=None, device=None, **kw):
    dev = device or x.device
    if _is_cuda(dev) and x.is_contiguous() and not kw.get('memory_format'):
        t = _guarded(tuple(x.shape), dtype or x.dtype, dev, True, kw)
        if t is not None:
            return t
    return _zeros_like(x, dtype=dtype, device=device, **kw)


torch.empty, torch.zeros, torch.empty_like, torch.zeros_like = empty, zeros, empty_like, zeros_like

from mlcomp_amd.ops import _lib  # noqa: E402

_call = _lib.call
ncalls = [0]


def check(where):
    torch.cuda.synchronize()
    alive = [e for e in live if e[0]() is not None]
    live[:] = alive
    by = {}
    for e in alive:
        by.setdefault(e[4], []).append(e)
    for dt, es in by.items():
        s = SENT[dt]
        bad = torch.cat([torch.cat([e[1], e[2]]) for e in es]) != s
        if bool(bad.any()):
            for e in es:
                if bool((e[1] != s).any()) or bool((e[2] != s).any()):
                    lo = int((e[1] != s).sum())
                    hi = int((e[2] != s).sum())
                    print(f'GUARD HIT after {where}: tensor {e[3]} {e[4]} lo={lo} hi={hi}\n{e[5]}', flush=True)
                    return True
    return False


def call(name, *args):
    rc = _call(name, *args)
    ncalls[0] += 1
    if check(f'{name} (native call #{ncalls[0]})'):
        traceback.print_stack(limit=8)
        sys.exit(3)
    return rc


_lib.call = call

from test_generic_gpu import _models, _no_stochastic  # noqa: E402
from mlcomp_amd.train.native_generic_step import NativeGenericStep  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'efficientnet-b0'
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
make, shape, ncls = _models()[name]
torch.manual_seed(0)
m = _no_stochastic(make())
x, y = torch.randn(*shape), torch.randint(0, ncls, (shape[0],))
s = NativeGenericStep(m, x, y, device='cuda', use_graph=False, optimizer='SGD', lr=0.02, momentum=0.9)
for i in range(steps):
    s()
    print('step', i + 1, 'loss', s.last_loss(), 'native calls', ncalls[0], 'guarded', len(live), flush=True)
print('no guard hit')
