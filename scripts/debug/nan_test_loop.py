"""The graph-vs-eager test loop verbatim (efficientnet-b0, lr from argv), NaN step report."""
import math
import sys
import torch
sys.path[:0] = ['.', 'tests']
from test_generic_gpu import _models, _no_stochastic  # noqa: E402
from mlcomp_amd.train.native_generic_step import NativeGenericStep  # noqa: E402

name, lr = sys.argv[1], float(sys.argv[2])
if 'setstream' in (sys.argv[4] if len(sys.argv) > 4 else ''):
    torch.cuda.set_stream(torch.cuda.Stream())   # nothing runs on the NULL stream
if 'fill' in (sys.argv[4] if len(sys.argv) > 4 else ''):
    # torch.empty -> NaN: a kernel that reads memory nothing wrote shows up at once
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.utils.deterministic.fill_uninitialized_memory = True
which = sys.argv[3] if len(sys.argv) > 3 else 'eg'   # e, g, eg
make, shape, ncls = _models()[name]
torch.manual_seed(0)
ms = [_no_stochastic(make()) for _ in range(2)]
ms[1].load_state_dict(ms[0].state_dict())
x, y = torch.randn(*shape), torch.randint(0, ncls, (shape[0],))
opt = sys.argv[4] if len(sys.argv) > 4 else ''
xs, ys = [x, x], [y, y]
for o in opt.split(','):
    if o.startswith('other='):   # a different model as the eager one
        mk2, sh2, nc2 = _models()[o[6:]]
        ms[0] = _no_stochastic(mk2())
        xs[0], ys[0] = torch.randn(*sh2), torch.randint(0, nc2, (sh2[0],))
if which in ('ee', 'gg'):   # two models, both eager / both graphed
    steps = [NativeGenericStep(m, xx, yy, device='cuda', use_graph=which[0] == 'g', optimizer='SGD', lr=lr,
                               momentum=0.9) for m, xx, yy in zip(ms, xs, ys)]
else:
    steps = [NativeGenericStep(m, xx, yy, device='cuda', use_graph=g, optimizer='SGD', lr=lr, momentum=0.9)
             if k in which else None for m, xx, yy, g, k in zip(ms, xs, ys, (False, True), 'eg')]
from mlcomp_amd.ops import functional as Fn  # noqa: E402
from mlcomp_amd.ops import transformer as Tr  # noqa: E402
if 'pregrow' in opt:
    Fn.slab_workspace(torch.device('cuda:0'), 64 << 20)
    Tr.gemm_workspace(torch.device('cuda:0'), 64 << 20)
cur = {'tag': 0}
if 'separate' in opt:
    orig_key = Fn.workspace_key
    Fn.workspace_key = lambda d: f"{orig_key(d)}#{cur['tag']}"
if 'watch' in opt:   # tensors handed to native kernels during capture that die afterwards
    import weakref
    from mlcomp_amd.ops import _lib
    seen = {}
    orig_ptr = _lib.ptr

    def ptr(t):
        if t is not None and torch.cuda.is_current_stream_capturing():
            import traceback
            seen[id(t)] = (weakref.ref(t), t.data_ptr(), tuple(t.shape), t.dtype,
                           ''.join(traceback.format_stack(limit=4)[:-1]))
        return orig_ptr(t)
    _lib.ptr = ptr
if 'free' in opt:   # pointers the captured kernels use that lie in FREE allocator blocks
    import traceback
    from mlcomp_amd.ops import _lib
    rec = []
    orig_ptr2 = _lib.ptr

    def ptr2(t):
        if t is not None and torch.cuda.is_current_stream_capturing():
            rec.append((t.data_ptr(), t.numel() * t.element_size(), tuple(t.shape), t.dtype,
                        ''.join(traceback.format_stack(limit=6)[:-1])))
        return orig_ptr2(t)
    _lib.ptr = ptr2
    # every tensor an aten op reads or writes during the capture, too
    from torch.utils._python_dispatch import TorchDispatchMode
    from torch.utils._pytree import tree_leaves
    from mlcomp_amd.train.graphed import GraphedStep

    class Rec(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            for t in tree_leaves((args, kwargs, out)):
                if isinstance(t, torch.Tensor) and t.is_cuda and torch.cuda.is_current_stream_capturing():
                    st = t.untyped_storage()
                    rec.append((st.data_ptr(), st.nbytes(), tuple(t.shape), t.dtype, str(func)))
            return out
    orig_cap = GraphedStep._capture

    def cap(self):
        with Rec():
            return orig_cap(self)
    GraphedStep._capture = cap
if 'dump' in opt:
    torch.cuda.graphs.CUDAGraph  # noqa
    import mlcomp_amd.train.graphed as _gd
    _oc = _gd.GraphedStep._capture

    def _cap(self):
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        g.enable_debug_mode()
        with torch.cuda.graph(g):
            self._body()
        torch.cuda.synchronize(self.device)
        return g
    _gd.GraphedStep._capture = _cap
junk = []
le, lg = [], []
for i in range(30):
    for k, (s, out) in enumerate(zip(steps, (le, lg))):
        if s is not None:
            cur['tag'] = k
            if 'estream' in opt and k == 0:
                if 'st2' not in cur:
                    cur['st2'] = torch.cuda.Stream()
                cur['st2'].wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(cur['st2']):
                    s()
                torch.cuda.current_stream().wait_stream(cur['st2'])
            else:
                s()
            if 'tiny' in opt and k == 1:
                torch.ones(1, device='cuda').add_(1)
            out.append(s.last_loss())
            if 'sync' in opt and (('syncg' not in opt and 'synce' not in opt) or
                                  ('syncg' in opt and k == 1) or ('synce' in opt and k == 0)):
                torch.cuda.synchronize()
            if 'sleep' in opt and k == 1:
                import time
                time.sleep(0.2)
            if 'ssync' in opt and k == 1:
                torch.cuda.current_stream().synchronize()
            if 'esync' in opt and k == 1:
                ev = torch.cuda.Event()
                ev.record()
                ev.synchronize()
            if 'dump' in opt and k == 1 and i == 2:
                s.graph.debug_dump('gpurun_out/graph.dot')
    if 'watch' in opt and i == 3:
        import gc
        gc.collect()
        dead = [v for v in seen.values() if v[0]() is None]
        print('watched', len(seen), 'dead after capture', len(dead))
        for v in dead[:20]:
            print(hex(v[1]), v[2], v[3], v[4])
    if 'free' in opt and i == 3:
        import gc
        gc.collect()
        snap = torch.cuda.memory._snapshot()
        blocks = []
        for seg in snap['segments']:
            a = seg['address']
            for b in seg['blocks']:
                blocks.append((a, a + b['size'], b['state'], tuple(seg.get('segment_pool_id', (0, 0)))))
                a += b['size']
        blocks.sort()
        import bisect
        starts = [b[0] for b in blocks]
        nbad = 0
        for p, nb, shp, dt, stk in rec:
            k = bisect.bisect_right(starts, p) - 1
            if k < 0 or p >= blocks[k][1]:
                print('UNMAPPED', hex(p), shp, dt, stk); nbad += 1
                continue
            b = blocks[k]
            if (b[2] != 'active_allocated' and b[3] == (0, 0)) or p + nb > b[1]:
                print('FREE/OVERRUN', b[2], b[3], hex(p), nb, hex(b[0]), hex(b[1]), shp, dt, stk)
                nbad += 1
        print('captured pointers', len(rec), 'bad', nbad, flush=True)
    if 'junk' in opt:
        junk = [torch.full((n,), float('nan'), device='cuda') for n in (1 << 10, 1 << 14, 1 << 18, 1 << 20, 1 << 22)]
        junk = None
    if not all(math.isfinite(v[-1]) for v in (le, lg) if v):
        break
print('eager', [round(v, 5) for v in le])
print('graph', [round(v, 5) for v in lg])
