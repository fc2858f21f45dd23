"""Node kinds and topology of the generic engine's captured step graph (hipGraphGetNodes /
hipGraphGetEdges on the raw graph), to see whether the capture is one linear chain."""
import collections
import ctypes as C
import sys
import torch
sys.path[:0] = ['.', 'tests']
from test_generic_gpu import _models, _no_stochastic  # noqa: E402
import mlcomp_amd.train.graphed as gd  # noqa: E402
from mlcomp_amd.train.native_generic_step import NativeGenericStep  # noqa: E402

hip = C.CDLL('libamdhip64.so')
KIND = {0: 'kernel', 1: 'memcpy', 2: 'memset', 3: 'host', 4: 'graph', 5: 'empty', 6: 'wait_event',
        7: 'event_record', 10: 'mem_alloc', 11: 'mem_free'}
kept = {}


def _cap(self):
    torch.cuda.synchronize(self.device)
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        self._body()
    g.instantiate()
    torch.cuda.synchronize(self.device)
    kept['g'] = g
    return g


gd.GraphedStep._capture = _cap
name = sys.argv[1] if len(sys.argv) > 1 else 'efficientnet-b0'
make, shape, ncls = _models()[name]
torch.manual_seed(0)
m = _no_stochastic(make())
x, y = torch.randn(*shape), torch.randint(0, ncls, (shape[0],))
s = NativeGenericStep(m, x, y, device='cuda', optimizer='SGD', lr=0.02, momentum=0.9)
for _ in range(3):
    s()
torch.cuda.synchronize()
graph = C.c_void_p(kept['g'].raw_cuda_graph())
n = C.c_size_t(0)
assert hip.hipGraphGetNodes(graph, None, C.byref(n)) == 0
nodes = (C.c_void_p * n.value)()
assert hip.hipGraphGetNodes(graph, nodes, C.byref(n)) == 0
kinds = collections.Counter()
kind_of = {}
for nd in nodes:
    t = C.c_int(-1)
    hip.hipGraphNodeGetType(C.c_void_p(nd), C.byref(t))
    kinds[KIND.get(t.value, t.value)] += 1
    kind_of[nd] = KIND.get(t.value, t.value)
e = C.c_size_t(0)
assert hip.hipGraphGetEdges(graph, None, None, C.byref(e)) == 0
fr, to = (C.c_void_p * e.value)(), (C.c_void_p * e.value)()
assert hip.hipGraphGetEdges(graph, fr, to, C.byref(e)) == 0
indeg, outdeg = collections.Counter(), collections.Counter()
for a, b in zip(fr, to):
    outdeg[a] += 1
    indeg[b] += 1
print('nodes', n.value, 'edges', e.value, dict(kinds))
roots = [nd for nd in nodes if indeg[nd] == 0]
leaves = [nd for nd in nodes if outdeg[nd] == 0]
print('roots', len(roots), [kind_of[r] for r in roots][:10])
print('leaves', len(leaves), [kind_of[r] for r in leaves][:10])
fo = [nd for nd in nodes if outdeg[nd] > 1]
fi = [nd for nd in nodes if indeg[nd] > 1]
print('fan-out>1', len(fo), collections.Counter(kind_of[x] for x in fo))
print('fan-in>1', len(fi), collections.Counter(kind_of[x] for x in fi))


# chain order and the memset nodes' targets
class MemsetParams(C.Structure):
    _fields_ = [('dst', C.c_void_p), ('elementSize', C.c_uint), ('height', C.c_size_t), ('pitch', C.c_size_t),
                ('value', C.c_uint), ('width', C.c_size_t)]


nxt = {a: b for a, b in zip(fr, to)}
order, cur = [], roots[0]
while cur is not None:
    order.append(cur)
    cur = nxt.get(cur)
known = {'ctx.ws': s.net.ctx.ws.buf if hasattr(s.net.ctx.ws, 'buf') else None}
for a in s.net.arena.arenas():
    known[a.name + '.grad'] = a.grad
    known[a.name + '.master'] = a.master
known['x'] = s.x
for i, nd in enumerate(order):
    if kind_of[nd] == 'memset':
        p = MemsetParams()
        rc = hip.hipGraphMemsetNodeGetParams(C.c_void_p(nd), C.byref(p))
        hit = [k for k, t in known.items() if t is not None and t.data_ptr() <= (p.dst or 0) < t.data_ptr() + t.numel() * t.element_size()]
        print('memset node at chain position', i, 'rc', rc, 'dst', hex(p.dst or 0), 'elem', p.elementSize,
              'width', p.width, 'height', p.height, 'value', p.value, 'target', hit)
print('ws attrs', [a for a in dir(s.net.ctx.ws) if not a.startswith('__')][:20])
