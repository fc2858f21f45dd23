"""Two generic steps in one process (as the graph-vs-eager test): which combination makes
the graph-replayed one produce non-finite gradients?"""
import sys
import torch
sys.path[:0] = ['.', 'tests']
from test_generic_gpu import _models, _no_stochastic  # noqa: E402
from mlcomp_amd.train.native_generic_step import NativeGenericStep  # noqa: E402

name, lr, mode = sys.argv[1], float(sys.argv[2]), sys.argv[3]
make, shape, ncls = _models()[name]
torch.manual_seed(0)
ms = [_no_stochastic(make()) for _ in range(2)]
ms[1].load_state_dict(ms[0].state_dict())
x, y = torch.randn(*shape), torch.randint(0, ncls, (shape[0],))
graphs = {'eg': (False, True), 'ge': (True, False), 'gg': (True, True)}[mode]
st = [NativeGenericStep(m, x, y, device='cuda', use_graph=g, optimizer='SGD', lr=lr, momentum=0.9)
      for m, g in zip(ms, graphs)]
for i in range(int(sys.argv[4]) if len(sys.argv) > 4 else 10):
    for k, s in enumerate(st):
        s()
        torch.cuda.synchronize()
        bad = [n for n, sl in s.net.arena.by_name.items() if not torch.isfinite(sl.grad).all()]
        if bad:
            print(f'{mode} step {i} model {k} (graph={graphs[k]}): {len(bad)} non-finite grads, last {bad[-4:]}')
            sys.exit(0)
    print(f'{mode} step {i} losses {[round(s.last_loss(), 5) for s in st]}', flush=True)
