"""Eager vs HIP-graph generic step, slot by slot: after each step, the relative difference of
every gradient slot between an eager and a graph-replayed NativeGenericStep on the same
batch (large differences localise an op that misbehaves under graph replay)."""
import sys
import torch
sys.path[:0] = ['.', 'tests']
from test_generic_gpu import _models, _no_stochastic  # noqa: E402
from mlcomp_amd.train.native_generic_step import NativeGenericStep  # noqa: E402

name, lr = sys.argv[1], float(sys.argv[2])
make, shape, ncls = _models()[name]
torch.manual_seed(0)
ms = [_no_stochastic(make()) for _ in range(2)]
ms[1].load_state_dict(ms[0].state_dict())
x, y = torch.randn(*shape), torch.randint(0, ncls, (shape[0],))
st = [NativeGenericStep(m, x, y, device='cuda', use_graph=g, optimizer='SGD', lr=lr, momentum=0.9)
      for m, g in zip(ms, (False, True))]
for i in range(6):
    for s in st:
        s()
    torch.cuda.synchronize()
    print(f'step {i}: loss eager {st[0].last_loss():.5f} graph {st[1].last_loss():.5f}', flush=True)
    worst = []
    for (n, a), b in zip(st[0].net.arena.by_name.items(), st[1].net.arena.by_name.values()):
        ga, gb = a.grad.float(), b.grad.float()
        r = ((ga - gb).norm() / (ga.norm() + 1e-20)).item()
        worst.append((r, n, ga.norm().item(), gb.norm().item()))
    worst.sort(reverse=True)
    for r, n, na, nb in worst[:6]:
        print(f'   {n:40s} rel {r:.4f}  |g| eager {na:.4g} graph {nb:.4g}')
