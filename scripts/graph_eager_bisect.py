"""Where does the graph-replayed model of the graph-vs-eager reproducer go wrong?

Same setup as scripts/graph_eager_variants.py (EfficientNet-b0 eager on the NULL stream
beside a graph-replayed twin, MLC_WORK_STREAM=0).  After every step of both models the
grad and master arenas are cloned on the NULL stream (stream-ordered, no host sync), and
at the end the first step / slots where the twins disagree beyond bf16 noise are listed.

    MLC_WORK_STREAM=0 python scripts/graph_eager_bisect.py"""
import os
import sys

import torch

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [root, os.path.join(root, 'tests')]
from test_generic_gpu import _models, _no_stochastic  # noqa: E402
from mlcomp_amd.train.native_generic_step import NativeGenericStep  # noqa: E402

make, shape, ncls = _models()['efficientnet-b0']
torch.manual_seed(0)
ms = [_no_stochastic(make()) for _ in range(2)]
ms[1].load_state_dict(ms[0].state_dict())
x, y = torch.randn(*shape), torch.randint(0, ncls, (shape[0],))
steps = [NativeGenericStep(m, x, y, device='cuda', use_graph=g, optimizer='SGD', lr=0.02, momentum=0.9)
         for m, g in zip(ms, (False, True))]
snaps = ([], [])
for i in range(12):
    for k, s in enumerate(steps):
        s()
        ar = s.net.arena
        snaps[k].append({'loss': s._loss.clone(),
                         'grad': [a.grad.clone() for a in ar.arenas()],
                         'master': [a.master.clone() for a in ar.arenas()]})
torch.cuda.synchronize()
slots = [(ai, sl) for ai, a in enumerate(steps[1].net.arena.arenas()) for sl in a.slots]


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


for i in range(12):
    e, g = snaps[0][i], snaps[1][i]
    lo = (e['loss'].item(), g['loss'].item())
    gr = max(rel(g['grad'][j], e['grad'][j]) for j in range(len(e['grad'])))
    mr = max(rel(g['master'][j], e['master'][j]) for j in range(len(e['master'])))
    print(f'step {i}: loss eager {lo[0]:.5f} graph {lo[1]:.5f}  max arena rel diff grad {gr:.3e} master {mr:.3e}',
          flush=True)
    if gr > 0.2 or not torch.isfinite(g['grad'][0]).all():
        bad = []
        for ai, sl in slots:
            ge = e['grad'][ai][sl.offset:sl.offset + sl.numel]
            gg = g['grad'][ai][sl.offset:sl.offset + sl.numel]
            r = rel(gg, ge)
            if r > 0.2 or not torch.isfinite(gg).all():
                bad.append((sl.name, round(r, 3), bool(torch.isfinite(gg).all())))
        print(f'  {len(bad)} of {len(slots)} slots differ; first (backward order) / last:',
              sorted(bad, key=lambda b: b[0])[:6], flush=True)
        names = [sl.name for _, sl in slots]
        order = {n: k for k, n in enumerate(names)}
        bad.sort(key=lambda b: order[b[0]])
        print('  forward-order first bad:', bad[:5], ' last bad:', bad[-5:], flush=True)
        break
