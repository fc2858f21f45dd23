"""Snapshot the graph model's state before every step of the eager+graph loop; at the
first non-finite loss restore the snapshot and re-run that step (a) by graph replay and
(b) eagerly, then report which arena tensors went non-finite."""
import math
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
se, sg = [NativeGenericStep(m, x, y, device='cuda', use_graph=g, optimizer='SGD', lr=lr, momentum=0.9)
          for m, g in zip(ms, (False, True))]


def state(s):
    out = {}
    for a in s.net.arena.arenas():
        out[a.name + '.master'] = a.master
        if a.mirror is not None:
            out[a.name + '.mirror'] = a.mirror
        for k, v in a.state.items():
            out[f'{a.name}.{k}'] = v
    if s.bn_buffers is not None:
        out['bn'] = s.bn_buffers
    out['hyper'] = s.opt.hyper
    return out


def snap(s):
    return {k: v.clone() for k, v in state(s).items()}


def restore(s, sn):
    for k, v in state(s).items():
        v.copy_(sn[k])


def bad(s):
    r = {k: int((~torch.isfinite(v.float())).sum()) for k, v in state(s).items()}
    for a in s.net.arena.arenas():
        r[a.name + '.grad'] = int((~torch.isfinite(a.grad)).sum())
    return {k: v for k, v in r.items() if v}


le, lg = [], []
for i in range(30):
    se()
    le.append(se.last_loss())
    sn = snap(sg)
    steps0 = sg.opt.steps
    sg()
    lg.append(sg.last_loss())
    torch.cuda.synchronize()
    if not math.isfinite(lg[-1]):
        print('step', i + 1, 'graph loss', lg[-1], 'bad', bad(sg), flush=True)
        print('out finite', bool(torch.isfinite(sg.out).all()), flush=True)
        for trial in ('replay', 'replay', 'eager'):
            restore(sg, sn)
            sg.opt.steps = steps0
            sg.opt.prepare()
            if trial == 'replay':
                sg.graph.replay()
            else:
                sg._body()
            torch.cuda.synchronize()
            print(trial, 'loss', sg.last_loss(), 'bad', bad(sg), flush=True)
        break
print('eager', [round(v, 5) for v in le])
print('graph', [round(v, 5) for v in lg])
