"""The round-4 graph-vs-eager reproducer under environment variants (one subprocess each).

EfficientNet-b0 trained eagerly on the NULL stream beside a graph-replayed twin
(``MLC_WORK_STREAM=0``); prints the first non-finite step of each model per variant.

    python scripts/graph_eager_variants.py            # all variants
    python scripts/graph_eager_variants.py child ENV=VAL,...   (internal)"""
import math
import os
import subprocess
import sys

VARIANTS = [
    'MLC_WORK_STREAM=0',
    'MLC_WORK_STREAM=0,MLC_BLASLT=0',
    'MLC_WORK_STREAM=0,MLC_WGRAD_STREAM=0',
    'MLC_WORK_STREAM=0,SYNC=graph',
    'MLC_WORK_STREAM=0,SYNC=eager',
    'MLC_WORK_STREAM=0,EAGER_STREAM=1',
    'MLC_WORK_STREAM=1',
    'MLC_WORK_STREAM=0,EAGER_TORCH=1',
    'MLC_WORK_STREAM=0,GRAPH_STREAM=1',
]


def child(spec):
    env = dict(kv.split('=') for kv in spec.split(',') if kv)
    import torch
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
    sys.path[:0] = [root, os.path.join(root, 'tests')]
    from test_generic_gpu import _models, _no_stochastic
    from mlcomp_amd.train.native_generic_step import NativeGenericStep
    make, shape, ncls = _models()['efficientnet-b0']
    torch.manual_seed(0)
    ms = [_no_stochastic(make()) for _ in range(2)]
    ms[1].load_state_dict(ms[0].state_dict())
    x, y = torch.randn(*shape), torch.randint(0, ncls, (shape[0],))
    steps = [NativeGenericStep(m, x, y, device='cuda', use_graph=g, optimizer='SGD', lr=0.02, momentum=0.9)
             for m, g in zip(ms, (False, True))]
    if env.get('EAGER_TORCH'):          # the eager twin on stock PyTorch ops (MIOpen / hipBLASLt)
        tm = ms[0].cuda()
        topt = torch.optim.SGD(tm.parameters(), lr=0.02, momentum=0.9)
        xc, yc = x.cuda(), y.cuda()

        class TorchStep:
            _l = None

            def __call__(self):
                topt.zero_grad()
                with torch.autocast('cuda', dtype=torch.bfloat16):
                    out = tm(xc)
                loss = torch.nn.functional.cross_entropy(out.float(), yc)
                loss.backward()
                topt.step()
                self._l = loss.detach()

            def last_loss(self):
                return float(self._l.item())
        steps[0] = TorchStep()
    gs = torch.cuda.Stream() if env.get('GRAPH_STREAM') else None
    if gs is not None:                  # replay the graphed twin on a created stream
        inner = steps[1]

        class OnStream:
            graph = None

            def __call__(self):
                gs.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(gs):
                    inner()
                torch.cuda.current_stream().wait_stream(gs)

            def last_loss(self):
                return inner.last_loss()
        steps[1] = OnStream()
    es = torch.cuda.Stream() if env.get('EAGER_STREAM') else None
    bad = {0: None, 1: None}
    losses = ([], [])
    for i in range(30):
        for k, s in enumerate(steps):
            if k == 0 and es is not None:
                es.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(es):
                    s()
                torch.cuda.current_stream().wait_stream(es)
            else:
                s()
            if (env.get('SYNC') == 'graph' and k == 1) or (env.get('SYNC') == 'eager' and k == 0):
                torch.cuda.synchronize()
            v = s.last_loss()
            losses[k].append(v)
            if not math.isfinite(v) and bad[k] is None:
                bad[k] = i
        if bad[0] is not None and bad[1] is not None:
            break
    print(f'{spec:45s} first non-finite step: eager {bad[0]}, graph {bad[1]}; '
          f'loss[0..3] eager {[round(v, 4) for v in losses[0][:4]]} graph {[round(v, 4) for v in losses[1][:4]]}',
          flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == 'child':
        child(sys.argv[2])
        return 0
    rc = 0
    for spec in VARIANTS:
        env = dict(os.environ)
        env.update(kv.split('=') for kv in spec.split(',') if kv.startswith('MLC_'))
        r = subprocess.run([sys.executable, os.path.abspath(__file__), 'child', spec], env=env, timeout=300)
        rc = rc or r.returncode
        if r.returncode not in (0, 1):
            break    # a crash: stop here
    return rc


if __name__ == '__main__':
    sys.exit(main())
