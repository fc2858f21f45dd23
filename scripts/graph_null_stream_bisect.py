"""Bounded bisection of the graph-replay corruption next to NULL-stream eager work
(round-5 verdict item 8; profiles/round5/graph_null_stream.md).  NO mlcomp_amd code: two
stock-PyTorch twins of a small model, the graphed twin's whole training step captured with
``torch.cuda.graph`` after a side-stream warm-up, the eager twin trained on the NULL stream
after every replay.  Prints one JSON line: first non-finite step of each twin, and whether
the graphed twin's loss sequence equals an eager reference run of the same model (a
corruption that stays finite shows up there).

    python scripts/graph_null_stream_bisect.py MODEL MODE

MODEL: mlp (Linear+ReLU: hipBLASLt GEMMs + elementwise), conv (Conv2d+ReLU, no BN: MIOpen
convolutions), bn (Conv2d+BatchNorm2d+ReLU: MIOpen BN), dw (a depthwise conv between BNs),
silu (conv+BN+SiLU), se (a squeeze-excitation gate), effnet (EfficientNet-b0 from the
generic-engine test models).
MODE: null (baseline), estream (eager twin on a created stream), sharedpool (the capture
shares a pool handle made up front), nocache (run under PYTORCH_NO_HIP_MEMORY_CACHING=1, set
by the caller), noeager (no eager twin at all: the graph alone), evalnull (the eager twin
runs forward only, no_grad, on the NULL stream), nomiopen / nomiopen_eval (null / evalnull
with MIOpen disabled: torch.backends.cudnn.enabled = False, PyTorch's own conv kernels)."""
import json
import math
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [root, os.path.join(root, 'tests')]

name = sys.argv[1] if len(sys.argv) > 1 else 'mlp'
mode = sys.argv[2] if len(sys.argv) > 2 else 'null'
if mode.startswith('nomiopen'):
    torch.backends.cudnn.enabled = False
    mode = 'null' if mode == 'nomiopen' else 'evalnull'
    tag = 'nomiopen'
else:
    tag = ''
STEPS = 20


def make():
    if name == 'mlp':
        return nn.Sequential(nn.Flatten(), nn.Linear(3 * 32 * 32, 1024), nn.ReLU(), nn.Linear(1024, 1024), nn.ReLU(),
                             nn.Linear(1024, 10))
    if name == 'conv':
        return nn.Sequential(nn.Conv2d(3, 64, 3, 1, 1), nn.ReLU(), nn.Conv2d(64, 64, 3, 2, 1), nn.ReLU(),
                             nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(64, 10))
    if name == 'bn':
        return nn.Sequential(nn.Conv2d(3, 64, 3, 1, 1), nn.BatchNorm2d(64), nn.ReLU(), nn.Conv2d(64, 64, 3, 2, 1),
                             nn.BatchNorm2d(64), nn.ReLU(), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(64, 10))
    if name == 'dw':        # depthwise conv + BN + ReLU (EfficientNet's MBConv core, MIOpen grouped conv)
        return nn.Sequential(nn.Conv2d(3, 64, 3, 1, 1), nn.BatchNorm2d(64), nn.ReLU(),
                             nn.Conv2d(64, 64, 3, 1, 1, groups=64), nn.BatchNorm2d(64), nn.ReLU(),
                             nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(64, 10))
    if name == 'silu':      # the same without the depthwise conv, SiLU activations
        return nn.Sequential(nn.Conv2d(3, 64, 3, 1, 1), nn.BatchNorm2d(64), nn.SiLU(), nn.Conv2d(64, 64, 3, 1, 1),
                             nn.BatchNorm2d(64), nn.SiLU(), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(64, 10))
    if name == 'se':        # a squeeze-excitation gate (global pool, 1x1 convs, sigmoid, multiply)
        class SE(nn.Module):
            def __init__(self):
                super().__init__()
                self.c = nn.Sequential(nn.Conv2d(3, 64, 3, 1, 1), nn.BatchNorm2d(64), nn.ReLU())
                self.g = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(64, 16, 1), nn.ReLU(), nn.Conv2d(16, 64, 1),
                                       nn.Sigmoid())
                self.h = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(64, 10))

            def forward(self, x):
                y = self.c(x)
                return self.h(y * self.g(y))
        return SE()
    from test_generic_gpu import _models, _no_stochastic
    mk, _, _ = _models()['efficientnet-b0']
    return _no_stochastic(mk())


torch.manual_seed(0)
ms = [make().cuda().to(memory_format=torch.channels_last) for _ in range(3)]
ms[1].load_state_dict(ms[0].state_dict())
ms[2].load_state_dict(ms[0].state_dict())
x = torch.randn(64, 3, 32 if name != 'effnet' else 64, 32 if name != 'effnet' else 64, device='cuda')
x = x.contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (64,), device='cuda')
opts = [torch.optim.SGD(m.parameters(), lr=0.02, momentum=0.9) for m in ms]
loss_buf = [None, None, None]


def body(k, train=True):
    if not train:
        with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False):
            ms[k](x)
        return
    opts[k].zero_grad(set_to_none=False)
    with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False):
        out = ms[k](x)
    loss = F.cross_entropy(out.float(), y)
    loss.backward()
    opts[k].step()
    loss_buf[k] = loss.detach()


# eager reference of the graphed twin's trajectory (same start, run first, side stream)
ref = []
s0 = torch.cuda.Stream()
with torch.cuda.stream(s0):
    for i in range(3 + STEPS):
        body(2)
        ref.append(loss_buf[2])
        print(f'reference step {i}', file=sys.stderr, flush=True)   # progress (slow without MIOpen)
torch.cuda.synchronize()
ref = [float(v.item()) for v in ref][3:]

s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        body(1)
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
pool = torch.cuda.graph_pool_handle() if mode == 'sharedpool' else None
try:
    with torch.cuda.graph(g, pool=pool):
        body(1)
    torch.cuda.synchronize()
except Exception as e:        # e.g. PYTORCH_NO_HIP_MEMORY_CACHING=1: hipMalloc inside the capture
    print(json.dumps({'model': name, 'mode': mode + (f'+{tag}' if tag else ''), 'nocache_env': os.environ.get('PYTORCH_NO_HIP_MEMORY_CACHING'),
                      'capture_error': str(e).splitlines()[0][:160]}), flush=True)
    sys.exit(0)
es = torch.cuda.Stream() if mode == 'estream' else None
bad = [None, None]
losses = ([], [])
for i in range(STEPS):
    if mode != 'noeager':
        if es is not None:
            es.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(es):
                body(0)
            torch.cuda.current_stream().wait_stream(es)
        else:
            body(0, train=mode != 'evalnull')
        if mode != 'evalnull':
            losses[0].append(float(loss_buf[0].item()))
    g.replay()
    losses[1].append(float(loss_buf[1].item()))
    print(f'step {i}: graph loss {losses[1][-1]:.4f}', file=sys.stderr, flush=True)   # progress
    for k in range(2):
        if bad[k] is None and losses[k] and not math.isfinite(losses[k][-1]):
            bad[k] = i
dev = max(abs(a - b) / max(abs(b), 1e-6) for a, b in zip(losses[1], ref))
print(json.dumps({'model': name, 'mode': mode + (f'+{tag}' if tag else ''), 'nocache_env': os.environ.get('PYTORCH_NO_HIP_MEMORY_CACHING'),
                  'first_nonfinite_eager': bad[0], 'first_nonfinite_graph': bad[1],
                  'graph_vs_eager_ref_max_rel': round(dev, 5),
                  'graph_losses': [round(v, 4) for v in losses[1][:8]], 'ref_losses': [round(v, 4) for v in ref[:8]]}),
      flush=True)
