"""Graph-vs-eager twins with NO mlcomp_amd code: stock PyTorch EfficientNet-b0 training steps.

The graphed twin's whole step (bf16 autocast forward, loss, backward, SGD momentum) is
captured with ``torch.cuda.graph`` (after warm-up on a side stream, as the PyTorch docs
prescribe) and replayed on the NULL stream; the eager twin trains on the NULL stream right
after every replay.  Prints the first non-finite step of each.  If the graphed twin goes
NaN here too, the corruption of round 4 is a property of the runtime (graph replay followed
by NULL-stream work), not of the framework's kernels.

    python scripts/graph_torch_twin.py [model] [mode]

mode: '' (replay and eager work on the NULL stream), 'sync' (device sync after each
replay), 'estream' (the eager twin on a created stream), 'gstream' (the replay on a created
stream, fenced to the NULL stream on both sides)."""
import math
import os
import sys

import torch
import torch.nn.functional as F

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [root, os.path.join(root, 'tests')]
from test_generic_gpu import _models, _no_stochastic  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'efficientnet-b0'
mode = sys.argv[2] if len(sys.argv) > 2 else ''
sync = mode == 'sync'
es = torch.cuda.Stream() if mode == 'estream' else None
gs = torch.cuda.Stream() if mode == 'gstream' else None
make, shape, ncls = _models()[name]
torch.manual_seed(0)
ms = [_no_stochastic(make()).cuda() for _ in range(2)]
ms[1].load_state_dict(ms[0].state_dict())
x = torch.randn(*shape, device='cuda')
y = torch.randint(0, ncls, (shape[0],), device='cuda')
opts = [torch.optim.SGD(m.parameters(), lr=0.02, momentum=0.9) for m in ms]
loss_buf = [None, None]


def body(k):
    opts[k].zero_grad(set_to_none=False)
    with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False):
        out = ms[k](x)
    loss = F.cross_entropy(out.float(), y)
    loss.backward()
    opts[k].step()
    loss_buf[k] = loss.detach()


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        body(1)
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body(1)
torch.cuda.synchronize()
bad = [None, None]
losses = ([], [])
def on(stream, fn):
    if stream is None:
        fn()
        return
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        fn()
    torch.cuda.current_stream().wait_stream(stream)


for i in range(30):
    on(es, lambda: body(0))
    losses[0].append(float(loss_buf[0].item()))
    on(gs, g.replay)
    if sync:
        torch.cuda.synchronize()
    losses[1].append(float(loss_buf[1].item()))
    for k in range(2):
        if bad[k] is None and not math.isfinite(losses[k][-1]):
            bad[k] = i
print(f'{name} mode={mode or "null"}: first non-finite step eager {bad[0]}, graph {bad[1]}; '
      f'losses eager {[round(v, 4) for v in losses[0][:6]]} graph {[round(v, 4) for v in losses[1][:6]]}',
      flush=True)
