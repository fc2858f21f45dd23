"""Is work launched on a stream after a HIP graph replay ordered after the WHOLE graph?

The graph: a long chain of matmuls (tens of ms), then `flag.fill_(k)` as its last node
(k = the replay counter, read from a device tensor).  After each replay the host launches an
eager copy of `flag` (no sync in between); a late value in the copies means the eager
kernel ran before the graph finished.  Variants put an `.item()` of an early graph tensor
between the replay and the eager copy (the pattern of a training loop logging its loss).
"""
import sys
import torch

dev = torch.device('cuda')
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
a = torch.randn(2048, 2048, device=dev)
b = torch.randn(2048, 2048, device=dev)
counter = torch.zeros(1, device=dev)
flag = torch.zeros(1, device=dev)
early = torch.zeros(1, device=dev)


def body():
    early.copy_(counter)               # an early node (read back by .item())
    c = a
    for _ in range(n):
        c = torch.tanh(c @ b) * 0.5
    flag.copy_(counter + (c[0, 0] * 0))   # the last node depends on the whole chain


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body()
torch.cuda.synchronize()
for mode in ('none', 'item'):
    seen = torch.zeros(50, device=dev)
    for k in range(50):
        counter.fill_(k + 1)
        g.replay()
        if mode == 'item':
            float(early.item())
        seen[k].copy_(flag[0])          # eager kernel right after the replay
    torch.cuda.synchronize()
    late = int((seen != torch.arange(1, 51, device=dev, dtype=torch.float32)).sum())
    print(f'mode={mode}: {late} of 50 eager copies saw a stale flag', flush=True)
