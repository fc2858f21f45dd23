"""Does eager kernel traffic right after a graph replay corrupt the graph's kernels?

A graph of N small dependent kernels (y += i for i in 1..N: every node has its own scalar
argument) is replayed, and without any host sync the host immediately launches M eager
kernels with different arguments (z += 1e6).  After a final sync y must equal sum(1..N)
exactly (fp64); anything else means a graph node ran with the wrong arguments or out of
order.  Repeated R times, with and without a stream sync after the replay.
"""
import sys
import torch

N = int(sys.argv[1]) if len(sys.argv) > 1 else 900
M = int(sys.argv[2]) if len(sys.argv) > 2 else 600
R = int(sys.argv[3]) if len(sys.argv) > 3 else 40
ON = sys.argv[4] if len(sys.argv) > 4 else 'null'    # null: everything on the NULL stream; created
dev = torch.device('cuda')
if ON == 'created':
    torch.cuda.set_stream(torch.cuda.Stream())
y = torch.zeros(1 << 12, device=dev, dtype=torch.float64)
z = torch.zeros(1 << 12, device=dev, dtype=torch.float64)


def body():
    y.zero_()
    for i in range(1, N + 1):
        y.add_(float(i))


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
want = N * (N + 1) / 2
for mode in ('nosync', 'sync'):
    bad = 0
    for r in range(R):
        g.replay()
        if mode == 'sync':
            torch.cuda.current_stream().synchronize()
        for _ in range(M):
            z.add_(1e6)
        torch.cuda.synchronize()
        got = y.double()
        if not bool((got == want).all()):
            bad += 1
            if bad <= 3:
                print(f'  {mode} rep {r}: y[0]={float(got[0])} want {want} '
                      f'(wrong elements {int((got != want).sum())})', flush=True)
    print(f'stream={ON} mode={mode}: {bad} of {R} replays gave a wrong result (N={N} graph kernels, M={M} eager)',
          flush=True)
