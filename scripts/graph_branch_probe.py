"""Do the parallel branches of a captured HIP graph run concurrently on this ROCm?
Two 1-thread spin kernels (torch.cuda._sleep) on a compute stream and a side stream, forked
and joined with events exactly like the gradient bucketer does; eager vs graph replay.
concurrent ~= 1x one kernel, serialised ~= 2x."""
import time

import torch

CYC = 20_000_000   # ~10 ms at ~2 GHz


def body(side):
    cur = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(cur)
    side.wait_event(ev)
    with torch.cuda.stream(side):
        torch.cuda._sleep(CYC)
    torch.cuda._sleep(CYC)
    ev2 = torch.cuda.Event()
    ev2.record(side)
    cur.wait_event(ev2)


def timed(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


side = torch.cuda.Stream()
one = timed(lambda: torch.cuda._sleep(CYC))
eager = timed(lambda: body(side))
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body(side)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body(side)
graph = timed(g.replay)
print(f'one kernel {one:.2f} ms | eager fork/join {eager:.2f} ms ({eager / one:.2f}x) | '
      f'graph replay {graph:.2f} ms ({graph / one:.2f}x)', flush=True)
