"""Does a replayed multi-branch HIP graph stay ordered with eager work on the same stream?

Pure PyTorch, no mlcomp_amd kernels.  The graph has the shape of a captured training step:
a main branch and a branch forked onto a second stream inside the capture, joined back
before the end.  Each check writes a marker tensor ``x`` from both sides with a long
``torch.cuda._sleep`` in front of the earlier writer, so a missing dependency shows up as
the wrong final value:

  after  - graph (forked branch: sleep, x = 1), then eager x = 2 on the launch stream:
           x must end 2; 1 means the eager kernel ran before the graph's forked branch ended
  before - eager (sleep, x = 2) on the launch stream, then the graph (forked branch: x = 1
           at once): x must end 1; 2 means the forked branch started before the eager work
           that precedes the replay had finished
  root   - as 'before' but the graph's MAIN branch writes x = 1 at once

Each check runs with the replay launched on the NULL stream and on a created stream.

    python scripts/graph_null_stream_probe.py [reps]"""
import sys

import torch

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
SLEEP = 2_000_000   # cycles, ~1 ms


def build(kind):
    x = torch.zeros(1, device='cuda')
    y = torch.zeros(1, device='cuda')
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        side.wait_stream(cap)
        with torch.cuda.stream(side):
            if kind == 'after':
                torch.cuda._sleep(SLEEP)
                x.fill_(1.0)
            elif kind == 'before':
                x.fill_(1.0)
            else:
                y.add_(1.0)
        if kind == 'root':
            x.fill_(1.0)
        else:
            y.add_(1.0)
        cap.wait_stream(side)
    return g, x


def check(kind, stream):
    g, x = build(kind)
    torch.cuda.synchronize()
    bad = 0
    with torch.cuda.stream(stream):
        for _ in range(REPS):
            x.zero_()
            torch.cuda.synchronize()
            if kind == 'after':
                g.replay()
                x.fill_(2.0)
                want = 2.0
            else:
                torch.cuda._sleep(SLEEP)
                x.fill_(2.0)
                g.replay()
                want = 1.0
            torch.cuda.synchronize()
            bad += int(float(x.item()) != want)
    return bad


def main():
    created = torch.cuda.Stream()
    null = torch.cuda.default_stream()
    print(f'null stream handle {null.cuda_stream}, created {created.cuda_stream}')
    for kind in ('after', 'before', 'root'):
        for name, st in (('NULL', null), ('created', created)):
            bad = check(kind, st)
            print(f'{kind:6s} replay on {name:7s}: {bad} of {REPS} out of order', flush=True)


if __name__ == '__main__':
    main()
