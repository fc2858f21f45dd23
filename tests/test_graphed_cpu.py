"""Host-side protocol of the native graphed steps (`mlcomp_amd/train/graphed.py`):
optimizer step counting lives in ``prepare()``, and a HIP-graph capture failure on one
rank makes EVERY rank fall back to eager execution (decided by one all-reduce), so the
collective sequence stays identical across ranks.  The capture machinery is replaced by
fakes so this runs on CPU over gloo."""
import contextlib
import os
import socket

import torch
import torch.multiprocessing as mp

from mlcomp_amd.ops.arena import ParamArena
from mlcomp_amd.train import graphed
from mlcomp_amd.train.optim import FusedAdam, FusedSGD


def _arena():
    pa = ParamArena()
    pa.weight('w', (4, 8))
    pa.vector('b', (4,))
    pa.finalize('cpu')
    pa.decay.master.normal_()
    pa.decay.grad.normal_()
    return pa


def test_adam_bias_correction_advances_in_prepare_only():
    """``step()`` (what a graph captures) must not own the counter: N prepare() calls give
    the bias corrections of step N whether or not step() ran in Python each time."""
    pa = _arena()
    opt = FusedAdam(pa, lr=1e-3)
    opt.prepare()
    opt.step()
    for _ in range(19):   # graph replays: host prepare() only
        opt.prepare()
    assert opt.steps == 20
    assert abs(float(opt.hyper[2]) - (1 - 0.9 ** 20)) < 1e-6
    assert abs(float(opt.hyper[3]) - (1 - 0.999 ** 20)) < 1e-6
    sgd = FusedSGD(pa, lr=0.1)
    sgd.prepare()
    sgd.step()
    sgd.step()
    assert sgd.steps == 1


class _FakeOpt:
    def __init__(self):
        self.steps = 0

    def prepare(self):
        self.steps += 1


class _FakeStep(graphed.GraphedStep):
    def __init__(self, comm, fail_capture):
        self.device = torch.device('cpu')
        self.comm = comm
        self.opt = _FakeOpt()
        self.use_graph = True
        self.warmup_eager = 0
        self.graph = None
        self.calls = 0
        self.fail_capture = fail_capture
        self.capturing = False
        self.eager_runs = 0
        self.w = torch.zeros(4)

    def _body(self):
        if self.capturing:
            return   # capture records work without running it
        self.eager_runs += 1
        g = torch.full((4,), float(self.comm.rank + 1))
        self.comm.all_reduce(g)   # the step's collective (bucketed all-reduce)
        self.w += g


class _FakeGraph:
    owner = None

    def replay(self):
        st = _FakeGraph.owner
        st.capturing = False
        st._body()


def _patch(step):
    @contextlib.contextmanager
    def fake_graph(g):
        step.capturing = True
        try:
            yield
        finally:
            step.capturing = False
        if step.fail_capture:
            raise RuntimeError('hipStreamEndCapture: operation not permitted when stream is capturing')
    _FakeGraph.owner = step
    graphed.torch.cuda.graph = fake_graph
    graphed.torch.cuda.CUDAGraph = _FakeGraph
    graphed.torch.cuda.synchronize = lambda *a, **k: None


def _worker(rank, world, port, out):
    import torch.distributed as dist
    from mlcomp_amd.parallel.comm import TorchComm
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    step = _FakeStep(TorchComm(rank, world), fail_capture=(rank == 1))
    _patch(step)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        for _ in range(5):
            step()
    torch.save({'w': step.w, 'graph': step.graph is not None, 'use_graph': step.use_graph,
                'eager': step.eager_runs, 'steps': step.opt.steps}, os.path.join(out, f'g{rank}.pt'))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_capture_failure_on_one_rank_falls_back_everywhere(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2)
    a = torch.load(tmp_path / 'g0.pt', weights_only=True)
    b = torch.load(tmp_path / 'g1.pt', weights_only=True)
    for r in (a, b):
        assert not r['graph'] and not r['use_graph']
        assert r['eager'] == 5 and r['steps'] == 5
    # every all-reduce matched up: 5 steps x (1 + 2)
    assert torch.equal(a['w'], b['w']) and torch.equal(a['w'], torch.full((4,), 15.0))
