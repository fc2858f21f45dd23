"""End-to-end native engine on the GPU: eager step vs HIP-graph replay, convergence on a
fixed batch, RCCL communicator plumbing (single rank)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(**kw):
    from mlcomp_amd.train.native_step import NativeClassifierStep
    return NativeClassifierStep(**kw)


def test_native_resnet18_overfits_fixed_batch():
    st = _step(model_name='resnet18', batch=32, image_size=64, device='cuda', num_classes=10,
               lr=0.05, momentum=0.9, use_graph=False)
    losses = []
    for _ in range(30):
        st()
        losses.append(st.last_loss())
    assert all(l == l for l in losses)  # no NaN
    assert losses[-1] < 0.5 * losses[0], losses


def test_graph_replay_matches_eager():
    """Default (fast) mode: split-K weight gradients and BN statistics add with float
    atomics, so a graph replay and an eager step differ in the last bits; after a few
    moderate SGD steps that stays under 1e-3.  (Deterministic mode makes the two bitwise
    equal: tests/test_deterministic_gpu.py.)"""
    torch.manual_seed(3)
    from mlcomp_amd.models import build_model
    tm1 = build_model('resnet18', num_classes=10)
    tm2 = build_model('resnet18', num_classes=10)
    tm2.load_state_dict(tm1.state_dict())
    kw = dict(batch=16, image_size=64, device='cuda', num_classes=10, lr=0.02, momentum=0.9)
    a = _step(torch_model=tm1, use_graph=False, **kw)
    b = _step(torch_model=tm2, use_graph=True, warmup_eager=2, **kw)
    for _ in range(4):
        a()
        b()
    torch.cuda.synchronize()
    assert b.graph is not None
    la, lb = a.last_loss(), b.last_loss()
    assert abs(la - lb) <= 1e-3 * max(1.0, abs(la)), (la, lb)
    pa = a.net.arena.decay.master
    pb = b.net.arena.decay.master
    assert ((pa - pb).norm() / pa.norm()).item() < 1e-3


def test_rccl_single_rank():
    import torch.distributed as dist
    from mlcomp_amd.parallel.comm import RcclComm
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29611')
    store = dist.TCPStore('127.0.0.1', 29611, 1, True)
    comm = RcclComm(0, 1, torch.device('cuda', 0), store=store, tag='t1')
    t = torch.arange(1024, device='cuda', dtype=torch.float32)
    comm.all_reduce(t)
    comm.broadcast(t, 0)
    out = torch.empty(1024, device='cuda')
    comm.all_gather(out, t)
    torch.cuda.synchronize()
    assert torch.equal(t, torch.arange(1024, device='cuda', dtype=torch.float32))
    assert torch.equal(out, t)
    comm.close()


def test_runner_native_engine_on_device_data(tmp_path):
    """Config-driven runner picks the native engine for a ResNet on the GPU; checkpoints
    export the native arenas back into the torch module."""
    from mlcomp_amd.train.experiment import ConfigExperiment
    from mlcomp_amd.train.runner import Runner
    cfg = {'model_params': {'model': 'resnet18', 'num_classes': 10},
           'args': {'logdir': str(tmp_path), 'engine': 'auto'},
           'stages': {
               'data_params': {'dataset': 'synthetic_classification', 'on_device': True,
                               'batch_size': 32, 'steps': 6, 'image_size': 64, 'num_classes': 10},
               'state_params': {'num_epochs': 2},
               'optimizer_params': {'optimizer': 'SGD', 'lr': 0.05, 'momentum': 0.9},
               'scheduler_params': {'scheduler': 'OneCycleCosineAnnealLR', 'T_max': 2},
               'callbacks_params': {'loss': {'callback': 'CriterionCallback'},
                                    'opt': {'callback': 'OptimizerCallback'},
                                    'acc': {'callback': 'AccuracyCallback'},
                                    'sched': {'callback': 'SchedulerCallback'},
                                    'saver': {'callback': 'CheckpointCallback'}},
               'stage1': {}}}
    r = Runner(ConfigExperiment(cfg), device='cuda')
    st = r.run_experiment()
    assert st.native and r.native_step is not None
    m = st.epoch_metrics
    assert m['train_loss'] == m['train_loss'] and m['train_loss'] > 0
    assert 0 <= m['train_accuracy01'] <= 1
    ck = torch.load(tmp_path / 'checkpoints' / 'last_full.pth', weights_only=True)
    w = ck['model_state_dict']['fc.weight']
    assert torch.isfinite(w).all()
    assert not torch.equal(w, torch.zeros_like(w))


def test_graph_captured_rccl_bucketed_allreduce():
    """The data-parallel path (gradient buckets all-reduced on a side stream while the
    backward runs, everything captured in one HIP graph) on a 1-rank RCCL communicator:
    the all-reduce is then an identity, so parameters must track a run without one."""
    import torch.distributed as dist
    from mlcomp_amd.models import build_model
    from mlcomp_amd.parallel.comm import RcclComm
    from mlcomp_amd.train.native_step import NativeClassifierStep
    torch.manual_seed(7)
    store = dist.TCPStore('127.0.0.1', 29613, 1, True)
    comm = RcclComm(0, 1, torch.device('cuda', 0), store=store, tag='t2')
    tm1 = build_model('resnet18', num_classes=10)
    tm2 = build_model('resnet18', num_classes=10)
    tm2.load_state_dict(tm1.state_dict())
    a = NativeClassifierStep(torch_model=tm1, batch=8, image_size=64, device="cuda", num_classes=10,
                             use_graph=True, comm=comm)
    b = NativeClassifierStep(torch_model=tm2, batch=8, image_size=64, device="cuda", num_classes=10,
                             use_graph=True)
    b.load_batch(a.x, a.y)
    for _ in range(5):
        a()
        b()
    torch.cuda.synchronize()
    assert a.graph is not None
    pa, pb = a.net.arena.decay.master, b.net.arena.decay.master
    assert ((pa - pb).norm() / pa.norm()).item() < 5e-3
    assert abs(a.last_loss() - b.last_loss()) < 5e-2 * abs(b.last_loss()) + 1e-3
    comm.close()
