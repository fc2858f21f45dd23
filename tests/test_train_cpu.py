"""Config-driven training engine on CPU: experiment parsing, runner loop + callbacks,
checkpoint/resume, contrib losses/schedulers, gloo DDP (world_size 2) and the
``catalyst``/``train`` executor run end-to-end through a DAG."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
import yaml

from mlcomp_amd.train.experiment import ConfigExperiment
from mlcomp_amd.train.runner import Runner


def _cfg(logdir, epochs=2, stages=('stage1',), sched=None, n=64):
    st = {
        'data_params': {'dataset': 'synthetic_classification', 'batch_size': 16, 'num_samples': n,
                        'valid_samples': 32, 'image_size': 16, 'num_classes': 4},
        'state_params': {'num_epochs': epochs, 'main_metric': 'accuracy01', 'minimize_metric': False},
        'criterion_params': {'criterion': 'CrossEntropyLoss'},
        'optimizer_params': {'optimizer': 'Adam', 'lr': 0.01},
        'callbacks_params': {
            'loss': {'callback': 'CriterionCallback'},
            'optimizer': {'callback': 'OptimizerCallback'},
            'accuracy': {'callback': 'AccuracyCallback', 'accuracy_args': [1, 2]},
            'saver': {'callback': 'CheckpointCallback'},
        },
    }
    if sched:
        st['scheduler_params'] = sched
        st['callbacks_params']['scheduler'] = {'callback': 'SchedulerCallback', 'reduced_metric': 'accuracy01'}
    for s in stages:
        st[s] = {}
    return {'model_params': {'model': 'SimpleCNN', 'num_classes': 4, 'width': 8},
            'args': {'expdir': '.', 'logdir': str(logdir), 'engine': 'torch'},
            'stages': st}


def test_experiment_merges_shared_sections(tmp_path):
    cfg = _cfg(tmp_path, stages=('warm', 'main'))
    cfg['stages']['main'] = {'optimizer_params': {'lr': 0.5}}
    e = ConfigExperiment(cfg)
    assert e.stages == ['warm', 'main']
    assert e.stage_params('warm', 'optimizer_params')['lr'] == 0.01
    assert e.stage_params('main', 'optimizer_params') == {'optimizer': 'Adam', 'lr': 0.5}
    assert e.stage_params('main', 'data_params')['batch_size'] == 16


def test_runner_trains_checkpoints_and_resumes(tmp_path):
    torch.manual_seed(0)
    cfg = _cfg(tmp_path, epochs=3, sched={'scheduler': 'OneCycleCosineAnnealLR', 'T_max': 2})
    r = Runner(ConfigExperiment(cfg), device='cpu')
    st = r.run_experiment()
    for k in ('train_loss', 'train_accuracy01', 'train_accuracy02', 'valid_loss', 'valid_accuracy01',
              'train__timer/_fps', 'lr'):
        assert k in st.epoch_metrics, k
    assert st.epoch == 2
    ck = tmp_path / 'checkpoints'
    for f in ('last_full.pth', 'best_full.pth', 'last.pth', 'best.pth'):
        assert (ck / f).exists()
    d = torch.load(ck / 'last_full.pth', map_location='cpu', weights_only=True)
    assert d['stage'] == 'stage1' and d['checkpoint_data']['epoch'] == 2
    # resume: a fresh runner restores the weights from the checkpoint
    r2 = Runner(ConfigExperiment(cfg), device='cpu')
    r2.model = r2.experiment.get_model('stage1')
    r2.model.load_state_dict(d['model_state_dict'])
    for k, v in r.model.state_dict().items():
        assert torch.equal(v.cpu(), r2.model.state_dict()[k])


def test_runner_learns_separable_data(tmp_path):
    """A learnable synthetic task: class = sign pattern of the first two pixels."""
    from collections import OrderedDict

    class Sep(torch.utils.data.Dataset):
        def __init__(self, n, seed):
            g = torch.Generator().manual_seed(seed)
            self.x = torch.randn(n, 3, 8, 8, generator=g)
            self.y = ((self.x[:, 0].mean((1, 2)) > 0).long() * 2 + (self.x[:, 1].mean((1, 2)) > 0).long())

        def __len__(self):
            return len(self.y)

        def __getitem__(self, i):
            return self.x[i], int(self.y[i])

    class E(ConfigExperiment):
        def get_datasets(self, stage, **kw):
            return OrderedDict(train=Sep(512, 0), valid=Sep(128, 1))

    cfg = _cfg(tmp_path, epochs=6)
    cfg['stages']['data_params']['batch_size'] = 32
    r = Runner(E(cfg), device='cpu')
    st = r.run_experiment()
    assert st.valid_metrics['accuracy01'] > 0.6, st.valid_metrics


def test_contrib_losses_match_definitions():
    from mlcomp_amd.contrib.criterion import LabelSmoothingCrossEntropy, RingLoss, triplet_loss
    torch.manual_seed(0)
    x = torch.randn(16, 5)
    y = torch.randint(0, 5, (16,))
    eps = 0.2
    ref = (1 - eps) * torch.nn.functional.cross_entropy(x, y) + eps * (-torch.log_softmax(x, 1).mean(1)).mean()
    assert torch.allclose(LabelSmoothingCrossEntropy(eps)(x, y), ref, atol=1e-6)
    assert torch.allclose(LabelSmoothingCrossEntropy(eps)(x, y),
                          torch.nn.functional.cross_entropy(x, y, label_smoothing=eps), atol=1e-6)
    rl = RingLoss(type='l2', loss_weight=1.0)
    v = rl(x, y)
    assert torch.allclose(rl.radius.detach(), x.norm(dim=1).mean().reshape(1))
    assert v.item() >= torch.nn.functional.cross_entropy(x, y).item() - 1e-6
    # triplet: brute force over all (a, p, n)
    e = torch.randn(6, 4)
    lab = torch.tensor([0, 0, 1, 1, 2, 0])
    en = torch.nn.functional.normalize(e, dim=1)
    d = 1 - en @ en.t()
    vals = []
    for a in range(6):
        for p in range(6):
            for n in range(6):
                if len({a, p, n}) == 3 and lab[a] == lab[p] and lab[a] != lab[n]:
                    vals.append(torch.relu(d[a, p] - d[a, n] + 0.3))
    vals = torch.stack(vals)
    ref = vals.sum() / ((vals > 1e-8).sum() + 1e-8)
    assert torch.allclose(triplet_loss(e, lab), ref, atol=1e-5)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ddp_worker(rank, world, port, logdir, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.manual_seed(0)
    cfg = _cfg(logdir, epochs=1)
    r = Runner(ConfigExperiment(cfg), device='cpu', rank=rank, world_size=world)
    st = r.run_experiment()
    w = torch.cat([p.detach().flatten() for p in r.model.parameters()])
    torch.save({'w': w, 'n': len(r.loaders['train'].sampler), 'fps_node': st.epoch_metrics.get(
        'train__timer/_fps_node'), 'fps': st.epoch_metrics.get('train__timer/_fps')}, os.path.join(out, f'r{rank}.pt'))
    dist.destroy_process_group()


def test_ddp_gloo_two_ranks_stay_in_sync(tmp_path):
    mp.spawn(_ddp_worker, args=(2, _free_port(), str(tmp_path / 'log'), str(tmp_path)), nprocs=2)
    a = torch.load(tmp_path / 'r0.pt', weights_only=True)
    b = torch.load(tmp_path / 'r1.pt', weights_only=True)
    assert a['n'] == b['n'] == 32          # 64 samples split over 2 ranks
    assert torch.allclose(a['w'], b['w'])  # gradients all-reduced -> identical weights
    # whole-node throughput is the sum of the ranks' own rates, the same on every rank
    assert a['fps_node'] == pytest.approx(a['fps'] + b['fps'], rel=1e-6)
    assert b['fps_node'] == pytest.approx(a['fps_node'], rel=1e-9)
    assert (tmp_path / 'log' / 'checkpoints' / 'last_full.pth').exists()


# ---------------------------------------------------------------------------- executor
from test_lifecycle import _submit, _wait, cluster  # noqa: E402,F401


def test_train_executor_through_dag(cluster, tmp_path):
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.enums import TaskStatus
    from mlcomp_amd.db.models import ReportSeries, Step, Task
    cat = _cfg('log', epochs=2, stages=('warm', 'main'))
    cfg = {'info': {'name': 'trn', 'project': 'p_train', 'layout': 'classify'},
           'executors': {'train': {'type': 'catalyst', 'args': {'config': 'catalyst.yml'}}}}
    created = _submit(cluster['tmp'], cfg, files={'catalyst.yml': yaml.safe_dump(cat)})
    ids = [t.id for t in created[1]] if isinstance(created, tuple) else None
    if ids is None:
        s = Session.create_session(key='q')
        ids = [t.id for t in s.query(Task).all()]
    res = _wait(cluster['sup'], ids, timeout=240)
    assert all(v == TaskStatus.Success for v in res.values()), res
    s = Session.create_session(key='q2')
    tid = ids[0]
    series = s.query(ReportSeries).filter(ReportSeries.task == tid).all()
    names = {(r.part, r.name, r.stage) for r in series}
    assert ('train', 'loss', 'warm') in names and ('valid', 'accuracy01', 'main') in names
    steps = s.query(Step).filter(Step.task == tid).all()
    assert {'warm', 'main'} <= {st.name for st in steps}
    t = s.get(Task, tid)
    assert t.score is not None and t.loss is not None
    # the engine that trained each stage (and why) is stored on the task and in its DB log
    from mlcomp_amd.db.models import Log
    from mlcomp_amd.utils.misc import yaml_load
    eng = (yaml_load(t.additional_info) or {})['engine']
    assert set(eng) == {'warm', 'main'} and eng['main']['engine'] == 'torch', eng
    assert eng['main']['reason'] == 'engine: torch requested' and eng['main']['precision'] == 'bf16'
    msgs = [lg.message for lg in s.query(Log).filter(Log.task == tid).all()]
    assert any('stage main: torch engine' in m for m in msgs), msgs[-20:]


# ---------------------------------------------------------------------------- native DP
def _native_dp_worker(rank, world, port, kind, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.manual_seed(0)
    if kind == 'resnet':
        from mlcomp_amd.train.native_step import NativeClassifierStep
        step = NativeClassifierStep('resnet18', batch=4, image_size=32, device='cpu', world_size=world,
                                    num_classes=10, use_graph=False)
    elif kind == 'unet':
        from mlcomp_amd.train.native_seg_step import NativeSegmentationStep
        step = NativeSegmentationStep('resnet18', batch=2, image_size=64, device='cpu', world_size=world,
                                      use_graph=False)
    else:
        from mlcomp_amd.train.native_bert_step import NativeBertStep
        step = NativeBertStep('bert-tiny', batch=4, seq_len=16, device='cpu', world_size=world, use_graph=False)
    for _ in range(2):
        step()
    arena = step.net.arena
    w = torch.cat([a.master.flatten() for a in arena.arenas()])
    g = torch.cat([a.grad.flatten() for a in arena.arenas()])
    torch.save({'w': w, 'g': g}, os.path.join(out, f'{kind}{rank}.pt'))
    dist.destroy_process_group()


@pytest.mark.parametrize('kind', ['resnet', 'unet', 'bert'])
def test_native_engines_data_parallel_two_ranks(tmp_path, kind):
    """Native engines over 2 gloo ranks with different data per rank: the bucketed gradient
    all-reduce leaves identical gradients and identical weights on both ranks."""
    mp.spawn(_native_dp_worker, args=(2, _free_port(), kind, str(tmp_path)), nprocs=2)
    a = torch.load(tmp_path / f'{kind}0.pt', weights_only=True)
    b = torch.load(tmp_path / f'{kind}1.pt', weights_only=True)
    assert torch.isfinite(a['w']).all() and a['g'].abs().sum() > 0
    assert torch.allclose(a['g'], b['g']) and torch.allclose(a['w'], b['w'])


def test_resume_mid_stage_restores_optimizer_schedule_and_best(tmp_path):
    """Resuming at epoch k restores the optimizer moments, the LR-schedule position and the
    best score (`catalyst_.py:341-345`), so a worse first resumed epoch does not overwrite
    best_full.pth."""
    sched = {'scheduler': 'StepLR', 'step_size': 1, 'gamma': 0.5}
    torch.manual_seed(0)
    r = Runner(ConfigExperiment(_cfg(tmp_path, epochs=2, sched=sched)), device='cpu')
    r.run_experiment()
    ck = tmp_path / 'checkpoints'
    d = torch.load(ck / 'last_full.pth', map_location='cpu', weights_only=True)
    assert d['checkpoint_data']['epoch'] == 1 and d['best_score'] is not None
    # pretend the best score so far was unbeatable: a resumed epoch must not replace it
    d['best_score'] = 2.0
    torch.save(d, ck / 'last_full.pth')
    best_before = (ck / 'best_full.pth').read_bytes()
    r2 = Runner(ConfigExperiment(_cfg(tmp_path, epochs=3, sched=sched)), device='cpu')
    r2.resume(str(ck / 'last_full.pth'))
    seen = {}

    class Probe:
        order = 1
        master_only = False

        def __getattr__(self, name):
            return lambda state: None

        def on_epoch_start(self, state):
            seen.setdefault('lr', state.current_lr())
            seen.setdefault('exp_avg', [v['exp_avg'].clone() for v in state.optimizer.state.values()])

    r2.extra_callbacks['probe'] = Probe()
    st = r2.run_experiment(start_epoch=2)
    assert st.epoch == 2
    assert abs(seen['lr'] - 0.01 * 0.5 ** 2) < 1e-9          # StepLR position carried over
    opt_state = d['optimizer_state_dict']['state']
    assert len(seen['exp_avg']) == len(opt_state) > 0
    for got, ref in zip(seen['exp_avg'], [v['exp_avg'] for v in opt_state.values()]):
        assert torch.equal(got, ref)                             # Adam moments restored
    saver = [c for c in r2.callbacks if type(c).__name__ == 'CheckpointCallback'][0]
    assert saver.best_score == 2.0
    assert (ck / 'best_full.pth').read_bytes() == best_before


def test_bucket_plan_caps_the_exposed_last_bucket():
    """Buckets tile the arena contiguously in backward order; the first is small and the
    final one (first layers, ready only at the end of backward) is capped."""
    from mlcomp_amd.models import build_model
    from mlcomp_amd.models.native_resnet import NativeResNet
    from mlcomp_amd.parallel.ddp import plan_buckets
    net = NativeResNet(build_model('resnet50', num_classes=1000), 'cpu')
    a = net.arena.decay
    mb = 2 ** 20
    for last in (None, 4 * mb, 1 * mb):
        bs = plan_buckets(a, 32 * mb, 8 * mb, last)
        assert bs[0].start == 0 and bs[-1].end == a.numel
        assert all(x.end == y.start for x, y in zip(bs, bs[1:]))
        assert sum(len(b.slots) for b in bs) == len(a.slots)
        assert bs[0].nbytes >= 8 * mb
        if last:
            assert bs[-1].nbytes <= last and len(bs[-1].slots) >= 1
    assert plan_buckets(a, 32 * mb, 8 * mb, 4 * mb)[-1].nbytes < plan_buckets(a, 32 * mb, 8 * mb)[-1].nbytes


@pytest.mark.parametrize('kind', ['resnet', 'unet', 'bert'])
def test_optimizer_in_backward_matches_step_at_end(kind, monkeypatch):
    """Each gradient bucket is updated as soon as its last gradient is marked ready.  On the
    CPU that update runs immediately, so a weight read in backward after its slot was marked
    (a dgrad after its wgrad) would change the result: both modes must agree exactly."""
    # one bucket per parameter: every slot is updated the moment it is marked
    monkeypatch.setenv('MLC_BUCKET_MB', '0.0001')
    monkeypatch.setenv('MLC_FIRST_BUCKET_MB', '0.0001')
    monkeypatch.setenv('MLC_LAST_BUCKET_MB', '0')

    def run(flag):
        monkeypatch.setenv('MLC_OPT_IN_BWD', flag)
        torch.manual_seed(0)
        if kind == 'resnet':
            from mlcomp_amd.train.native_step import NativeClassifierStep
            st = NativeClassifierStep('resnet18', batch=4, image_size=32, device='cpu', num_classes=10,
                                      use_graph=False, lr=0.1)
        elif kind == 'unet':
            from mlcomp_amd.train.native_seg_step import NativeSegmentationStep
            st = NativeSegmentationStep('resnet18', batch=2, image_size=64, device='cpu', use_graph=False, lr=1e-2)
        else:
            from mlcomp_amd.train.native_bert_step import NativeBertStep
            st = NativeBertStep('bert-tiny', batch=4, seq_len=16, device='cpu', use_graph=False, lr=1e-2)
        assert st.opt_in_bwd == (flag == '1')
        for _ in range(2):
            st()
        return torch.cat([a.master.flatten() for a in st.net.arena.arenas()])
    a, b = run('1'), run('0')
    assert torch.isfinite(a).all()
    assert torch.allclose(a, b, atol=1e-6, rtol=1e-5), (a - b).abs().max()


# ---------------------------------------------------------------------------- engine choice
def test_engine_choice_records_the_fallback_reason(tmp_path, monkeypatch):
    """engine: auto never falls back silently: the reason lands in runner.engine_log (and
    the hook the train executor turns into a task log line + additional_info)."""
    import mlcomp_amd.train.runner as R
    cfg = _cfg(tmp_path, epochs=1)
    cfg['args']['engine'] = 'auto'
    seen = []
    r = Runner(ConfigExperiment(cfg), device='cpu')
    r.engine_hook = seen.append
    r.run_experiment()
    assert seen == r.engine_log and len(seen) == 1
    assert seen[0]['engine'] == 'torch' and 'no HIP device' in seen[0]['reason']
    # a GPU-capable model whose stage asks for an optimizer the native engines lack
    cfg['stages']['optimizer_params'] = {'optimizer': 'RMSprop', 'lr': 0.01}
    r = Runner(ConfigExperiment(cfg), device='cpu')
    r.model = r.experiment.get_model('stage1')
    monkeypatch.setattr(R, '_native_kind', lambda m, d: 'resnet')
    r.device = torch.device('cuda')          # selection only; nothing is built
    got = r._select_engine('stage1')
    assert got['engine'] == 'torch' and 'RMSprop' in got['reason']
    r.engine = 'native'
    with pytest.raises(RuntimeError, match='RMSprop'):
        r._select_engine('stage1')
    # precision fp32 keeps the stage on the torch engine, and says so
    cfg['stages']['optimizer_params'] = {'optimizer': 'Adam', 'lr': 0.01}
    cfg['args']['precision'] = 'fp32'
    r = Runner(ConfigExperiment(cfg), device='cpu')
    r.model = r.experiment.get_model('stage1')
    r.device = torch.device('cuda')
    got = r._select_engine('stage1')
    assert got['engine'] == 'torch' and got['precision'] == 'fp32' and 'fp32' in got['reason']
    with pytest.raises(ValueError, match='precision'):
        Runner(ConfigExperiment(dict(cfg, args=dict(cfg['args'], precision='fp16'))), device='cpu')


def test_fp32_torch_engine_matches_plain_fp32_training(tmp_path):
    """precision: fp32 is plain fp32 autograd + torch.optim (no autocast): the runner's
    weights after an epoch equal a hand-written fp32 loop over the same batches."""
    cfg = _cfg(tmp_path, epochs=1, n=32)
    cfg['args']['precision'] = 'fp32'
    cfg['stages']['callbacks_params'].pop('saver')
    torch.manual_seed(3)
    r = Runner(ConfigExperiment(cfg), device='cpu')
    r.run_experiment()
    torch.manual_seed(3)
    e = ConfigExperiment(cfg)
    m = e.get_model('stage1')
    opt = torch.optim.Adam(m.parameters(), lr=0.01)
    for b in r.loaders['train']:
        m.train()
        loss = torch.nn.functional.cross_entropy(m(b['features']), b['targets'])
        opt.zero_grad()
        loss.backward()
        opt.step()
    for k, v in m.state_dict().items():
        assert torch.allclose(v, r.model.state_dict()[k], atol=1e-6, rtol=1e-5), k
