"""The generic native engine on CPU (the ops' reference paths, same bf16 rounding points as
the kernels): fx lowering coverage of the reference's example nets and the zoo, per-site
numerics against fp32 autograd, the step (fused optimizer with torch.optim semantics,
gradient arena), gloo data parallelism, and the runner's engine choice.

Reference models: `examples/digit-recognizer/model.py:8-25` (LeNet), `examples/cifar_simple/
model.py:8-26` (CIFAR Net), `mlcomp/contrib/segmentation/encoders/__init__.py:12-18`
(resnext / senet / dpn / densenet encoders)."""
import os
import socket

import pytest
import operator

import torch
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

from mlcomp_amd.models import build_model
from mlcomp_amd.models.native_generic import GenericNet, lower_or_none
from mlcomp_amd.ops import functional as Fn


class RefCifarNet(nn.Module):
    """The reference's cifar_simple ``Net`` (conv5 6 / 16, pools, three Linear layers)."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 6, 5)
        self.pool = nn.MaxPool2d(2, 2)
        self.conv2 = nn.Conv2d(6, 16, 5)
        self.fc1 = nn.Linear(16 * 5 * 5, 120)
        self.fc2 = nn.Linear(120, 84)
        self.fc3 = nn.Linear(84, 10)

    def forward(self, x):
        x = self.pool(F.relu(self.conv1(x)))
        x = self.pool(F.relu(self.conv2(x)))
        x = x.view(-1, 16 * 5 * 5)
        x = F.relu(self.fc1(x))
        x = F.relu(self.fc2(x))
        return self.fc3(x)


def _cos(a, b):
    a, b = a.flatten().float(), b.flatten().float()
    return (a @ b / (a.norm() * b.norm() + 1e-12)).item()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _torch_grad(p, ref):
    """The reference module's gradient of a parameter set, in the set's layout."""
    m = dict(ref.named_modules())[p.name]
    if getattr(p, 'kind', None) == 'tr':
        return _torch_grad_tr(p, ref)
    if hasattr(p, 'kind'):
        g = m.weight.grad
        if p.kind == 's2d':
            return F.pad(Fn.stem_w_to_s2d(g), (0, 0, 0, 0, 0, 0, 0, p.Cop - p.Co))
        if p.kind == 'dense':
            return F.pad(g.permute(0, 2, 3, 1), (0, p.Cip - p.Ci, 0, 0, 0, 0, 0, p.Cop - p.Co))
        if p.kind == 'dw':
            return F.pad(g[:, 0].permute(1, 2, 0), (0, p.Cop - p.Co))
        return g.permute(0, 2, 3, 1)
    if hasattr(p, 'O'):
        return F.pad(m.weight.grad, (0, p.Ip - p.I, 0, p.Op - p.O))
    return F.pad(m.weight.grad, (0, p.Cp - p.C))


def _torch_grad_tr(p, ref):
    g = dict(ref.named_modules())[p.name].weight.grad      # [Cin, Cout, KH, KW]
    return F.pad(g.permute(0, 2, 3, 1), (0, p.Cop - p.Co, 0, 0, 0, 0, 0, p.Cip - p.Ci))


def _pair(make, seed=0):
    torch.manual_seed(seed)
    m = make()
    ref = make()
    ref.load_state_dict(m.state_dict())
    for mm in (m, ref):
        for d in mm.modules():
            if isinstance(d, nn.Dropout):
                d.p = 0.0
            if hasattr(d, 'drop_path'):
                d.drop_path = 0.0
    return m, ref


@pytest.mark.parametrize('name', ['LeNet', 'resnext50_32x4d', 'se_resnext50_32x4d', 'efficientnet-b0', 'dpn92', 'senet154', 'inceptionresnetv2',
                                  'mobilenet_v2', 'densenet121', 'dpn68', 'xception', 'vgg16', 'resnet18'])
def test_zoo_lowers_completely(name):
    """Every conv / BN / linear / pool of these models becomes a native site: no call that
    would reach MIOpen / hipBLASLt / rocBLAS is left in the train or eval graph."""
    m = build_model(name, num_classes=10)
    assert lower_or_none(m) is None
    net = GenericNet.__new__(GenericNet)
    from mlcomp_amd.models.native_generic import _Lowering
    from mlcomp_amd.ops.layers import NativeContext
    import torch.fx as fx
    net.ctx, net._params = NativeContext(), {}
    gm = _Lowering(net, fx.symbolic_trace(m.train())).run()
    left = [type(mod).__name__ for mod in gm.modules()
            if isinstance(mod, (nn.Conv2d, nn.Linear, nn.BatchNorm2d, nn.BatchNorm1d, nn.ConvTranspose2d))]
    assert not left, left
    for n in gm.graph.nodes:
        assert n.target not in (F.conv2d, F.linear, F.batch_norm, torch.matmul), n


def test_reference_example_nets_match_fp32_autograd():
    """The reference's LeNet and CIFAR Net: outputs and every parameter gradient against
    fp32 autograd of the same weights (bf16 activations: loose but discriminating)."""
    for make, shape in ((RefCifarNet, (16, 3, 32, 32)), (lambda: build_model('LeNet', num_classes=10),
                                                          (16, 1, 28, 28))):
        m, ref = _pair(make)
        x = torch.randn(*shape)
        y = torch.randint(0, 10, (shape[0],))
        net = GenericNet(m, 'cpu')
        out = net(x)
        F.cross_entropy(out.float(), y).backward()
        want = ref(x)
        F.cross_entropy(want, y).backward()
        assert _rel(out, want) < 2e-2
        # the gradients reach conv1 through bf16 max-pool argmaxes and ReLU masks, where a
        # rounding can flip a window's winner: directions, not magnitudes per element
        for p in net.param_sets():
            g = p.w.grad if hasattr(p, 'w') else p.gamma.grad
            assert _cos(g, _torch_grad(p, ref)) > 0.98, p.name
            if getattr(p, 'b', None) is not None:
                bb = dict(ref.named_modules())[p.name].bias.grad
                assert _cos(p.b.grad[:bb.numel()], bb) > 0.98, p.name


@pytest.mark.parametrize('act', ['relu', 'relu6', 'silu', 'sigmoid', 'tanh', 'hardswish', 'leaky_relu', 'gelu',
                                 'elu', 'hardsigmoid'])
@pytest.mark.parametrize('groups', [1, 2, 8, 64])
def test_conv_bn_act_residual_site(act, groups):
    """conv (dense / grouped Cg=32 / Cg=8 / depthwise) -> BN -> + residual -> act."""
    mods = {'relu': nn.ReLU(), 'relu6': nn.ReLU6(), 'silu': nn.SiLU(), 'sigmoid': nn.Sigmoid(), 'tanh': nn.Tanh(),
            'hardswish': nn.Hardswish(), 'leaky_relu': nn.LeakyReLU(0.2), 'gelu': nn.GELU(), 'elu': nn.ELU(0.7),
            'hardsigmoid': nn.Hardsigmoid()}

    class Block(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv = nn.Conv2d(64, 64, 3, 1, 1, groups=groups, bias=False)
            self.bn = nn.BatchNorm2d(64)
            self.act = mods[act]
            self.head = nn.Conv2d(64, 16, 1)

        def forward(self, x):
            return self.head(self.act(self.bn(self.conv(x)) + x))

    m, ref = _pair(Block)
    with torch.no_grad():
        m.bn.weight.uniform_(0.5, 1.5)
        m.bn.bias.uniform_(-0.5, 0.5)
        ref.load_state_dict(m.state_dict())
    x = torch.randn(8, 64, 12, 12)
    net = GenericNet(m, 'cpu')
    sites = [type(s).__name__ for s in net.train_gm.modules() if hasattr(s, 'fwd')]
    assert sites == ['ConvBNAct', 'ConvBNAct'], sites
    xr = x.clone().requires_grad_()
    xn = x.clone().requires_grad_()
    out = net(xn)
    d = torch.randn_like(out.float())
    (out.float() * d).sum().backward()
    want = ref(xr)
    (want * d).sum().backward()
    assert _rel(out, want) < 2e-2
    assert _rel(xn.grad, xr.grad) < 5e-2
    for p in net.param_sets():
        g = p.w.grad if hasattr(p, 'w') else p.gamma.grad
        assert _rel(g, _torch_grad(p, ref)) < 5e-2, (p.name, _rel(g, _torch_grad(p, ref)))
    # running statistics moved exactly like torch's (momentum 0.1, unbiased variance)
    bn = [p for p in net.param_sets() if hasattr(p, 'run_mean')][0]
    assert torch.allclose(bn.run_mean[:64], ref.bn.running_mean, rtol=2e-2, atol=2e-3)
    assert torch.allclose(bn.run_var[:64], ref.bn.running_var, rtol=2e-2, atol=2e-3)


def test_linear_bn1d_pool_sites_and_eval_graph():
    class Head(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv = nn.Conv2d(5, 24, 3, padding=1)
            self.pool = nn.MaxPool2d(3, 2, 1, ceil_mode=True)
            self.gap = nn.AdaptiveAvgPool2d(1)
            self.fc = nn.Linear(24, 36)
            self.bn1 = nn.BatchNorm1d(36)
            self.out = nn.Linear(36, 7)

        def forward(self, x):
            x = self.gap(self.pool(F.relu(self.conv(x)))).flatten(1)
            return self.out(F.silu(self.bn1(self.fc(x))))

    m, ref = _pair(Head)
    x = torch.randn(16, 5, 11, 13)
    net = GenericNet(m, 'cpu')
    kinds = sorted(type(s).__name__ for s in net.train_gm.modules() if hasattr(s, 'fwd'))
    assert kinds == ['BNAct', 'ConvBNAct', 'GlobalAvgPool', 'LinearAct', 'LinearAct', 'MaxPool'], kinds
    out = net(x)
    out.float().sum().backward()
    want = ref(x)
    want.sum().backward()
    assert _rel(out, want) < 4e-2          # BatchNorm1d over 16 rows amplifies bf16 rounding
    for p in net.param_sets():           # through a bf16 max-pool: directions (see above)
        g = p.w.grad if hasattr(p, 'w') else p.gamma.grad
        assert _cos(g, _torch_grad(p, ref)) > 0.99, p.name
    # inference graph: running statistics, no autograd
    net.eval()
    ref.eval()
    with torch.no_grad():
        assert _rel(net(x), ref(x)) < 5e-2


def test_generic_step_optimizer_matches_torch_optim_semantics():
    """One NativeGenericStep = forward + criterion + backward + fused update with torch.optim's
    semantics (weight decay on EVERY parameter, BN and biases included): the arena after a
    step equals torch.optim.<opt> applied to the step's own gradients."""
    from mlcomp_amd.train.native_generic_step import NativeGenericStep
    for opt, kw in (('SGD', dict(lr=0.1, momentum=0.9, weight_decay=1e-2)),
                    ('AdamW', dict(lr=1e-2, weight_decay=0.1)), ('Adam', dict(lr=1e-2, weight_decay=1e-2))):
        torch.manual_seed(0)
        m = RefCifarNet()
        x, y = torch.randn(8, 3, 32, 32), torch.randint(0, 10, (8,))
        step = NativeGenericStep(m, x, y, device='cpu', use_graph=False, optimizer=opt, **kw)
        arena = step.net.arena
        before = [a.master.clone() for a in arena.arenas()]
        step()                     # GraphedStep.__call__ runs opt.prepare() itself
        grads = [a.grad.clone() for a in arena.arenas()]
        params = [torch.nn.Parameter(b.clone()) for b in before]
        for p, g in zip(params, grads):
            p.grad = g
        tkw = dict(kw)
        o = getattr(torch.optim, opt)(params, **tkw)
        o.step()
        for p, a in zip(params, arena.arenas()):
            assert torch.allclose(a.master, p.detach(), rtol=1e-5, atol=1e-6), opt
        with torch.no_grad():            # the torch model still holds the initial weights
            want = float(F.cross_entropy(m(x), y))
        assert step.last_loss() == pytest.approx(want, rel=0.02)


def test_eval_graph_runs_dropout_in_eval_mode():
    """A model with a live Dropout (p = 0.5): net.eval() outputs are deterministic and equal
    torch's eval() outputs, and net.train() drops again (the leaf Dropout module is shared
    by both lowered graphs and the user model)."""
    class Drop(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc1 = nn.Linear(32, 64)
            self.drop = nn.Dropout(0.5)
            self.fc2 = nn.Linear(64, 8)

        def forward(self, x):
            return self.fc2(self.drop(F.relu(self.fc1(x))))

    torch.manual_seed(0)
    m = Drop()
    ref = Drop()
    ref.load_state_dict(m.state_dict())
    net = GenericNet(m, 'cpu')
    x = torch.randn(16, 32)
    with torch.no_grad():
        t1, t2 = net(x), net(x)
        assert _rel(t1, t2) > 1e-2            # training graph: dropout active
        net.eval()
        e1, e2 = net(x), net(x)
        assert torch.equal(e1, e2)
        assert _rel(e1, ref.eval()(x)) < 2e-2
        net.train()
        assert _rel(net(x), net(x)) > 1e-2


def test_frozen_and_non_affine_parameters_are_not_updated():
    """requires_grad=False parameters and an affine=False BatchNorm's gamma / beta keep their
    values through a fused SGD step with weight decay (torch.optim skips them), while the
    trainable ones move."""
    from mlcomp_amd.train.native_generic_step import NativeGenericStep

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv1 = nn.Conv2d(3, 16, 3, padding=1)
            self.bn1 = nn.BatchNorm2d(16, affine=False)
            self.conv2 = nn.Conv2d(16, 16, 3, padding=1)
            self.bn2 = nn.BatchNorm2d(16)
            self.fc = nn.Linear(16, 10)

        def forward(self, x):
            x = F.relu(self.bn1(self.conv1(x)))
            x = F.relu(self.bn2(self.conv2(x)))
            return self.fc(x.mean((2, 3)))

    torch.manual_seed(0)
    m = Net()
    for p in list(m.conv1.parameters()) + list(m.bn2.parameters()):
        p.requires_grad_(False)
    x, y = torch.randn(4, 3, 8, 8), torch.randint(0, 10, (4,))
    step = NativeGenericStep(m, x, y, device='cpu', use_graph=False, optimizer='SGD', lr=0.1, momentum=0.9,
                             weight_decay=0.1)
    by = step.net.arena.by_name
    before = {k: s.master.clone() for k, s in by.items()}
    step()
    frozen = {k for k, s in by.items() if s.frozen}
    # (conv1.bias has no slot: a bias in front of a batch-statistics BN only shifts its mean)
    assert {'conv1.weight', 'bn1.weight', 'bn1.bias', 'bn2.weight', 'bn2.bias'} <= frozen, frozen
    for k, s in by.items():
        moved = not torch.equal(s.master, before[k])
        assert moved != (k in frozen), (k, moved)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_make(world, rank):
    from mlcomp_amd.train.native_generic_step import NativeGenericStep
    torch.manual_seed(0)
    m = build_model('resnext50_32x4d', num_classes=10)
    g = torch.Generator().manual_seed(100 + rank)
    x, y = torch.randn(2, 3, 32, 32, generator=g), torch.randint(0, 10, (2,), generator=g)
    return NativeGenericStep(m, x, y, device='cpu', world_size=world, use_graph=False, optimizer='SGD', lr=0.1,
                             momentum=0.9, weight_decay=1e-4)


def _flat(step, what):
    return torch.cat([getattr(a, what).detach().flatten().clone() for a in step.net.arena.arenas()])


def _dp_worker(rank, world, port, out):
    import torch.distributed as dist
    torch.set_num_threads(1)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    step = _dp_make(world, rank)
    step()
    torch.save({'g': _flat(step, 'grad'), 'w': _flat(step, 'master')}, os.path.join(out, f'r{rank}.pt'))
    dist.destroy_process_group()


def test_generic_data_parallel_equals_sum_of_shards(tmp_path):
    """ResNeXt-50 (grouped convs) on the generic engine over 2 gloo ranks with different data:
    the all-reduced gradient arena is the sum of the per-shard single-process gradients and
    the weights are one optimizer step on their mean, identical on both ranks."""
    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        mp.spawn(_dp_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2)
        got = [torch.load(tmp_path / f'r{r}.pt', weights_only=True) for r in range(2)]
        gsum = None
        for r in range(2):
            ref = _dp_make(1, r)
            ref()
            g = _flat(ref, 'grad')
            gsum = g if gsum is None else gsum + g
        scale = gsum.abs().max()
        for r in range(2):
            assert torch.allclose(got[r]['g'], gsum, rtol=1e-4, atol=1e-5 * scale)
            assert torch.equal(got[r]['w'], got[0]['w'])
    finally:
        torch.set_num_threads(threads)


def test_runner_picks_the_generic_engine_with_a_reason_for_the_rest(monkeypatch, tmp_path):
    from mlcomp_amd.train.experiment import ConfigExperiment
    from mlcomp_amd.train.runner import Runner, _native_kind
    assert _native_kind(build_model('LeNet', num_classes=10), torch.device('cuda')) == 'generic'
    assert _native_kind(build_model('efficientnet-b0', num_classes=10), torch.device('cuda')) == 'generic'

    class Odd(nn.Module):
        def __init__(self):
            super().__init__()
            self.c = nn.Conv2d(3, 8, 3, padding=1, padding_mode='reflect')

        def forward(self, x):
            return self.c(x).mean((2, 3))

    cfg = {'model_params': {'model': 'LeNet', 'num_classes': 10}, 'args': {'logdir': str(tmp_path)},
           'stages': {'optimizer_params': {'optimizer': 'Adam', 'lr': 1e-3}, 'stage1': {}}}
    r = Runner(ConfigExperiment(cfg), device='cpu')
    r.model = Odd()
    r.device = torch.device('cuda')      # selection only
    got = r._select_engine('stage1')
    assert got['engine'] == 'torch' and 'padding_mode' in got['reason'], got
    r.model = build_model('LeNet', num_classes=10)
    got = r._select_engine('stage1')
    assert got == {'stage': 'stage1', 'engine': 'native', 'kind': 'generic', 'precision': 'bf16', 'reason': None}


def test_act_codes_reference_derivatives():
    """The CPU references of the 10 activation codes and their derivatives (what the GPU
    tests compare the kernels against) agree with torch autograd."""
    a = torch.linspace(-7, 7, 1001)
    for name, code in Fn.ACT.items():
        if code == 0:
            continue
        x = a.clone().requires_grad_()
        Fn.act_ref(x, code, 0.3).sum().backward()
        g = Fn.act_grad_ref(a, code, 0.3)
        keep = (a.abs() > 1e-3) & ((a.abs() - 3).abs() > 1e-3) & ((a - 6).abs() > 1e-3)   # kinks
        assert torch.allclose(g[keep], x.grad[keep], atol=1e-5), name


class _UpNet(nn.Module):
    """LinkNet-style up path: 4x4 / stride-2 transposed conv + BN + ReLU, a 3x3 stride-2
    transposed conv with output padding and a bias (no BN), odd channel counts."""

    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 20, 3, 2, 1)
        self.up1 = nn.ConvTranspose2d(20, 12, 4, 2, 1)
        self.bn1 = nn.BatchNorm2d(12)
        self.up2 = nn.ConvTranspose2d(12, 5, 3, 2, 1, output_padding=1)

    def forward(self, x):
        x = F.relu(self.conv(x))
        x = F.relu(self.bn1(self.up1(x)))
        return self.up2(x)


def test_transposed_conv_sites_match_fp32_autograd():
    m, ref = _pair(_UpNet)
    x = torch.randn(4, 3, 16, 16)
    net = GenericNet(m, 'cpu')
    out = net(x)
    want = ref(x)
    assert out.shape == want.shape == (4, 5, 32, 32)
    g = torch.randn_like(want)
    (out.float() * g).sum().backward()
    (want * g).sum().backward()
    assert _rel(out, want) < 2e-2
    kinds = {p.name: getattr(p, 'kind', None) for p in net.param_sets()}
    assert kinds['up1'] == 'tr' and kinds['up2'] == 'tr'
    for p in net.param_sets():
        gg = p.w.grad if hasattr(p, 'w') else p.gamma.grad
        assert _cos(gg, _torch_grad(p, ref)) > 0.98, p.name
        if getattr(p, 'b', None) is not None:
            bb = dict(ref.named_modules())[p.name].bias.grad
            assert _cos(p.b.grad[:bb.numel()], bb) > 0.98, p.name
    # round trip of the transposed filters through the arena layout
    net.export_to_torch()
    assert torch.allclose(m.up2.weight, ref.up2.weight)


class _UpcatNet(nn.Module):
    """A two-level decoder: nearest x2 + concat with a skip (one with 5 / 3 channels, the
    other with multiples of 8), a standalone nearest x2, bilinear (align_corners) by scale
    and by a traced size."""

    def __init__(self):
        super().__init__()
        self.enc = nn.Conv2d(3, 16, 3, 2, 1)
        self.mid = nn.Conv2d(16, 5, 3, 2, 1)
        self.dec1 = nn.Conv2d(5 + 16, 8, 3, 1, 1)
        self.dec2 = nn.Conv2d(8 + 3, 8, 3, 1, 1)
        self.head = nn.Conv2d(8, 8, 1)

    def forward(self, x):
        e = torch.relu(self.enc(x))                                       # 16 @ H/2
        m = torch.relu(self.mid(e))                                       # 5 @ H/4
        d = F.interpolate(m, scale_factor=2, mode='nearest')
        d = torch.relu(self.dec1(torch.cat([d, e], 1)))                   # 8 @ H/2
        d = torch.cat([F.interpolate(d, scale_factor=2, mode='nearest'), x], 1)
        d = torch.relu(self.dec2(d))                                      # 8 @ H
        h = self.head(F.interpolate(d, scale_factor=2, mode='nearest'))   # 8 @ 2H
        h = F.interpolate(h, scale_factor=0.5, mode='bilinear', align_corners=True)
        return F.interpolate(h, size=x.shape[-2:], mode='bilinear', align_corners=True)


def test_upsample_concat_sites_match_fp32_autograd():
    """nearest x2 [+ concat] lowers to UpCat and bilinear (align_corners) to BilinearUp;
    forward and every gradient match the fp32 torch graph."""
    m, ref = _pair(_UpcatNet)
    net = GenericNet(m, 'cpu')
    kinds = [type(s).__name__ for s in net.train_gm.modules()]
    assert kinds.count('UpCat') == 3 and kinds.count('BilinearUp') == 2, kinds
    assert not [n for n in net.train_gm.graph.nodes if n.op == 'call_function' and n.target is torch.cat]
    x = torch.randn(2, 3, 16, 16)
    xi, xr = x.clone().requires_grad_(), x.clone().requires_grad_()
    out, want = net(xi), ref(xr)
    assert out.shape == want.shape == (2, 8, 16, 16)
    g = torch.randn_like(want)
    (out.float() * g).sum().backward()
    (want * g).sum().backward()
    assert _rel(out, want) < 2e-2
    assert _cos(xi.grad, xr.grad) > 0.98
    for p in net.param_sets():
        assert _cos(p.w.grad, _torch_grad(p, ref)) > 0.98, p.name


class _SENet(nn.Module):
    """Squeeze-excitation twice: EfficientNet's form (the gate multiplies its source) with 20
    channels (not a multiple of 8) and SE-ResNeXt's form (gate first) with 32."""

    def __init__(self):
        super().__init__()
        self.c1 = nn.Conv2d(3, 20, 3, 1, 1)
        self.se1 = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(20, 5, 1), nn.SiLU(), nn.Conv2d(5, 20, 1),
                                 nn.Sigmoid())
        self.c2 = nn.Conv2d(20, 32, 3, 2, 1)
        self.fc1, self.fc2 = nn.Conv2d(32, 8, 1), nn.Conv2d(8, 32, 1)
        self.head = nn.Linear(32, 6)

    def forward(self, x):
        y = F.silu(self.c1(x))
        y = y * self.se1(y)
        z = torch.relu(self.c2(y))
        g = torch.sigmoid(self.fc2(torch.relu(self.fc1(F.adaptive_avg_pool2d(z, 1)))))
        z = g * z
        return self.head(F.adaptive_avg_pool2d(z, 1).flatten(1))


def test_squeeze_excitation_gates_match_fp32_autograd():
    m, ref = _pair(_SENet)
    net = GenericNet(m, 'cpu')
    kinds = [type(s).__name__ for s in net.train_gm.modules()]
    assert kinds.count('ChannelGate') == 2, kinds
    x = torch.randn(4, 3, 12, 12)
    xi, xr = x.clone().requires_grad_(), x.clone().requires_grad_()
    out, want = net(xi), ref(xr)
    g = torch.randn_like(want)
    (out.float() * g).sum().backward()
    (want * g).sum().backward()
    assert _rel(out, want) < 2e-2
    assert _cos(xi.grad, xr.grad) > 0.98
    for p in net.param_sets():
        gg = p.w.grad if hasattr(p, 'w') else p.gamma.grad
        assert _cos(gg, _torch_grad(p, ref)) > 0.98, p.name


class _SampleGateNet(nn.Module):
    """A per-sample gate ([N, 1, 1, 1]) computed from the value's global average: a valid
    torch broadcast that is not a per-channel gate, so it must stay a torch op."""

    def __init__(self):
        super().__init__()
        self.c1 = nn.Conv2d(3, 16, 3, 1, 1)
        self.fc = nn.Conv2d(16, 1, 1)
        self.head = nn.Linear(16, 4)

    def forward(self, x):
        y = torch.relu(self.c1(x))
        y = y * torch.sigmoid(self.fc(F.adaptive_avg_pool2d(y, 1)))
        return self.head(F.adaptive_avg_pool2d(y, 1).flatten(1))


def test_per_sample_gate_stays_a_torch_op():
    m, ref = _pair(_SampleGateNet)
    net = GenericNet(m, 'cpu')
    kinds = [type(s).__name__ for s in net.train_gm.modules()]
    assert 'ChannelGate' not in kinds, kinds
    x = torch.randn(3, 3, 8, 8)
    out, want = net(x), ref(x)
    assert _rel(out, want) < 2e-2


class _DropPathNet(nn.Module):
    """Residual blocks ending in conv -> BN -> stochastic depth -> + x (EfficientNet's MBConv)."""

    def __init__(self):
        super().__init__()
        self.stem = nn.Conv2d(3, 16, 3, 1, 1)
        self.blocks = nn.ModuleList([nn.Sequential(nn.Conv2d(16, 32, 1), nn.BatchNorm2d(32), nn.SiLU(),
                                                   nn.Conv2d(32, 16, 1, bias=False), nn.BatchNorm2d(16))
                                     for _ in range(2)])
        self.head = nn.Linear(16, 5)

    def forward(self, x):
        x = self.stem(x)
        for i, b in enumerate(self.blocks):
            y = b(x)
            keep = 0.75 - 0.25 * i
            mask = torch.rand_like(y[:, :1, :1, :1].float()) < keep   # fp32 draws in both graphs
            x = y * mask / keep + x
        return self.head(F.adaptive_avg_pool2d(x, 1).flatten(1))


def test_drop_path_residual_folds_into_the_bn_site():
    """stochastic depth + residual add lower into the block's last conv+BN site (mask / keep
    applied in its BN pass); the same RNG draws give the torch graph's output and gradients."""
    m, ref = _pair(_DropPathNet)
    net = GenericNet(m, 'cpu')
    sites = list(net.train_gm.modules())
    assert sum(getattr(s, 'drop_keep', None) is not None for s in sites) == 2
    assert not [n for n in net.train_gm.graph.nodes if n.op == 'call_function' and n.target is operator.truediv]
    x = torch.randn(8, 3, 8, 8)
    torch.manual_seed(11)
    out = net(x)
    torch.manual_seed(11)
    want = ref(x)
    g = torch.randn_like(want)
    (out.float() * g).sum().backward()
    (want * g).sum().backward()
    assert _rel(out, want) < 2e-2
    for p in net.param_sets():
        gg = p.w.grad if hasattr(p, 'w') else p.gamma.grad
        assert _cos(gg, _torch_grad(p, ref)) > 0.98, p.name


def test_linknet_lowers_completely():
    from mlcomp_amd.contrib.segmentation.models import Linknet
    assert lower_or_none(Linknet(encoder_name='resnet34', classes=1)) is None


@pytest.mark.parametrize('kw', [
    dict(residual_transformation_type='postactivated_bottleneck_transformation', num_groups=2, width_per_group=8),
    dict(residual_transformation_type='basic_transformation'),
    dict(residual_transformation_type='basic_r2plus1d_transformation', stem_name='r2plus1d_stem', stem_maxpool=True),
    dict(residual_transformation_type='preactivated_bottleneck_transformation',
         skip_transformation_type='preactivated_shortcut', stem_maxpool=True)])
def test_video_resnext3d_lowers_and_matches_fp32_autograd(kw):
    """The reference's 3D video models (ResNeXt3D / R(2+1)D stems, bottleneck / basic /
    R(2+1)D blocks, pre- and post-activated shortcuts; `mlcomp/contrib/model/video/
    resnext3d/resnext3d_stem.py:68-80`, `r2plus1_util.py:53-65`): every Conv3d / BatchNorm3d /
    MaxPool3d becomes a native site (temporal taps unfolded into channels, the 2D kernels
    over N*T frames); output and every conv weight gradient against fp32 autograd."""
    from mlcomp_amd.contrib.video import ResNeXt3D
    cfg = dict(num_blocks=(1, 1), stem_planes=16, stage_planes=16, stage_temporal_kernel_basis=([3], [3]),
               temporal_conv_1x1=(False, True), stage_temporal_stride=(1, 2), stage_spatial_stride=(1, 2),
               in_plane=32, num_classes=5, stem_spatial_kernel=3)
    cfg.update(kw)
    m, ref = _pair(lambda: ResNeXt3D(**cfg))
    assert lower_or_none(m) is None
    net = GenericNet(m, 'cpu')
    left = [type(mod).__name__ for mod in net.train_gm.modules()
            if isinstance(mod, (nn.Conv3d, nn.BatchNorm3d, nn.MaxPool3d, nn.Linear, nn.AdaptiveAvgPool1d))]
    assert not left, left
    # the head's AdaptiveAvgPool1d over the flattened [N, 1, C*T*H*W] is a global pool per channel
    assert any(type(mod).__name__ == 'VolumePool' for mod in net.train_gm.modules())
    x = torch.randn(4, 3, 4, 16, 16)
    y = torch.randint(0, 5, (4,))
    out = net(x)
    F.cross_entropy(out.float(), y).backward()
    want = ref(x)
    F.cross_entropy(want, y).backward()
    assert _rel(out, want) < 2e-2
    mods = dict(ref.named_modules())
    n = 0
    for p in net.param_sets():
        if not hasattr(p, 'kind'):
            continue
        g3 = mods[p.name].weight.grad
        g = g3.reshape(p.src.weight.shape)          # [Co, Cg*kt, kh, kw], as the lowering sees it
        if p.kind == 'dense':
            want_g = F.pad(g.permute(0, 2, 3, 1), (0, p.Cip - p.Ci, 0, 0, 0, 0, 0, p.Cop - p.Co))
        elif p.kind == 'dw':
            want_g = F.pad(g[:, 0].permute(1, 2, 0), (0, p.Cop - p.Co))
        else:
            want_g = g.permute(0, 2, 3, 1)
        # bf16 activations through 6-10 BatchNorms over a few frames (and bf16 max-pool
        # argmaxes): directions, not per-element magnitudes (a layout bug gives cos << 0.9)
        assert _cos(p.w.grad, want_g) > 0.95, p.name
        n += 1
    assert n >= 6
    # eval graph: running statistics, deterministic
    net.eval()
    ref.eval()
    with torch.no_grad():
        assert _rel(net(x), ref(x)) < 5e-2


def test_video_residual_gradients_are_handed_off_not_added(monkeypatch):
    """ResNeXt3D blocks: the identity residual's gradient and the shortcut conv's input
    gradient are handed to the block's first Conv3d site (Frames.grad_expected) and summed in
    its temporal fold (native) / one add (here) instead of by autograd; the gradients equal
    the unlinked lowering's."""
    from mlcomp_amd.contrib.video import ResNeXt3D
    from mlcomp_amd.models.native_generic import _Lowering as NativeLowering
    from mlcomp_amd.ops.glayers import Frames
    cfg = dict(residual_transformation_type='basic_transformation', num_blocks=(2, 2), stem_planes=16,
               stage_planes=16, stage_temporal_kernel_basis=([3], [3]), temporal_conv_1x1=(False, False),
               stage_temporal_stride=(1, 2), stage_spatial_stride=(1, 2), in_plane=32, num_classes=5,
               stem_spatial_kernel=3)
    x = torch.randn(2, 3, 4, 16, 16)
    y = torch.randint(0, 5, (2,))

    def run(linked):
        torch.manual_seed(0)
        if not linked:
            monkeypatch.setattr(NativeLowering, '_link_frames', lambda self: None)
        net = GenericNet(ResNeXt3D(**cfg), 'cpu')
        monkeypatch.undo()
        fr = [m for m in net.train_gm.modules() if isinstance(m, Frames)]
        links = (sum(m.grad_expected for m in fr), sum(m.send_to is not None for m in fr),
                 sum(getattr(m.site, 'res_link', None) is not None for m in fr))
        F.cross_entropy(net(x).float(), y).backward()
        return links, [p.w.grad.clone() for p in net.param_sets() if hasattr(p, 'kind')]

    links, g1 = run(True)
    nolinks, g0 = run(False)
    assert links == (4, 1, 3), links          # 3 identity residuals + 1 shortcut, 4 receivers
    assert nolinks == (0, 0, 0)
    for a, b in zip(g1, g0):
        assert torch.allclose(a, b, rtol=1e-3, atol=1e-5)


def test_conv1d_bn1d_lowers_and_matches_fp32_autograd():
    """nn.Conv1d [-> BatchNorm1d -> ReLU] through the same temporal unfold (a Conv1d is a
    Conv3d with a 1x1 spatial kernel)."""
    class Net1d(nn.Module):
        def __init__(self):
            super().__init__()
            self.c1 = nn.Conv1d(8, 16, 5, stride=2, padding=2, bias=False)
            self.b1 = nn.BatchNorm1d(16)
            self.c2 = nn.Conv1d(16, 16, 3, padding=2, dilation=2)
            self.fc = nn.Linear(16, 4)

        def forward(self, x):
            x = F.relu(self.b1(self.c1(x)))
            x = F.relu(self.c2(x))
            return self.fc(x.mean(2))

    m, ref = _pair(Net1d)
    net = GenericNet(m, 'cpu')
    x = torch.randn(4, 8, 40)
    out = net(x)
    out.float().sum().backward()
    want = ref(x)
    want.sum().backward()
    assert _rel(out, want) < 2e-2
    for name in ('c1', 'c2'):
        p = [q for q in net.param_sets() if q.name == name][0]
        g = getattr(ref, name).weight.grad.reshape(p.src.weight.shape)
        want_g = F.pad(g.permute(0, 2, 3, 1), (0, p.Cip - p.Ci, 0, 0, 0, 0, 0, p.Cop - p.Co))
        assert _cos(p.w.grad, want_g) > 0.98, name


def test_identity_residual_and_bn_backward_links_are_exact():
    """ResNet basic blocks: the identity residual's gradient is handed from the block's last
    conv site to its first conv site's dgrad epilogue (one gradient per value, no autograd
    sum); a downsample block's shortcut conv hands its input gradient to the block's first
    conv the same way and applies the folded BN of the block's last conv as its residual's
    affine; a conv site whose input is another conv site's BN(-ReLU) output computes that
    BN's (and its folded partner's) backward reduction and ReLU mask in its dgrad epilogue
    (no reduction pass).  Input and weight gradients equal the unlinked ones and match fp32
    autograd."""
    m, ref = _pair(lambda: build_model('resnet18', num_classes=10))
    net = GenericNet(m, 'cpu')
    sites = list(net.train_gm.modules())
    links = [s for s in sites if getattr(s, 'res_link', None) is not None]
    assert len(links) == 5, len(links)            # 8 blocks, 3 of them with a downsample shortcut
    glinks = [s for s in sites if getattr(s, 'grad_link', None) is not None]
    folds = [s for s in sites if getattr(s, 'res_bn', None) is not None]
    assert len(glinks) == 3 and len(folds) == 3, (len(glinks), len(folds))
    # the stem's conv -> BN -> ReLU -> max-pool runs as one fused site
    assert sum(bool(getattr(s, 'pool3', False)) for s in sites) == 1
    bn_links = [s for s in sites if getattr(s, 'bn_link', None) is not None]
    # each block's second conv reads its first conv's BN-ReLU (8); the first conv of every
    # block after layer1.0 (whose input is the max-pool's output) also reads the previous
    # block's output, whose other gradient (identity residual or shortcut conv) it sums (7)
    assert len(bn_links) == 15, len(bn_links)
    torch.manual_seed(3)
    x = torch.randn(4, 3, 32, 32)
    y = torch.randint(0, 10, (4,))

    def run(linked):
        for s in links:
            object.__setattr__(s, '_saved_link', getattr(s, '_saved_link', s.res_link))
            object.__setattr__(s, 'res_link', s._saved_link if linked else None)
        for s in glinks:
            object.__setattr__(s, '_saved_glink', getattr(s, '_saved_glink', s.grad_link))
            object.__setattr__(s, 'grad_link', s._saved_glink if linked else None)
            object.__setattr__(s._saved_glink, 'grad_expected', linked)
        for s in folds:
            object.__setattr__(s, '_saved_fold', getattr(s, '_saved_fold', s.res_bn))
            object.__setattr__(s, 'res_bn', s._saved_fold if linked else None)
            object.__setattr__(s._saved_fold, 'bn_folded', linked)
            object.__setattr__(s._saved_fold, 'bn_prereduced', linked)
        for s in bn_links:
            object.__setattr__(s, '_saved_bn', getattr(s, '_saved_bn', s.bn_link))
            object.__setattr__(s, 'bn_link', s._saved_bn if linked else None)
            object.__setattr__(s._saved_bn, 'bn_prereduced', linked)
        net.ctx.ws.zero()                 # what the step does first (BN reduction scratch)
        net.arena.zero_grad()
        xi = x.clone().requires_grad_()
        F.cross_entropy(net(xi).float(), y).backward()
        return xi.grad.clone(), [(p.w if hasattr(p, 'w') else p.gamma).grad.clone() for p in net.param_sets()]
    gx_l, gw_l = run(True)
    # the fused path ran for every link and every folded shortcut BN
    assert sum(getattr(s._saved_bn, 'n_prereduced', 0) for s in bn_links) == 15
    assert sum(getattr(s._saved_fold, 'n_prereduced', 0) for s in folds) == 3
    gx_u, gw_u = run(False)
    assert sum(getattr(s._saved_bn, 'n_prereduced', 0) for s in bn_links) == 15
    assert sum(getattr(s._saved_fold, 'n_prereduced', 0) for s in folds) == 3
    assert _rel(gx_l, gx_u) < 1e-2
    for a, b in zip(gw_l, gw_u):
        assert _rel(a, b) < 1e-2
    xr = x.clone().requires_grad_()
    F.cross_entropy(ref(xr), y).backward()
    assert _cos(gx_l, xr.grad) > 0.98


class _AvgPoolNet(nn.Module):
    """Inception's 3x3/1 pad-1 branch pool (functional), a DenseNet 2x2/2 transition (module),
    and a 3x3/2 pad-1 pool without the padding in the divisor, on 20 channels."""

    def __init__(self):
        super().__init__()
        self.c1 = nn.Conv2d(3, 20, 3, 1, 1)
        self.b1 = nn.BatchNorm2d(20)
        self.trans = nn.AvgPool2d(2, 2)
        self.c2 = nn.Conv2d(20, 16, 1)
        self.head = nn.Linear(16, 6)

    def forward(self, x):
        y = torch.relu(self.b1(self.c1(x)))
        y = F.avg_pool2d(y, kernel_size=3, stride=1, padding=1) + y
        y = self.trans(y)
        y = F.avg_pool2d(self.c2(y), 3, 2, 1, count_include_pad=False)
        return self.head(F.adaptive_avg_pool2d(y, 1).flatten(1))


def test_average_pools_lower_and_match_fp32_autograd():
    m, ref = _pair(_AvgPoolNet)
    net = GenericNet(m, 'cpu')
    kinds = [type(s).__name__ for s in net.train_gm.modules()]
    assert kinds.count('AvgPool') == 3, kinds
    x = torch.randn(4, 3, 13, 15)
    xi, xr = x.clone().requires_grad_(), x.clone().requires_grad_()
    out, want = net(xi), ref(xr)
    g = torch.randn_like(want)
    (out.float() * g).sum().backward()
    (want * g).sum().backward()
    assert _rel(out, want) < 2e-2
    assert _cos(xi.grad, xr.grad) > 0.98
    for p in net.param_sets():
        gg = p.w.grad if hasattr(p, 'w') else p.gamma.grad
        assert _cos(gg, _torch_grad(p, ref)) > 0.98, p.name


def test_adaptive_avg_pool_sizes_lower_natively():
    """AdaptiveAvgPool2d / F.adaptive_avg_pool2d to sizes > 1 (PSPNet's pyramid, overlapping
    bins when the size does not divide the input) lower to the native AdaptiveAvgPool site;
    output and input gradient against fp32 autograd."""
    from mlcomp_amd.ops.glayers import AdaptiveAvgPool

    class Pyr(nn.Module):
        def __init__(self):
            super().__init__()
            self.c = nn.Conv2d(3, 16, 3, padding=1)
            self.p = nn.AdaptiveAvgPool2d(6)

        def forward(self, x):
            y = self.c(x)
            return self.p(y).flatten(1).sum(1) + F.adaptive_avg_pool2d(y, (3, 3)).flatten(1).sum(1)

    m, ref = _pair(Pyr)
    net = GenericNet(m, 'cpu')
    assert sum(isinstance(mod, AdaptiveAvgPool) for mod in net.train_gm.modules()) == 2
    x = torch.randn(2, 3, 16, 16)
    out = net(x)
    out.float().sum().backward()
    want = ref(x)
    want.sum().backward()
    assert _rel(out, want) < 2e-2
    for p in net.param_sets():
        gg = p.w.grad if hasattr(p, 'w') else p.gamma.grad
        assert _cos(gg, _torch_grad(p, ref)) > 0.98, p.name


def test_branch_point_gradients_summed_in_the_consumers(monkeypatch):
    """An Inception-style branch point (one activation feeding three convs and an average
    pool) shares a GradAcc: the running sum of the input gradient passes through the
    consumers' dgrad epilogues / pool backward in whatever order autograd runs them, and the
    result equals the unlinked lowering's (autograd's adds) and fp32 autograd's direction."""
    from mlcomp_amd.models.native_generic import _Lowering
    from mlcomp_amd.ops.glayers import GradAcc

    class Block(nn.Module):
        def __init__(self):
            super().__init__()
            self.stem = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1, bias=False), nn.BatchNorm2d(16), nn.ReLU())
            self.b1 = nn.Sequential(nn.Conv2d(16, 8, 1, bias=False), nn.BatchNorm2d(8), nn.ReLU())
            self.b2 = nn.Sequential(nn.Conv2d(16, 8, 1, bias=False), nn.BatchNorm2d(8), nn.ReLU(),
                                    nn.Conv2d(8, 8, 3, padding=1, bias=False), nn.BatchNorm2d(8), nn.ReLU())
            self.b3 = nn.Sequential(nn.Conv2d(16, 8, 3, padding=1, bias=False), nn.BatchNorm2d(8), nn.ReLU())
            self.b4 = nn.Sequential(nn.AvgPool2d(3, 1, 1), nn.Conv2d(16, 8, 1, bias=False), nn.BatchNorm2d(8), nn.ReLU())
            self.head = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(32, 5))

        def forward(self, x):
            x = self.stem(x)
            return self.head(torch.cat([self.b1(x), self.b2(x), self.b3(x), self.b4(x)], 1))

    x = torch.randn(2, 3, 12, 12)
    y = torch.randint(0, 5, (2,))

    handed = []
    give = GradAcc.give

    def counting_give(self, dx):
        r = give(self, dx)
        handed.append(r is None)
        return r

    def run(linked):
        torch.manual_seed(0)
        if not linked:
            monkeypatch.setattr(_Lowering, '_link_fanout', lambda self: None)
        net = GenericNet(Block(), 'cpu')
        monkeypatch.undo()
        monkeypatch.setattr(GradAcc, 'give', counting_give)
        accs = {id(m.acc) for m in net.train_gm.modules() if getattr(m, 'acc', None) is not None}
        F.cross_entropy(net(x).float(), y).backward()
        monkeypatch.undo()
        return len(accs), [p.w.grad.clone() for p in net.param_sets() if hasattr(p, 'kind')]

    n1, g1 = run(True)
    # three of the four consumers hand their sum on, the last returns it to autograd
    assert sorted(handed) == [False, True, True, True], handed
    n0, g0 = run(False)
    assert (n1, n0) == (1, 0)
    # the same sum in another association: bf16 roundings of the partial sums differ
    for a, b in zip(g1, g0):
        assert _rel(a, b) < 3e-2 and _cos(a, b) > 0.999
    assert GradAcc('t').give(torch.zeros(1)) is not None     # no forward counted: passes through


def test_se_block_input_gradient_summed_in_pool_and_gate(monkeypatch):
    """A squeeze-excitation block's input feeds its global pool and its gate multiply: the
    pool backward and the gate backward kernels share a GradAcc (no autograd add), with the
    gradients of the unlinked lowering."""
    from mlcomp_amd.models.native_generic import _Lowering
    from mlcomp_amd.ops.glayers import GradAcc

    class SE(nn.Module):
        def __init__(self):
            super().__init__()
            self.c = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1, bias=False), nn.BatchNorm2d(16), nn.SiLU())
            self.g = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(16, 4, 1), nn.SiLU(), nn.Conv2d(4, 16, 1),
                                   nn.Sigmoid())
            self.h = nn.Sequential(nn.Conv2d(16, 8, 1, bias=False), nn.BatchNorm2d(8), nn.AdaptiveAvgPool2d(1),
                                   nn.Flatten(), nn.Linear(8, 5))

        def forward(self, x):
            y = self.c(x)
            return self.h(y * self.g(y))

    x = torch.randn(2, 3, 10, 10)
    t = torch.randint(0, 5, (2,))
    handed = []
    give = GradAcc.give

    def counting_give(self, dx):
        r = give(self, dx)
        handed.append(r is None)
        return r

    def run(linked):
        torch.manual_seed(0)
        if not linked:
            monkeypatch.setattr(_Lowering, '_link_fanout', lambda self: None)
        net = GenericNet(SE(), 'cpu')
        monkeypatch.undo()
        monkeypatch.setattr(GradAcc, 'give', counting_give)
        F.cross_entropy(net(x).float(), t).backward()
        monkeypatch.undo()
        return [p.w.grad.clone() for p in net.param_sets() if hasattr(p, 'kind')]

    g1 = run(True)
    assert sorted(handed) == [False, True], handed
    g0 = run(False)
    for a, b in zip(g1, g0):
        assert _rel(a, b) < 3e-2 and _cos(a, b) > 0.999


def test_dense_block_bn_statistics_reuse_the_previous_layers(monkeypatch):
    """DenseNet's BN over cat([x_i, f_i]): the site copies x_i's per-channel sums from the
    previous layer's BN and reduces only the new channels (BNAct.cat_prev), and the concat's
    backward hands x_i's gradient slice to that BN's apply pass (DenseCat); output, running
    statistics and weight gradients equal the plain lowering's.  The block's concatenations
    share one buffer (DenseChain): each BN reads its input as the buffer's leading channels."""
    from mlcomp_amd.contrib.segmentation.encoders import _DenseLayer
    from mlcomp_amd.models.native_generic import _Lowering
    from mlcomp_amd.ops.glayers import BNAct, DenseCat

    class Dense(nn.Module):
        def __init__(self):
            super().__init__()
            self.stem = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1, bias=False), nn.BatchNorm2d(16), nn.ReLU())
            self.layers = nn.Sequential(_DenseLayer(16, 8, 2), _DenseLayer(24, 8, 2), _DenseLayer(32, 8, 2))
            self.final = nn.BatchNorm2d(40)
            self.head = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(40, 5))

        def forward(self, x):
            return self.head(torch.relu(self.final(self.layers(self.stem(x)))))

    x = torch.randn(2, 3, 12, 12)
    y = torch.randint(0, 5, (2,))

    def run(linked):
        torch.manual_seed(0)
        if not linked:
            monkeypatch.setattr(_Lowering, '_link_cat_stats', lambda self: None)
            monkeypatch.setattr(_Lowering, '_lower_dense_cats', lambda self: None)
        net = GenericNet(Dense(), 'cpu')
        monkeypatch.undo()
        k = sum(isinstance(m, BNAct) and m.cat_prev is not None for m in net.train_gm.modules())
        k += 10 * sum(isinstance(m, DenseCat) for m in net.train_gm.modules())
        k += 100 * sum(isinstance(m, DenseCat) and m.chain is not None for m in net.train_gm.modules())
        k += 1000 * sum(getattr(m, 'cat_out', None) is not None for m in net.train_gm.modules())
        k += 10000 * sum(isinstance(m, BNAct) and m.split_to is not None for m in net.train_gm.modules())
        out = net(x)
        F.cross_entropy(out.float(), y).backward()
        rv = [m.bn.run_var.clone() for m in net.train_gm.modules() if isinstance(m, BNAct)]
        return k, out.detach(), rv, [p.w.grad.clone() for p in net.param_sets() if hasattr(p, 'kind')]

    k1, o1, r1, g1 = run(True)
    k0, o0, r0, g0 = run(False)
    # 3 concat-statistics BNs (layers 2, 3, final), 3 DenseCats sharing one concat buffer, into
    # which the 3 growth convs write their outputs (on the GPU); the BN after each concat stores
    # its input gradient split into the concat's two operand gradients
    assert (k1, k0) == (33333, 0)
    assert _rel(o1, o0) < 1e-2
    for a, b in zip(r1, r0):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-6)
    for a, b in zip(g1, g0):
        assert _rel(a, b) < 3e-2 and _cos(a, b) > 0.999
