"""Data parallelism is CORRECT, not just consistent (verdict r2 #2): for each native
engine, world 2 and 4 gloo ranks with different data per rank.  After one step the
all-reduced gradient arena on every rank must equal the SUM of single-process gradients
of the per-rank shards (each shard's own BatchNorm batch statistics, as DDP without
SyncBN computes them), and the weights must equal a single-process optimizer step on the
averaged gradient (the 1/world scale folded into the optimizer).  BatchNorm running
statistics are rank 0's on every rank after the per-step buffer broadcast (SURVEY 2.11
C4).  A wrong grad scale, a bucket never reduced, or a bucket reduced twice fails here."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make(kind, world):
    torch.manual_seed(0)
    if kind == 'resnet':
        from mlcomp_amd.train.native_step import NativeClassifierStep
        return NativeClassifierStep('resnet18', batch=4, image_size=32, device='cpu', world_size=world,
                                    num_classes=10, use_graph=False, lr=0.05, momentum=0.9, weight_decay=1e-4)
    if kind == 'unet':
        from mlcomp_amd.train.native_seg_step import NativeSegmentationStep
        return NativeSegmentationStep('resnet18', batch=2, image_size=64, device='cpu', world_size=world,
                                      use_graph=False, lr=1e-3)
    if kind in ('linknet', 'fpn', 'pspnet'):
        from mlcomp_amd.contrib.segmentation.models import FPN, Linknet, PSPNet
        from mlcomp_amd.train.native_seg_step import NativeSegmentationStep
        tm = (Linknet(encoder_name='resnet18') if kind == 'linknet' else
              FPN(encoder_name='resnet18', dropout=0.0) if kind == 'fpn' else
              PSPNet(encoder_name='resnet18', classes=1, dropout=0.0))
        return NativeSegmentationStep(torch_model=tm, batch=2, image_size=64, device='cpu', world_size=world,
                                      use_graph=False, lr=1e-3)
    from mlcomp_amd.train.native_bert_step import NativeBertStep
    return NativeBertStep('bert-tiny', batch=4, seq_len=16, device='cpu', world_size=world, use_graph=False,
                          lr=1e-3)


def _flat(step, what):
    return torch.cat([getattr(a, what).detach().flatten().clone() for a in step.net.arena.arenas()])


def _bn(step):
    return step.bn_buffers.clone() if step.bn_buffers is not None else torch.zeros(0)


def _worker(rank, world, port, kind, out):
    import torch.distributed as dist
    # one intra-op thread: oneDNN's multi-threaded weight-gradient reductions schedule work
    # dynamically, so their summation order (and the last bits of every gradient) depends on
    # timing - under a loaded host (pytest -n 8) the rank results drifted 4e-4 from the
    # reference.  Single-threaded, both sides sum in one fixed order.
    torch.set_num_threads(1)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    step = _make(kind, world)
    step()
    torch.save({'g': _flat(step, 'grad'), 'w': _flat(step, 'master'), 'bn': _bn(step)},
               os.path.join(out, f'{kind}{rank}.pt'))
    dist.destroy_process_group()


@pytest.mark.parametrize('kind,world', [(k, w) for k in ('resnet', 'unet', 'bert') for w in (2, 4)]
                         + [('linknet', 2), ('fpn', 2), ('pspnet', 2)])
def test_dp_step_equals_single_process_on_the_shards(tmp_path, kind, world, monkeypatch):
    threads = torch.get_num_threads()
    torch.set_num_threads(1)      # the reference runs single-threaded too (see _worker)
    try:
        _check_dp(tmp_path, kind, world, monkeypatch)
    finally:
        torch.set_num_threads(threads)


def _check_dp(tmp_path, kind, world, monkeypatch):
    mp.spawn(_worker, args=(world, _free_port(), kind, str(tmp_path)), nprocs=world)
    got = [torch.load(tmp_path / f'{kind}{r}.pt', weights_only=True) for r in range(world)]
    # single process, one shard at a time (RANK selects the shard's synthetic data and
    # dropout stream, exactly as in the rank processes)
    gsum, bn0 = None, None
    for r in range(world):
        monkeypatch.setenv('RANK', str(r))
        ref = _make(kind, 1)
        ref()
        g = _flat(ref, 'grad')
        gsum = g if gsum is None else gsum + g
        if r == 0:
            bn0 = _bn(ref)
    scale = gsum.abs().max()
    for r in range(world):
        assert torch.allclose(got[r]['g'], gsum, rtol=1e-4, atol=1e-5 * scale), (kind, world, r)
        assert torch.equal(got[r]['w'], got[0]['w'])
        assert torch.equal(got[r]['bn'], got[0]['bn'])
    assert torch.allclose(got[0]['bn'], bn0, rtol=1e-5, atol=1e-6)     # rank 0's running stats
    # the update: one single-process optimizer step from the initial weights on sum/world
    monkeypatch.setenv('RANK', '0')
    ref = _make(kind, 1)
    for a, gs in zip(ref.net.arena.arenas(), torch.split(gsum, [a.grad.numel() for a in ref.net.arena.arenas()])):
        a.grad.copy_(gs.view_as(a.grad) / world)
    ref.opt.prepare()
    ref.opt.step()
    w = _flat(ref, 'master')
    # SGD (resnet) is linear in the gradient: tight.  Adam's first step is ~lr * g/|g|, which
    # turns summation-order noise of near-zero gradients into up to ~1e-5 (lr 1e-3)
    atol = 1e-6 if kind == 'resnet' else 3e-5
    assert torch.allclose(got[0]['w'], w, rtol=1e-4, atol=atol), (got[0]['w'] - w).abs().max()
