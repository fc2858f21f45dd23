"""Data parallelism of the native engines on the GPU with two ranks sharing the one card.

RCCL refuses two ranks on one device, so the ranks talk through ``TorchComm`` over gloo
(CUDA tensors staged through the host).  Everything else is the production path: the
gradient bucketer's side stream, the weight-gradient and shortcut streams, the arenas and
the fused optimizers, eager (a gloo collective cannot be captured into a HIP graph).  Each
rank draws different synthetic data; after the steps both ranks must hold identical
gradients and weights."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, kind, out):
    import torch.distributed as dist
    from mlcomp_amd.parallel.comm import TorchComm
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      HSA_ENABLE_IPC_MODE_LEGACY='0')
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.cuda.set_device(0)
    comm = TorchComm(rank, world)
    torch.manual_seed(0)
    common = dict(device='cuda', world_size=world, use_graph=False, comm=comm)
    if kind == 'resnet':
        from mlcomp_amd.train.native_step import NativeClassifierStep
        step = NativeClassifierStep('resnet50', batch=8, image_size=64, num_classes=10, **common)
    elif kind == 'unet':
        from mlcomp_amd.train.native_seg_step import NativeSegmentationStep
        step = NativeSegmentationStep('resnet18', batch=4, image_size=64, **common)
    else:
        from mlcomp_amd.train.native_bert_step import NativeBertStep
        step = NativeBertStep('bert-tiny', batch=8, seq_len=128, **common)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    arena = step.net.arena
    w = torch.cat([a.master.flatten() for a in arena.arenas()]).cpu()
    g = torch.cat([a.grad.flatten() for a in arena.arenas()]).cpu()
    torch.save({'w': w, 'g': g, 'loss': step.last_loss()}, os.path.join(out, f'{kind}{rank}.pt'))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('kind', ['resnet', 'unet', 'bert'])
def test_native_data_parallel_two_ranks_on_gpu(tmp_path, kind):
    mp.spawn(_worker, args=(2, _free_port(), kind, str(tmp_path)), nprocs=2)
    a = torch.load(tmp_path / f'{kind}0.pt', weights_only=True)
    b = torch.load(tmp_path / f'{kind}1.pt', weights_only=True)
    assert torch.isfinite(a['w']).all() and a['g'].abs().sum() > 0
    assert a['loss'] == a['loss'] and b['loss'] == b['loss']
    assert torch.equal(a['g'], b['g']), (a['g'] - b['g']).abs().max()
    assert torch.equal(a['w'], b['w']), (a['w'] - b['w']).abs().max()
