#!/usr/bin/env python
"""Headline benchmark: whole-node images/s of the ResNet-50 DAG train task.

Metric/config from BASELINE.json: "images/sec (whole node) ResNet-50 DAG train task at
1/2/4/8 MI355X", ImageNet-shape synthetic data (224x224x3, 1000 classes), random-init
weights.  One process per GPU (torchrun), data-parallel over RCCL; per-GPU batch is fixed
(weak scaling): 512 images by default (``--batch``; rounds 1-3 used 256).  A timed step is a full training step: forward, loss, backward, gradient
all-reduce, optimizer update.

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        bench.py --gpus 8 --steps 20 --warmup 5

``--impl native`` (default) runs the mlcomp_amd engine: NHWC bf16 activations, HIP
kernels for conv/BN/ReLU/optimizer/loss and the framework's own RCCL gradient bucketer.
``--impl torch`` runs stock PyTorch-ROCm (MIOpen convs, torch DDP) on the same model
and data, which is the measured comparison baseline (BASELINE.md has no published
number).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# the reference publishes no number (BASELINE.json "published": {}); the comparison
# baseline is the stock PyTorch-ROCm run measured on the same box (profiles/README.md)
BASELINE_VALUE = None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=50)
    p.add_argument('--warmup', type=int, default=10)
    p.add_argument('--batch', type=int, default=None,
                   help='per-GPU batch (ResNet-50 512 images, segmentation 32 images, BERT 32 sequences)')
    p.add_argument('--seq-len', type=int, default=128, help='BERT sequence length')
    p.add_argument('--model', default='resnet50')
    p.add_argument('--impl', default='native', choices=['native', 'torch'])
    p.add_argument('--image-size', type=int, default=224)
    p.add_argument('--graph', type=int, default=-1,
                   help='capture the step in a HIP graph (default: on for native)')
    p.add_argument('--json-out', default=None)
    p.add_argument('--data', default='synthetic', choices=['synthetic', 'records'],
                   help='records: feed the ResNet step from a record file through the native input '
                        'pipeline (C++ gather threads + GPU augment kernel) instead of a resident batch')
    p.add_argument('--records', default=None, help='record file for --data records (default: a generated one)')
    p.add_argument('--loader-threads', type=int, default=12)
    p.add_argument('--precision', default='bf16', choices=['bf16', 'fp32'],
                   help='fp32: --impl torch without autocast (the reference Catalyst default precision, which '
                        'the runner trains on the torch engine); the native engines are bf16 with fp32 master weights')
    p.add_argument('--comm', default='auto', choices=['auto', 'rccl1'],
                   help='rccl1: give a one-GPU run a world-1 RCCL communicator, so the production gradient '
                        'bucketer issues its RCCL all-reduces on the side stream (overlap evidence)')
    return p.parse_args()


def _world1_rccl(device):
    """A one-rank RCCL communicator over a private TCP store (``--comm rccl1``)."""
    import socket
    import torch.distributed as dist
    from mlcomp_amd.parallel.comm import RcclComm
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    store = dist.TCPStore('127.0.0.1', port, 1, True)
    return RcclComm(0, 1, device, store=store, tag='bench')


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus and rank == 0:
        print(f'warning: --gpus {args.gpus} but WORLD_SIZE={world}', file=sys.stderr)

    if not torch.cuda.is_available():
        print('bench.py needs a GPU', file=sys.stderr)
        sys.exit(2)
    # one GPU per rank; MLC_DIST_BACKEND=gloo (with --graph 0) rehearses the multi-rank path
    # with several ranks sharing the GPUs there are (local rank modulo the device count)
    backend = os.environ.get('MLC_DIST_BACKEND', 'nccl')
    dev_index = local_rank % torch.cuda.device_count() if backend != 'nccl' else local_rank
    torch.cuda.set_device(dev_index)
    device = torch.device('cuda', dev_index)
    if world > 1:
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=device)
        else:
            dist.init_process_group(backend)

    comm = _world1_rccl(device) if (args.comm == 'rccl1' and world == 1 and args.impl == 'native') else None
    is_bert = args.model.startswith('bert')
    is_unet = args.model.split('-')[0] in ('unet', 'linknet', 'fpn', 'pspnet', 'deeplab')
    # torch.nn-defined transformers (no hand engine): the generic native engine's fx lowering
    is_generic = args.model.startswith(('transformer-', 'vit-'))
    if args.batch is None:
        # ResNet-50: 512 images per GPU, sized for 288 GB of HBM3E (the reference's preset is 56
        # for 11-16 GB cards). Measured on one MI355X: 256 -> 12.4-12.7k img/s, 512 -> 13.3-13.4k,
        # 768 -> 13.5k; stock PyTorch-ROCm 6.0k / 6.4k at 256 / 512
        # (profiles/round4/resnet50_batch.txt). --batch 256 reproduces the earlier rounds' config.
        args.batch = 32 if (is_bert or is_unet or args.model.startswith('transformer-')) else \
            128 if args.model.startswith('vit-') else 512
    if is_generic:
        from mlcomp_amd.train.generic import build_generic_step
        step = build_generic_step(args.model, batch=args.batch, seq_len=args.seq_len, image_size=args.image_size,
                                  impl=args.impl, device=device, world_size=world,
                                  use_graph=(args.graph if args.graph >= 0 else None), comm=comm)
    elif is_unet:
        # U-Net (BASELINE config 3): --model unet[-<encoder>], 256x256 unless --image-size
        from mlcomp_amd.train.segment import build_seg_step
        if args.image_size == 224:
            args.image_size = 256
        # (--model linknet|fpn|pspnet[-<encoder>] / deeplab: that model on the same data / loss / optimizer)
        enc = args.model.split('-', 1)[1] if '-' in args.model else 'resnet34'
        step = build_seg_step(enc, batch=args.batch, impl=args.impl, image_size=args.image_size, device=device,
                              world_size=world, use_graph=(args.graph if args.graph >= 0 else None),
                              arch=args.model.split('-', 1)[0])
    elif is_bert:
        from mlcomp_amd.train.bert import build_bert_step
        step = build_bert_step(args.model, batch=args.batch, seq_len=args.seq_len, impl=args.impl,
                               device=device, world_size=world,
                               use_graph=(args.graph if args.graph >= 0 else None), comm=comm,
                               precision=args.precision)
    else:
        from mlcomp_amd.train.imagenet import build_train_step
        step = build_train_step(args.model, batch=args.batch, impl=args.impl,
                                image_size=args.image_size, device=device,
                                world_size=world,
                                use_graph=(args.graph if args.graph >= 0 else None), comm=comm,
                                precision=args.precision)

    if comm is not None and getattr(step, 'bucketer', None) is not None:
        step.bucketer.op = 'avg'     # world 1: scale 1.0, but RCCL launches its kernel per bucket
    feed = None
    if args.data == 'records':
        if is_bert or is_unet:
            print('--data records feeds the image classifiers only', file=sys.stderr)
            sys.exit(2)
        feed = _record_feed(args, rank, world, device, dist)
        inner = step

        def step():
            b = next(feed)
            inner.load_batch(b['features'], b['targets'])
            inner()
        step.last_loss = inner.last_loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms = elapsed * 1000.0 / args.steps
    images = args.batch * world * args.steps
    value = images / elapsed
    loss = step.last_loss()
    if rank == 0 and feed is not None:
        out = {
            'metric': 'images/sec (whole node) ResNet-50 DAG train task, record-file input pipeline',
            'value': round(value, 2), 'unit': 'images/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'bf16',
            'data': 'synthetic uint8 256x256x3 images in an mlrec file (RandomResizedCrop 224 + flip on the GPU), '
                    'random-init weights',
            'config': {'model': args.model, 'global_batch': args.batch * world, 'per_gpu_batch': args.batch,
                       'image_size': args.image_size, 'parallelism': f'dp{world}', 'impl': args.impl,
                       'loader_threads': args.loader_threads, 'final_loss': loss}}
        print(json.dumps(out), flush=True)
    elif rank == 0 and is_generic:
        text = args.model.startswith('transformer-')
        unit = 'sequences/s' if text else 'images/s'
        out = {
            'metric': f'{unit.split("/")[0]}/sec (whole node) {args.model} train task (torch.nn model, generic engine)',
            'value': round(value, 2), 'unit': unit, 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'bf16',
            'data': (f'synthetic (random token ids, seq_len {args.seq_len}, 2 labels, random-init weights)' if text else
                     f'synthetic ({args.image_size}x{args.image_size}x3 images, 1000 classes, random-init weights)'),
            'config': {'model': args.model, 'global_batch': args.batch * world, 'per_gpu_batch': args.batch,
                       'seq_len': args.seq_len if text else None, 'image_size': None if text else args.image_size,
                       'parallelism': f'dp{world}', 'impl': args.impl,
                       'optimizer': 'AdamW wd 0.01, fp32 master weights', 'final_loss': loss}}
        print(json.dumps(out), flush=True)
    elif rank == 0 and is_bert:
        out = {
            'metric': 'sequences/sec (whole node) BERT fine-tune DAG train task',
            'value': round(value, 2), 'unit': 'sequences/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': args.precision,
            'data': f'synthetic (random token ids, seq_len {args.seq_len}, 2 labels, random-init weights)',
            'config': {'model': args.model, 'global_batch': args.batch * world, 'per_gpu_batch': args.batch,
                       'seq_len': args.seq_len, 'parallelism': f'dp{world}', 'impl': args.impl,
                       'optimizer': 'AdamW lr 2e-5 wd 0.01, fp32 master weights', 'dropout': 0.1,
                       'final_loss': loss}}
        print(json.dumps(out), flush=True)
    elif rank == 0 and is_unet:
        out = {
            'metric': f"images/sec (whole node) {dict(linknet='LinkNet', fpn='FPN', pspnet='PSPNet', deeplab='DeepLab').get(args.model.split('-')[0], 'U-Net')} "
                      'segmentation DAG train task',
            'value': round(value, 2), 'unit': 'images/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'bf16',
            'data': f'synthetic ({args.image_size}x{args.image_size}x3 images, blob masks, 1 class, random-init weights)',
            'config': {'model': args.model, 'global_batch': args.batch * world, 'per_gpu_batch': args.batch,
                       'image_size': args.image_size, 'parallelism': f'dp{world}', 'impl': args.impl,
                       'optimizer': 'Adam lr 3e-4, fp32 master weights', 'loss': 'BCE + Dice',
                       'final_loss': loss}}
        print(json.dumps(out), flush=True)
    elif rank == 0:
        out = {
            'metric': 'images/sec (whole node) ResNet-50 DAG train task',
            'value': round(value, 2),
            'unit': 'images/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(ms, 3),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': (round(value / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
            'dtype': args.precision,
            'data': 'synthetic (ImageNet-shape 224x224x3, 1000 classes, random-init weights)',
            'config': {
                'model': args.model,
                'global_batch': args.batch * world,
                'per_gpu_batch': args.batch,
                'image_size': args.image_size,
                'seq_len': None,
                'parallelism': f'dp{world}',
                'impl': args.impl,
                'optimizer': 'SGD momentum 0.9, wd 5e-5, fp32 master weights',
                'final_loss': loss,
            },
        }
        if comm is not None:
            out['config']['comm'] = 'world-1 RCCL communicator (bucketed all-reduces issued)'
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, 'w') as f:
                f.write(line + '\n')
    if world > 1:
        dist.destroy_process_group()


def _record_feed(args, rank, world, device, dist):
    """An endless batch iterator over a record file through the native input pipeline
    (mlcomp_amd.train.records): C++ threads gather uint8 records into pinned slots, the
    augment kernel writes the stem's space-to-depth input."""
    import numpy as np
    from mlcomp_amd.train.records import RecordLoader, write_records
    path = args.records
    if path is None:
        path = os.path.join(os.environ.get('TMPDIR', '/tmp'), f'mlc_bench_{os.getpid() if world == 1 else "dp"}.mlrec')
        if rank == 0:
            n = max(2560, 4 * args.batch * world)
            rng = np.random.default_rng(0)
            chunks = (rng.integers(0, 256, (256, 256, 256, 3), dtype=np.uint8) for _ in range((n + 255) // 256))
            imgs = (im for c in chunks for im in c)
            write_records(path, imgs, (int(v) for v in rng.integers(0, 1000, n)), shape=(256, 256, 3))
        if world > 1:
            dist.barrier()
    loader = RecordLoader(path, args.batch, out_size=args.image_size, train=True, rank=rank, world_size=world,
                          threads=args.loader_threads, depth=4, layout='s2d', device=device)

    def gen():
        while True:
            yield from loader
    return gen()


if __name__ == '__main__':
    main()
