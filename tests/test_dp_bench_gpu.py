"""The multi-rank path of ``bench.py`` (the driver's N-GPU scaling run) rehearsed on one GPU:
torchrun starts two ranks that share the device over a gloo process group (RCCL needs one
GPU per rank), each runs the native data-parallel step eagerly (``--graph 0``: gloo
collectives cannot be captured) through the production gradient bucketer, and rank 0
prints the whole-job JSON line from the max-over-ranks time.  On an 8-GPU node the same
script runs with ``nccl`` (RCCL) and the captured step."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize('model,batch', [('resnet50', 32), ('bert-base', 8)])
def test_bench_two_ranks_share_one_gpu(model, batch):
    env = dict(os.environ, MLC_DIST_BACKEND='gloo', OMP_NUM_THREADS='4')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2',
           '--master-addr=127.0.0.1', f'--master-port={_port()}', 'bench.py', '--gpus', '2', '--steps', '3',
           '--warmup', '2', '--graph', '0', '--model', model, '--batch', str(batch)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 only
    out = json.loads(lines[0])
    assert out['n_gpus'] == 2 and out['steps'] == 3 and out['warmup'] == 2
    assert out['config']['parallelism'] == 'dp2' and out['config']['global_batch'] == 2 * batch
    assert out['value'] > 0 and out['ms_per_step'] > 0
    assert abs(out['value'] - 2 * batch * 1000.0 / out['ms_per_step']) / out['value'] < 1e-2
    loss = out['config']['final_loss']
    assert loss == loss and abs(loss) < 1e4                # finite
