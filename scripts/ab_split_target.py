"""A/B the dense split-K target (mlc_gemm_get_set key 2) on the BERT and ResNet-50 steps."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mlcomp_amd.ops import _lib


def timed(step, warm=5, n=20):
    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    lib = _lib.load()
    model = sys.argv[1] if len(sys.argv) > 1 else 'bert-base'
    for tgt in [int(v) for v in sys.argv[2:]] or [128, 256, 512, 1024]:
        old = lib.mlc_gemm_get_set(2, tgt)
        if model.startswith('bert'):
            from mlcomp_amd.train.bert import build_bert_step
            step = build_bert_step(model, batch=32, seq_len=128, impl='native', device=torch.device('cuda', 0),
                                   world_size=1, use_graph=None)
        else:
            from mlcomp_amd.train.imagenet import build_train_step
            step = build_train_step(model, batch=256, impl='native', image_size=224, device=torch.device('cuda', 0),
                                    world_size=1, use_graph=None)
        ms = timed(step)
        print(f'{model} split_target_mat={tgt}: {ms:.3f} ms/step', flush=True)
        lib.mlc_gemm_get_set(2, old)
        del step
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
