"""Plain GEMMs of the training steps on the native engine vs hipBLASLt (torch.mm): the
weight-gradient GEMMs (fp32 output, out_dtype) of BERT-base and of ResNet-50's 1x1
convs, and BERT's dense forward / dgrad (bf16 out).  Interleaved rounds, one process."""
import json
import sys

import torch

sys.path.insert(0, '.')
from mlcomp_amd.ops import functional as Fn  # noqa: E402
from mlcomp_amd.ops import transformer as Tx  # noqa: E402


def timeit(fns, rounds=5, iters=20):
    times = {k: [] for k in fns}
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, f in fns.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                f()
            e.record()
            torch.cuda.synchronize()
            times[k].append(s.elapsed_time(e) / iters)
    return {k: sorted(v)[len(v) // 2] for k, v in times.items()}


def r(*s):
    return torch.rand(*s, device='cuda').sub(0.5).to(torch.bfloat16)


def main():
    dev = 'cuda'
    # weight gradients dW[O][I] = dY^T X over T rows
    for (T, O, I, tag) in [(4096, 2304, 768, 'bert qkv'), (4096, 768, 768, 'bert out'), (4096, 3072, 768, 'bert ffn1'),
                           (4096, 768, 3072, 'bert ffn2'), (802816, 64, 256, 'r50 l1 conv1'),
                           (802816, 256, 64, 'r50 l1 conv3'), (200704, 128, 512, 'r50 l2 conv1'),
                           (50176, 1024, 256, 'r50 l3 conv3'), (12544, 512, 2048, 'r50 l4 conv1')]:
        dy, x = r(T, O), r(T, I)
        dw = torch.zeros(O, I, device=dev)
        db = torch.zeros(O, device=dev)
        fns = {'native': lambda: Fn.linear_wgrad_bias(dy, x, dw, db) if tag.startswith('bert')
               else Fn.linear_wgrad(dy, x, out=dw, accumulate=True),
               'hipblaslt': lambda: torch.mm(dy.t(), x, out_dtype=torch.float32)}
        t = timeit(fns)
        fl = 2.0 * T * O * I
        print(json.dumps({'wgrad': tag, 'shape': [T, O, I], **{k: {'ms': round(v, 4), 'TF': round(fl / v / 1e9, 1)}
                                                              for k, v in t.items()}}), flush=True)
    for (M, N, K, tag) in [(4096, 2304, 768, 'qkv fwd'), (4096, 3072, 768, 'ffn1 fwd'), (4096, 768, 3072, 'ffn2 fwd'),
                           (4096, 768, 768, 'out fwd')]:
        x, w = r(M, K), r(N, K)
        b = torch.zeros(N, device=dev)
        fns = {'native': lambda: Tx.dense_fwd(x, w, b), 'hipblaslt': lambda: torch.mm(x, w.t())}
        t = timeit(fns)
        fl = 2.0 * M * N * K
        print(json.dumps({'fwd': tag, 'shape': [M, N, K], **{k: {'ms': round(v, 4), 'TF': round(fl / v / 1e9, 1)}
                                                            for k, v in t.items()}}), flush=True)
        dy = r(M, N)
        fns = {'native': lambda: Tx.dense_dgrad(dy, w), 'hipblaslt': lambda: torch.mm(dy, w)}
        t = timeit(fns)
        print(json.dumps({'dgrad': tag, 'shape': [M, K, N], **{k: {'ms': round(v, 4), 'TF': round(fl / v / 1e9, 1)}
                                                              for k, v in t.items()}}), flush=True)


if __name__ == '__main__':
    main()
