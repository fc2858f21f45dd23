"""Where does the native PSPNet step's GPU forward leave its CPU twin?  (The deterministic
anchor, scripts/engines_det_compare.py, puts PSPNet at ~5x the fp32-ulp noise floor while
every other engine sits at 0.8-1.7x.)  Runs models/native_psp.py's forward stage by stage
on the CPU path and on the GPU kernels from the same weights and batch and prints the
relative error of every intermediate, next to the same error for a CPU twin whose weights
moved by one fp32 ulp.

    MLC_DETERMINISTIC=1 python scripts/psp_bisect.py"""
import json
import os
import sys

import torch

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [root, os.path.join(root, 'tests'), os.path.join(root, 'scripts')]

from engines_det_compare import copy_inputs, make  # noqa: E402
from mlcomp_amd.models.native_fpn import _BilinearFn  # noqa: E402
from mlcomp_amd.ops import functional as Fn  # noqa: E402
from mlcomp_amd.ops.layers import ConvBN  # noqa: E402


def trace(step):
    net = step.net
    net.ctx.ws.zero()
    out = {}
    with torch.no_grad():
        x0 = net.stem(step.x)
        out['stem'] = x0
        y = net.pool(x0, net.ctx.anchor)
        want = 3 - net.level
        feats = []
        for i, blk in enumerate(net.blocks):
            y = blk(y)
            out[f'block{i}'] = y
            if i in net.ends:
                feats.append(y)
                if len(feats) > want:
                    break
        f = feats[want]
        h, w = f.shape[1], f.shape[2]
        ys = []
        for k, (size, unit) in enumerate(net.stages):
            p = Fn.AdaptiveAvgFn.apply(f.contiguous(), size, size)
            out[f'psp{k}.pool'] = p
            q = unit(p) if isinstance(unit, ConvBN) else torch.relu(unit(p))
            out[f'psp{k}.conv'] = q
            u = _BilinearFn.apply(q.contiguous(), (h, w))
            out[f'psp{k}.up'] = u
            ys.append(u)
        z = net.fuse(torch.cat(ys + [f], dim=-1))
        out['fuse'] = z
        lg = net.head.logits(z)
        out['logits'] = lg
    if step.device.type == 'cuda':
        torch.cuda.synchronize()
    return {k: v.detach().float().cpu() for k, v in out.items()}


def main():
    cpu, gpu = make('pspnet', 'cpu'), make('pspnet', 'cuda')
    copy_inputs(gpu, cpu)
    per = make('pspnet', 'cpu')
    copy_inputs(per, cpu)
    gen = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for a in per.net.arena.arenas():
            a.master.mul_(1 + 2.0 ** -24 * torch.randn(a.master.shape, generator=gen))
            a.refresh_mirror()
    tc, tg, tp = trace(cpu), trace(gpu), trace(per)
    for k in tc:
        e = float((tg[k] - tc[k]).norm() / (tc[k].norm() + 1e-20))
        n = float((tp[k] - tc[k]).norm() / (tc[k].norm() + 1e-20))
        print(json.dumps({'stage': k, 'shape': list(tc[k].shape), 'gpu_vs_cpu': e, 'fp32ulp_noise': n,
                          'ratio': e / max(n, 1e-20)}), flush=True)


if __name__ == '__main__':
    main()
