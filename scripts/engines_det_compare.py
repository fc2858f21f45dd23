"""GPU step vs CPU step of every native engine in deterministic mode (per-slot gradient error).

Run with MLC_DETERMINISTIC=1 (ordered reductions, unsplit GEMMs on the GPU).  For each
engine one training step (lr 0) runs on the CPU path of the native ops and on the GPU
kernels from the same weights and batch; prints one JSON line per engine with the loss
error and the distribution of per-slot relative gradient errors ||g_gpu - g_cpu|| / ||g_cpu||.

    MLC_DETERMINISTIC=1 python scripts/engines_det_compare.py [--noise] [kind ...]

``--noise``: also run the CPU step with every fp32 master weight moved by about one fp32 ulp
(x (1 + eps n), eps = DET_NOISE_EPS, default 2^-24; this flips the bf16 rounding of ~0.003 %
of the weights) in DET_NOISE_DRAWS independent draws (default 2), and report the per-slot
errors that causes: the step's sensitivity to a change far below anything the GPU kernels
could introduce on purpose.  Batch-normalised networks at random init amplify such changes
enormously (docs/numerics.md: stock PyTorch bf16 autocast moves ResNeXt-50 slot gradients by
~100 % for the same perturbation), so this floor, not a fixed tolerance, is what a bf16 GPU
step can be held to.  ``noise_per_slot`` is the per-slot maximum over the draws.
"""
import json
import os
import sys

import torch

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [root, os.path.join(root, 'tests')]

B, R = int(os.environ.get('DET_BATCH', 8)), int(os.environ.get('DET_RES', 128))
NOISE_EPS = float(os.environ.get('DET_NOISE_EPS', 2.0 ** -24))
NOISE_DRAWS = int(os.environ.get('DET_NOISE_DRAWS', 2))


def make(kind, device):
    torch.manual_seed(0)
    if kind == 'resnet50':
        from mlcomp_amd.train.native_step import NativeClassifierStep
        return NativeClassifierStep('resnet50', batch=B, image_size=R, device=device, num_classes=10,
                                    use_graph=False, lr=0.0, momentum=0.0, weight_decay=0.0)
    from mlcomp_amd.train.native_seg_step import NativeSegmentationStep
    if kind == 'unet':
        return NativeSegmentationStep('resnet34', batch=B, image_size=R, device=device, use_graph=False, lr=0.0)
    if kind in ('linknet', 'fpn', 'pspnet', 'deeplab'):
        from mlcomp_amd.contrib.segmentation.deeplab import DeepLab
        from mlcomp_amd.contrib.segmentation.models import FPN, Linknet, PSPNet
        tm = (Linknet(encoder_name='resnet34') if kind == 'linknet' else
              FPN(encoder_name='resnet34', dropout=0.0) if kind == 'fpn' else
              PSPNet(encoder_name='resnet34', classes=1, dropout=0.0) if kind == 'pspnet' else
              DeepLab(backbone='resnet', num_classes=1))
        for m in tm.modules():           # dropout masks come from different RNGs on CPU / GPU
            if isinstance(m, (torch.nn.Dropout, torch.nn.Dropout2d)):
                m.p = 0.0
        return NativeSegmentationStep(torch_model=tm, batch=B, image_size=R, device=device, use_graph=False, lr=0.0)
    if kind == 'bert':
        from mlcomp_amd.train.native_bert_step import NativeBertStep
        return NativeBertStep('bert-base', batch=B, seq_len=64, device=device, use_graph=False, lr=0.0, dropout=0.0)
    # generic engine
    from test_generic_gpu import _models, _no_stochastic
    from mlcomp_amd.train.native_generic_step import NativeGenericStep
    mk, shape, ncls = _models()[kind]
    m = _no_stochastic(mk())
    g = torch.Generator().manual_seed(7)
    x = torch.randn(*shape, generator=g)
    if ncls is None:
        y = (torch.rand(shape[0], 1, shape[2], shape[3], generator=g) > 0.5).float()
        crit = torch.nn.BCEWithLogitsLoss()
    else:
        y = torch.randint(0, ncls, (shape[0],) + ((shape[2], shape[3]) if kind.startswith('psp') else ()), generator=g)
        crit = torch.nn.CrossEntropyLoss()
    return NativeGenericStep(m, x, y, device=device, use_graph=False, optimizer='SGD', lr=0.0, criterion=crit)


def copy_inputs(dst, src):
    for name in ('x', 'y', 't', 'ids', 'tt', 'key_bias'):
        a, b = getattr(dst, name, None), getattr(src, name, None)
        if isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor):
            a.copy_(b.to(a.device))


def grads(step):
    step()
    if step.device.type == 'cuda':
        torch.cuda.synchronize()
    out = {}
    for name, slot in step.net.arena.by_name.items():
        g = slot.grad.detach().float().cpu().flatten()
        if float(g.norm()) > 0:
            out[name] = g.clone()
    return step.last_loss(), out


def main():
    from mlcomp_amd.ops import _lib
    args = sys.argv[1:]
    noise = '--noise' in args
    args = [a for a in args if a != '--noise']
    kinds = args or ['resnet50', 'unet', 'linknet', 'fpn', 'pspnet', 'deeplab', 'bert',
                             'resnext50', 'efficientnet-b0', 'unet-resnext50']
    for kind in kinds:
        cpu, gpu = make(kind, 'cpu'), make(kind, 'cuda')
        copy_inputs(gpu, cpu)
        l_c, g_c = grads(cpu)
        l_g, g_g = grads(gpu)
        rel = {n: float((g_g[n] - g_c[n]).norm() / (g_c[n].norm() + 1e-20)) for n in g_c if n in g_g}
        v = sorted(rel.values())
        worst = sorted(rel.items(), key=lambda kv: -kv[1])[:4]
        out = {'kind': kind, 'deterministic': bool(_lib.DETERMINISTIC), 'batch': B, 'res': R,
               'slots': len(v), 'missing': sorted(set(g_c) ^ set(g_g))[:4], 'loss_rel_err': abs(l_g - l_c) / abs(l_c),
               'grad_rel_max': v[-1], 'grad_rel_p90': v[int(0.9 * (len(v) - 1))], 'grad_rel_median': v[len(v) // 2],
               'worst': [(n, round(e, 4)) for n, e in worst], 'per_slot': rel}
        if noise:
            env, draws, lrel = {}, [], 0.0
            for d in range(NOISE_DRAWS):
                per = make(kind, 'cpu')
                copy_inputs(per, cpu)
                gen = torch.Generator().manual_seed(1 + d)
                with torch.no_grad():
                    for a in per.net.arena.arenas():
                        a.master.mul_(1 + NOISE_EPS * torch.randn(a.master.shape, generator=gen))
                        a.refresh_mirror()
                l_p, g_p = grads(per)
                one = {n: float((g_p[n] - g_c[n]).norm() / (g_c[n].norm() + 1e-20)) for n in g_c if n in g_p}
                for n, e in one.items():
                    env[n] = max(env.get(n, 0.0), e)
                vd = sorted(one.values())
                draws.append(vd[len(vd) // 2])
                lrel = max(lrel, abs(l_p - l_c) / abs(l_c))
                del per
            out['noise_eps'], out['noise_draw_medians'] = NOISE_EPS, draws
            out['noise_per_slot'] = env
            vn = sorted(env.values())
            out['noise_median'], out['noise_max'] = vn[len(vn) // 2], vn[-1]
            out['noise_loss_rel'] = lrel
            out['ratio_median'] = out['grad_rel_median'] / max(out['noise_median'], 1e-20)
            out['ratio_slot_max'] = max(rel[n] / max(env.get(n, 0.0), 1e-20) for n in rel)
        print(json.dumps(out), flush=True)
        del cpu, gpu
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
