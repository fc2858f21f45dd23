"""Per-site GPU vs CPU comparison of a lowered model (forward outputs, input gradients)."""
import sys
import torch
import torch.nn as nn
sys.path[:0] = ['.', 'tests']
from test_generic_gpu import _models, _no_stochastic, rel  # noqa: E402
from mlcomp_amd.models.native_generic import GenericNet  # noqa: E402

name = sys.argv[1]
make, shape, ncls = _models()[name]
torch.manual_seed(0)
mg = _no_stochastic(make())
mc = _no_stochastic(make())
mc.load_state_dict(mg.state_dict())
x = torch.randn(*shape)
if ncls is None:
    y = (torch.rand(shape[0], 1, shape[2], shape[3]) > 0.5).float()
    crit = nn.BCEWithLogitsLoss()
else:
    y = torch.randint(0, ncls, (shape[0],) + ((shape[2], shape[3]) if name.startswith('psp') else ()))
    crit = nn.CrossEntropyLoss()
mf = _no_stochastic(make())
mf.load_state_dict(mg.state_dict())
mf.train()
crit(mf(x).float(), y).backward()
fgrad = {n: p.grad.detach().float().clone() for n, p in mf.named_parameters() if p.grad is not None}
rec = {}
nets = {}
for dev, m in (('cpu', mc), ('cuda', mg)):
    net = GenericNet(m, dev)
    outs, grads = {}, {}
    for n, mod in net.train_gm.named_modules():
        if hasattr(mod, 'fwd'):
            def hook(mod, inp, out, n=n):
                outs[n] = out.detach().float().cpu()
                if out.requires_grad:
                    out.register_hook(lambda g, n=n: grads.__setitem__(n, g.detach().float().cpu()))
            mod.register_forward_hook(hook)
    out = net(x.to(dev))
    loss = crit(out.float(), y.to(dev))
    loss.backward()
    rec[dev] = (outs, grads, loss.item())
    nets[dev] = net
print('loss', rec['cpu'][2], rec['cuda'][2])
for n in rec['cpu'][0]:
    o = rel(rec['cuda'][0][n], rec['cpu'][0][n])
    g = rel(rec['cuda'][1][n], rec['cpu'][1][n]) if n in rec['cpu'][1] and n in rec['cuda'][1] else -1
    print(f'{n:24s} out {o:.4f}  dout {g:.4f}  shape {tuple(rec["cpu"][0][n].shape)}')


def cos(a, b):
    a, b = a.flatten().float().cpu(), b.flatten().float().cpu()
    return float(a @ b / (a.norm() * b.norm() + 1e-20))


print('per-parameter gradient direction vs fp32 autograd: cos(cpu-native), cos(gpu-native), cos(gpu, cpu)')
for pc, pg in zip(nets['cpu'].param_sets(), nets['cuda'].param_sets()):
    w = pc.name + '.weight'
    if w not in fgrad:
        continue
    m = pc.src
    pc.export_to_torch = None
    gc = pc.w.grad if hasattr(pc, 'w') else pc.gamma.grad
    gg = pg.w.grad if hasattr(pg, 'w') else pg.gamma.grad
    f = fgrad[w]
    if hasattr(pc, 'kind'):
        if pc.kind == 'dense':
            f = torch.nn.functional.pad(f.permute(0, 2, 3, 1), (0, pc.Cip - pc.Ci, 0, 0, 0, 0, 0, pc.Cop - pc.Co))
        elif pc.kind == 'dw':
            f = torch.nn.functional.pad(f[:, 0].permute(1, 2, 0), (0, pc.Cop - pc.Co))
        else:
            f = f.permute(0, 2, 3, 1)
    elif hasattr(pc, 'O'):
        f = torch.nn.functional.pad(f, (0, pc.Ip - pc.I, 0, pc.Op - pc.O))
    else:
        f = torch.nn.functional.pad(f, (0, pc.Cp - pc.C))
    print(f'{pc.name:40s} {cos(gc, f):.4f} {cos(gg, f):.4f} {cos(gg, gc):.4f}')
if len(sys.argv) > 2:
    from mlcomp_amd.train.native_generic_step import NativeGenericStep
    torch.manual_seed(0)
    ms = [_no_stochastic(make()) for _ in range(2)]
    ms[1].load_state_dict(ms[0].state_dict())
    yy = torch.randint(0, ncls, (shape[0],))
    steps = [NativeGenericStep(m, x, yy, device='cuda', use_graph=g, optimizer='SGD', lr=float(sys.argv[2]),
                               momentum=0.9) for m, g in zip(ms, (False, True))]
    for i in range(30):
        for s in steps:
            s()
        print(i, steps[0].last_loss(), steps[1].last_loss())
# the stock mixed-precision path as the noise floor: torch autocast bf16 on the GPU
ma = _no_stochastic(make())
ma.load_state_dict(mg.state_dict())
ma = ma.cuda().to(memory_format=torch.channels_last).train()
with torch.autocast('cuda', dtype=torch.bfloat16):
    oa = ma(x.cuda().contiguous(memory_format=torch.channels_last))
crit(oa.float(), y.cuda()).backward()
cs = []
for n, p in ma.named_parameters():
    if p.grad is not None and n in fgrad:
        cs.append(cos(p.grad, fgrad[n]))
print(f'torch autocast bf16 vs fp32: mean cos {sum(cs) / len(cs):.4f} min {min(cs):.4f} over {len(cs)}')
