import os, sys, torch
sys.path.insert(0, os.getcwd())
from mlcomp_amd.models import build_model
from mlcomp_amd.train.native_step import NativeClassifierStep
for trial in range(3):
    torch.manual_seed(3)
    tm1 = build_model('resnet18', num_classes=10); tm2 = build_model('resnet18', num_classes=10)
    tm2.load_state_dict(tm1.state_dict())
    a = NativeClassifierStep(torch_model=tm1, batch=16, image_size=64, device='cuda', num_classes=10, use_graph=False)
    b = NativeClassifierStep(torch_model=tm2, batch=16, image_size=64, device='cuda', num_classes=10, use_graph=(trial != 2), warmup_eager=2)
    for _ in range(5):
        a(); b()
    torch.cuda.synchronize()
    pa, pb = a.net.arena.decay.master, b.net.arena.decay.master
    print(os.environ.get('MLC_DGRAD_WT'), 'graph' if trial != 2 else 'eager-eager', a.last_loss(), b.last_loss(), ((pa-pb).norm()/pa.norm()).item(), flush=True)
