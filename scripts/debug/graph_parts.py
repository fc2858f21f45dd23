"""Which part of an EfficientNet block misbehaves under HIP-graph replay: tiny models built
from one ingredient each, eager vs graph for 6 steps."""
import sys
import torch
import torch.nn as nn
sys.path[:0] = ['.']
from mlcomp_amd.train.native_generic_step import NativeGenericStep  # noqa: E402


class SE(nn.Module):
    def __init__(self, c, sq):
        super().__init__()
        self.se = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(c, sq, 1), nn.SiLU(), nn.Conv2d(sq, c, 1),
                                nn.Sigmoid())

    def forward(self, x):
        return x * self.se(x)


class Res(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.p = nn.Sequential(nn.Conv2d(c, c, 1, bias=False), nn.BatchNorm2d(c))

    def forward(self, x):
        return self.p(x) + x


def net(kind):
    body = {'dw': [nn.Conv2d(32, 32, 3, 1, 1, groups=32, bias=False), nn.BatchNorm2d(32), nn.SiLU()],
            'dw5s2': [nn.Conv2d(32, 32, 5, 2, 2, groups=32, bias=False), nn.BatchNorm2d(32), nn.SiLU()],
            'se': [SE(32, 8)], 'se6': [SE(32, 6)], 'res': [Res(32)],
            'silu': [nn.Conv2d(32, 32, 1, bias=False), nn.BatchNorm2d(32), nn.SiLU()]}[kind]
    return nn.Sequential(nn.Conv2d(3, 32, 3, 2, 1, bias=False), nn.BatchNorm2d(32), nn.SiLU(), *body, *body,
                         nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(32, 10))


for kind in sys.argv[1:]:
    torch.manual_seed(0)
    ms = [net(kind), net(kind)]
    ms[1].load_state_dict(ms[0].state_dict())
    x, y = torch.randn(8, 3, 32, 32), torch.randint(0, 10, (8,))
    st = [NativeGenericStep(m, x, y, device='cuda', use_graph=g, optimizer='SGD', lr=0.05, momentum=0.9)
          for m, g in zip(ms, (False, True))]
    le, lg = [], []
    for i in range(8):
        st[0]()
        st[1]()
        le.append(round(st[0].last_loss(), 4))
        lg.append(round(st[1].last_loss(), 4))
    print(kind, 'eager', le, '\n', kind, 'graph', lg, flush=True)
