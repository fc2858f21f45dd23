"""Eager vs graph-replayed BERT-small native steps (SGD): last loss and relative weight
difference after a few steps - the check of test_native_bert_step_trains_and_graph_matches,
printed instead of asserted (run under different MLC_* settings)."""
import sys

import torch

sys.path.insert(0, '.')
from mlcomp_amd.models import build_model  # noqa: E402
from mlcomp_amd.train.native_bert_step import NativeBertStep  # noqa: E402


def main():
    torch.manual_seed(0)
    tm1 = build_model('bert-small', num_labels=2)
    tm2 = build_model('bert-small', num_labels=2)
    tm3 = build_model('bert-small', num_labels=2)
    tm2.load_state_dict(tm1.state_dict())
    tm3.load_state_dict(tm1.state_dict())
    kw = dict(batch=8, seq_len=64, device='cuda', lr=2e-3, optimizer='SGD', momentum=0.9)
    a = NativeBertStep(torch_model=tm1, use_graph=False, **kw)
    c = NativeBertStep(torch_model=tm3, use_graph=False, **kw)
    b = NativeBertStep(torch_model=tm2, use_graph=True, warmup_eager=2, **kw)
    for i in range(4):
        a()
        b()
        c()
        torch.cuda.synchronize()
        pa, pb, pc = (s.net.arena.decay.master for s in (a, b, c))
        print(f'step {i}: loss eager {a.last_loss():.6f} eager2 {c.last_loss():.6f} graph {b.last_loss():.6f} '
              f'| w eager-graph {((pa - pb).norm() / pa.norm()).item():.2e} '
              f'eager-eager {((pa - pc).norm() / pa.norm()).item():.2e}', flush=True)


if __name__ == '__main__':
    main()
