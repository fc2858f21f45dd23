"""Which gradients differ between two identical eager steps (run with MLC_DETERMINISTIC=1)."""
import torch
from mlcomp_amd.train.native_bert_step import NativeBertStep


def grads(seed_steps=1):
    torch.manual_seed(0)
    st = NativeBertStep('bert-small', batch=8, seq_len=64, device='cuda', use_graph=False, lr=1e-4)
    for _ in range(seed_steps):
        st()
    torch.cuda.synchronize()
    return {n: s.grad.detach().clone() for n, s in st.net.arena.by_name.items()}, st


ga, st = grads()
gb, _ = grads()
bad = [(n, float((ga[n] - gb[n]).abs().max())) for n in ga if not torch.equal(ga[n], gb[n])]
print('differing grads:', len(bad), 'of', len(ga))
for n, d in bad[:40]:
    print(f'  {d:.3e}  {n}')
