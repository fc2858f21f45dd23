"""When does a graph-replayed generic step first produce non-finite values, and where."""
import sys
import torch
sys.path[:0] = ['.', 'tests']
from test_generic_gpu import _models, _no_stochastic  # noqa: E402
from mlcomp_amd.train.native_generic_step import NativeGenericStep  # noqa: E402

name, lr, graph = sys.argv[1], float(sys.argv[2]), sys.argv[3] == '1'
make, shape, ncls = _models()[name]
torch.manual_seed(0)
m = _no_stochastic(make())
x, y = torch.randn(*shape), torch.randint(0, ncls, (shape[0],))
st = NativeGenericStep(m, x, y, device='cuda', use_graph=graph, optimizer='SGD', lr=lr, momentum=0.9)
for i in range(int(sys.argv[4]) if len(sys.argv) > 4 else 14):
    st()
    torch.cuda.synchronize()
    bad_g = [n for n, s in st.net.arena.by_name.items() if not torch.isfinite(s.grad).all()]
    bad_w = [n for n, s in st.net.arena.by_name.items() if not torch.isfinite(s.master).all()]
    gmax = max(s.grad.abs().max().item() for s in st.net.arena.by_name.values())
    print(f'step {i} loss {st.last_loss():.6f} out|max| {st.out.float().abs().max().item():.4g} grad|max| {gmax:.4g}'
          f' nonfinite grads {len(bad_g)} {bad_g[-3:]} weights {len(bad_w)} {bad_w[-3:]}', flush=True)
    if bad_g or bad_w:
        break
