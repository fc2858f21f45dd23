"""Native BERT engine on CPU (kernel entry points fall back to their fp32 references):
gradients match the plain PyTorch BERT, dropout hash masks are reproducible."""
import math

import pytest
import torch

from mlcomp_amd.models import build_model
from mlcomp_amd.models.native_bert import NativeBert
from mlcomp_amd.ops import transformer as Tx


def _cos(a, b):
    a, b = a.flatten().float(), b.flatten().float()
    return (a @ b / (a.norm() * b.norm() + 1e-12)).item()


# S=64: whole-tile fused-attention path (head dim 64); (128, 256): head dim 128, flash path
@pytest.mark.parametrize('S,hidden', [(16, 128), (64, 128), (128, 256)])
def test_native_bert_matches_torch_autograd(S, hidden):
    torch.manual_seed(0)
    kw = dict(num_classes=3, hidden_dropout=0.0, attention_dropout=0.0, hidden=hidden)
    tm = build_model('bert-tiny', **kw)
    ref = build_model('bert-tiny', **kw)
    ref.load_state_dict(tm.state_dict())
    B = 4
    net = NativeBert(tm, 'cpu', B, S)
    ids = torch.randint(0, 1024, (B, S))
    tt = torch.zeros(B, S, dtype=torch.long)
    tt[:, S // 2:] = 1
    y = torch.randint(0, 3, (B,))
    am = torch.ones(B, S, dtype=torch.long)
    am[0, S - 4:] = 0                      # one padded sequence
    kb = ref.key_bias(am)
    net.ctx.ws.zero()
    net.arena.zero_grad()
    loss = net.loss(ids, tt, kb, y)
    loss.backward()
    lr = torch.nn.functional.cross_entropy(ref(ids, tt, am), y)
    lr.backward()
    assert abs(loss.item() - lr.item()) < 2e-3
    a = net.arena.by_name
    pairs = [('layers.0.qkv.weight', ref.layers[0].qkv.weight), ('layers.1.ffn1.weight', ref.layers[1].ffn1.weight),
             ('layers.1.ffn2.bias', ref.layers[1].ffn2.bias), ('layers.0.ln1.weight', ref.layers[0].ln1.weight),
             ('word', ref.word.weight), ('pos', ref.pos.weight), ('tok_type', ref.tok_type.weight),
             ('pooler.weight', ref.pooler.weight), ('ln.bias', ref.ln.bias)]
    for name, p in pairs:
        assert _cos(a[name].grad, p.grad) > 0.999, name
    assert _cos(a['classifier.weight'].grad[:3], ref.classifier.weight.grad) > 0.999
    net.export_to_torch()


def test_dropout_hash_masks():
    m1 = Tx.keep_mask((64, 128), 0.1, seed=5, salt=3)
    m2 = Tx.keep_mask((64, 128), 0.1, seed=5, salt=3)
    m3 = Tx.keep_mask((64, 128), 0.1, seed=6, salt=3)
    assert torch.equal(m1, m2) and not torch.equal(m1, m3)
    frac = m1.float().mean().item()
    assert 0.88 < frac < 0.92
    x = torch.randn(64, 128).to(torch.bfloat16)
    y = Tx.dropout(x, 0.1, torch.tensor([5]), 3)
    assert torch.equal(y == 0, ~m1 | (x == 0))


def test_native_bert_dropout_trains():
    torch.manual_seed(1)
    tm = build_model('bert-tiny', num_classes=2)
    net = NativeBert(tm, 'cpu', 8, 16)
    ids = torch.randint(0, 1024, (8, 16))
    tt = torch.zeros(8, 16, dtype=torch.long)
    y = torch.randint(0, 2, (8,))
    from mlcomp_amd.train.optim import FusedAdam
    opt = FusedAdam(net.arena, lr=1e-3, weight_decay=0.01, decoupled=True)
    losses = []
    for step in range(15):
        net.ctx.ws.zero()
        net.arena.zero_grad()
        net.seed.add_(1)
        opt.prepare()
        l = net.loss(ids, tt, None, y)
        l.backward()
        opt.step()
        losses.append(l.item())
    assert losses[-1] < losses[0]


@pytest.mark.parametrize('p', [0.0, 0.1])
def test_fused_attention_reference_matches_unfused_path(p):
    """attn_fwd / attn_bwd (the fused kernels' reference) == bmm + softmax kernels path."""
    torch.manual_seed(3)
    B, S, H = 2, 64, 3
    qkv = (torch.randn(B * S, 3 * H * 64) * 0.5).to(torch.bfloat16)
    dctx = torch.randn(B * S, H * 64).to(torch.bfloat16)
    kb = torch.zeros(B, S)
    kb[1, 50:] = float('-inf')
    seed, salt, scale = torch.tensor([9]), 5, 1.0 / math.sqrt(64)
    ctx, lse = Tx.attn_fwd(qkv, kb, B, S, H, scale, p, seed, salt)
    dqkv = Tx.attn_bwd(qkv, kb, dctx, lse, B, S, H, scale, p, seed, salt)
    # unfused reference: autograd through the softmax-kernel references
    x = qkv.float().requires_grad_(True)
    q, k, v = x.view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4).reshape(3, B * H, S, 64).unbind(0)
    sc = torch.bmm(q, k.transpose(1, 2)).reshape(-1, S) * scale + kb.repeat_interleave(H * S, 0)
    P = torch.softmax(sc, 1)
    if p > 0:
        P = torch.where(Tx.keep_mask(P.shape, p, 9, salt), P / (1 - p), torch.zeros_like(P))
    o = torch.bmm(P.view(B * H, S, S), v).view(B, H, S, 64).transpose(1, 2).reshape(B * S, H * 64)
    o.backward(dctx.float())
    assert (ctx.float() - o).abs().max().item() < 2e-2
    assert _cos(dqkv, x.grad) > 0.999


def test_native_bert_predict_matches_torch_eval():
    """Native validation forward: no dropout, any batch size, no loss accumulators."""
    torch.manual_seed(0)
    tm = build_model('bert-tiny', num_classes=3, hidden_dropout=0.1, attention_dropout=0.1)
    ref = build_model('bert-tiny', num_classes=3, hidden_dropout=0.1, attention_dropout=0.1)
    ref.load_state_dict(tm.state_dict())
    ref.eval()
    net = NativeBert(tm, 'cpu', 4, 16)
    net.ctx.ws.zero()
    ids = torch.randint(0, 1024, (5, 16))
    tt = torch.zeros(5, 16, dtype=torch.long)
    am = torch.ones(5, 16, dtype=torch.long)
    am[1, 12:] = 0
    logits = net.predict(ids, tt, ref.key_bias(am))
    with torch.no_grad():
        want = ref(ids, tt, am).float()
    assert logits.shape == (5, 3)
    assert _cos(logits, want) > 0.999 and (logits - want).abs().max() < 0.05
    assert net.loss_sum().item() == 0 and net.ctx.training and net.B == 4


def test_deterministic_embedding_segment_sums_match_index_add():
    """Deterministic mode's embedding backward: a stable sort + per-id sequential sums
    (no atomics, no one-hot GEMM) equal index_add_ for repeated ids."""
    import torch
    from mlcomp_amd.models.native_bert import _segment_sums
    g = torch.Generator().manual_seed(0)
    ix = torch.randint(0, 97, (2048,), generator=g)
    rows = torch.randn(2048, 24, generator=g)
    got = _segment_sums(ix, rows, 100)                # ids 97..99 never occur: zero rows
    want = torch.zeros(100, 24).index_add_(0, ix, rows)
    assert torch.allclose(got, want, atol=1e-5)


def test_head_dim_above_flash_limit_is_native_unsupported():
    """A head dim the fused attention does not take (> 128) raises NativeUnsupported at
    build time, and the runner's engine choice sends the model to the torch engine instead
    of asserting inside the first forward."""
    from mlcomp_amd.train.native_spec import NativeUnsupported
    from mlcomp_amd.train.runner import _generic_reason, _native_kind
    tm = build_model('bert-tiny', num_classes=2, hidden=512, heads=2, intermediate=512)
    assert tm.config.head_dim == 256
    with pytest.raises(NativeUnsupported, match='head_dim 256'):
        NativeBert(tm, 'cpu', 2, 16)
    assert _native_kind(tm, torch.device('cuda')) is None
    assert 'head_dim 256' in _generic_reason(tm)
    ok = build_model('bert-tiny', num_classes=2)
    assert _native_kind(ok, torch.device('cuda')) == 'bert'
