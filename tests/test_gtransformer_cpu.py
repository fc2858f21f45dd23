"""Transformer blocks on the generic native engine, CPU path (the kernels' fp32 references,
same bf16 rounding points): torch-defined ``nn.TransformerEncoder`` classifiers (post-norm
GELU with a key-padding mask, pre-norm ReLU sequence-first), ``nn.MultiheadAttention`` used
directly, and a ViT-style model (16x16 patch embedding, class token, position embedding,
LayerNorm + scaled_dot_product_attention blocks, Linear-GELU-Linear MLPs) lower to native
sites and match fp32 autograd in the forward and in every parameter gradient.

Reference: any model an experiment returns trains (`mlcomp/worker/executors/catalyst_/
catalyst_.py:365-372`), e.g. timm's ViT family through `mlcomp/contrib/model/timm.py:8-10`."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from mlcomp_amd.models.native_generic import GenericNet, lower_or_none
from mlcomp_amd.ops import gtransformer as GT


def _cos(a, b):
    a, b = a.flatten().float(), b.flatten().float()
    return (a @ b / (a.norm() * b.norm() + 1e-12)).item()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _pair(make, seed=0):
    torch.manual_seed(seed)
    m = make()
    ref = make()
    ref.load_state_dict(m.state_dict())
    return m, ref


def _slot_pairs(net, m):
    """(name, native grad, torch parameter of ``m``'s twin name) for every lowered set."""
    names = {id(p): n for n, p in m.named_parameters()}
    out = []
    for ps in net.param_sets():
        if isinstance(ps, GT.DenseSet):
            pairs = [(ps.src.weight, ps.w, (ps.O, ps.I)), (ps.src.bias, ps.b, None)]
        elif isinstance(ps, GT.LNParams):
            pairs = [(ps.src.weight, ps.g, None), (ps.src.bias, ps.b, None)]
        elif hasattr(ps, 'O'):          # LinearParams (padded to multiples of 8)
            pairs = [(ps.src.weight, ps.w, 'lin'), (ps.src.bias, ps.b, 'linb')]
        else:
            continue
        for t, slot, how in pairs:
            if t is None or slot is None:
                continue
            g = slot.grad
            if how == 'lin':
                g = g[:ps.O, :ps.I]
            elif how == 'linb':
                g = g[:ps.O]
            out.append((names[id(t)], g, t.shape))
    return out


def _check(make, x_fn, kinds_expected, seed=0, cos_min=0.98, extra=None):
    m, ref = _pair(make, seed)
    net = GenericNet(m, 'cpu')
    kinds = [type(s).__name__ for s in net.train_gm.modules()]
    for k, n in kinds_expected.items():
        assert kinds.count(k) == n, kinds
    args = x_fn()
    out = net(*args) if isinstance(args, tuple) else net(args)
    want = ref(*args) if isinstance(args, tuple) else ref(args)
    assert out.shape == want.shape
    assert _rel(out, want) < 3e-2, _rel(out, want)
    g = torch.randn_like(want)
    (out.float() * g).sum().backward()
    (want * g).sum().backward()
    refp = dict(ref.named_parameters())
    n = 0
    for name, got, shape in _slot_pairs(net, m):
        w = refp[name].grad.reshape(got.shape)
        assert _cos(got, w) > cos_min, (name, _cos(got, w))
        n += 1
    for name, p in m.named_parameters():          # parameters torch ops read (aliased into the arena)
        if p.grad is not None and any(name == nm for nm, _, _ in _slot_pairs(net, m)) is False:
            assert _cos(p.grad, refp[name].grad) > cos_min, name
    assert n > 0
    if extra:
        extra(net, m, ref)
    return net


class _EncClassifier(nn.Module):
    """Token embedding + post-norm GELU nn.TransformerEncoder (batch-first) + mean-pool head."""

    def __init__(self, norm_first=False, act='gelu', batch_first=True, final_norm=True):
        super().__init__()
        self.emb = nn.Embedding(50, 64)
        layer = nn.TransformerEncoderLayer(64, 4, 128, dropout=0.0, activation=act, batch_first=batch_first,
                                           norm_first=norm_first)
        self.enc = nn.TransformerEncoder(layer, 2, norm=nn.LayerNorm(64) if final_norm else None,
                                         enable_nested_tensor=False)
        self.head = nn.Linear(64, 5)
        self.batch_first = batch_first

    def forward(self, ids):
        pad = ids == 0                      # token id 0 pads
        x = self.emb(ids)
        if not self.batch_first:
            x = x.transpose(0, 1)
        h = self.enc(x, src_key_padding_mask=pad)
        if not self.batch_first:
            h = h.transpose(0, 1)
        return self.head(h.mean(1))


def _ids():
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(1, 50, (3, 24), generator=g)
    ids[1, 20:] = 0
    ids[2, 9:] = 0
    return ids


def test_transformer_encoder_post_norm_gelu_with_padding_mask():
    _check(_EncClassifier, _ids, {'EncoderSite': 1, 'LinearAct': 1})


def test_transformer_encoder_pre_norm_relu_sequence_first():
    _check(lambda: _EncClassifier(norm_first=True, act='relu', batch_first=False, final_norm=True), _ids,
           {'EncoderSite': 1})


class _MHANet(nn.Module):
    """nn.MultiheadAttention called directly (sequence-first, need_weights=False) inside a
    pre-norm residual block, LayerNorm fused with the residual add after it."""

    def __init__(self):
        super().__init__()
        self.inp = nn.Linear(16, 64)
        self.attn = nn.MultiheadAttention(64, 2)
        self.norm = nn.LayerNorm(64)
        self.head = nn.Linear(64, 3)

    def forward(self, x):                       # x [S, B, 16]
        h = self.inp(x)
        a = self.attn(h, h, h, need_weights=False)[0]
        h = self.norm(h + a)
        return self.head(h.mean(0))


def test_multihead_attention_module_and_fused_residual_layernorm():
    _check(_MHANet, lambda: torch.randn(20, 4, 16), {'MHASite': 1, 'LayerNormSite': 1})


class _Attention(nn.Module):
    """timm's ViT attention: packed qkv Linear, reshape / permute / unbind, SDPA."""

    def __init__(self, dim, heads):
        super().__init__()
        self.heads = heads
        self.qkv = nn.Linear(dim, dim * 3)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x):
        B, N, C = x.shape
        qkv = self.qkv(x).reshape(B, N, 3, self.heads, C // self.heads).permute(2, 0, 3, 1, 4)
        q, k, v = qkv.unbind(0)
        x = F.scaled_dot_product_attention(q, k, v)
        return self.proj(x.transpose(1, 2).reshape(B, N, C))


class _Block(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = _Attention(dim, heads)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.fc1 = nn.Linear(dim, 4 * dim)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(4 * dim, dim)

    def forward(self, x):
        x = x + self.attn(self.norm1(x))
        return x + self.fc2(self.act(self.fc1(self.norm2(x))))


class _ViT(nn.Module):
    """ViT-style: 16x16/16 patch conv, class token, learned positions, 2 pre-norm blocks."""

    def __init__(self, img=64, patch=16, dim=64, heads=2, depth=2, classes=7):
        super().__init__()
        self.patch = nn.Conv2d(3, dim, patch, patch)
        n = (img // patch) ** 2
        self.cls = nn.Parameter(torch.randn(1, 1, dim) * 0.02)
        self.pos = nn.Parameter(torch.randn(1, n + 1, dim) * 0.02)
        self.blocks = nn.Sequential(*[_Block(dim, heads) for _ in range(depth)])
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        self.head = nn.Linear(dim, classes)

    def forward(self, x):
        x = self.patch(x).flatten(2).transpose(1, 2)
        x = torch.cat([self.cls.expand(x.shape[0], -1, -1), x], dim=1) + self.pos
        x = self.norm(self.blocks(x))
        return self.head(x[:, 0])


def test_vit_style_model_lowers_and_matches_autograd():
    net = _check(_ViT, lambda: torch.randn(2, 3, 64, 64),
                 {'PatchEmbed': 1, 'SDPASite': 2, 'LayerNormSite': 5, 'MlpSite': 2})
    res = [s for s in net.train_gm.modules() if type(s).__name__ == 'LinearAct' and s.residual]
    assert len(res) == 2                      # attention projections with the residual add fused
    # the position embedding and class token stay torch ops on arena-aliased parameters
    assert any(n.op == 'call_function' and n.target is torch.cat for n in net.train_gm.graph.nodes)


class _GeluHead(nn.Module):
    """Linear -> GELU not followed by a Linear: the GELU epilogue site."""

    def __init__(self):
        super().__init__()
        self.fc = nn.Linear(24, 32)
        self.act = nn.GELU()

    def forward(self, x):
        return self.act(self.fc(x)).mean(1)


def test_linear_gelu_epilogue():
    _check(_GeluHead, lambda: torch.randn(6, 5, 24), {'LinearGelu': 1})


def test_transformer_models_choose_the_native_engine():
    assert lower_or_none(_EncClassifier()) is None
    assert lower_or_none(_ViT()) is None
    assert lower_or_none(_MHANet()) is None


class _CausalNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.layer = nn.TransformerEncoderLayer(32, 2, 64, dropout=0.0, batch_first=True)

    def forward(self, x):
        return self.layer(x, is_causal=True, src_mask=nn.Transformer.generate_square_subsequent_mask(x.shape[1]))


def test_unsupported_attention_forms_name_the_reason():
    assert 'mask' in lower_or_none(_CausalNet())
    big = nn.Sequential(nn.TransformerEncoder(nn.TransformerEncoderLayer(512, 2, 64, batch_first=True), 1,
                                              enable_nested_tensor=False))
    assert 'head dim 256' in lower_or_none(big)


def test_encoder_dropout_is_reproducible_and_changes_per_step():
    """Dropout masks come from the kernels' counter hash of (seed, salt, index): the same
    seed gives the same output, the per-step seed advance gives new masks."""
    torch.manual_seed(0)
    m = nn.Sequential(nn.TransformerEncoder(nn.TransformerEncoderLayer(32, 2, 64, dropout=0.3, batch_first=True), 1,
                                            enable_nested_tensor=False))
    net = GenericNet(m, 'cpu')
    x = torch.randn(2, 10, 32)
    net.ctx.seed.zero_()
    a = net(x).detach()
    net.ctx.seed.zero_()
    b = net(x).detach()
    c = net(x).detach()
    assert torch.equal(a, b) and not torch.equal(b, c)
    net.eval()
    e1, e2 = net(x), net(x)
    assert torch.equal(e1, e2)
