"""Transformer models written with stock ``torch.nn`` building blocks, as a user (or a
``timm`` / ``torchvision`` model, `mlcomp/contrib/model/timm.py:8-10`) would write them.

They have no hand-lowered engine: the runner trains them on the generic native engine
(:mod:`mlcomp_amd.models.native_generic`), whose fx lowering maps ``nn.TransformerEncoder``,
``nn.LayerNorm``, ``F.scaled_dot_product_attention``, Linear-GELU and the patch embedding onto
the framework's kernels (:mod:`mlcomp_amd.ops.gtransformer`).

* ``TransformerClassifier`` - token + position embeddings, ``nn.TransformerEncoder``
  (post-norm, exact GELU, batch-first), tanh pooler on the first token, classifier.
  ``transformer-base`` has BERT-base's shapes (12 x 768, 12 heads, 3072 FFN) for a
  like-for-like comparison with the hand BERT engine.
* ``VisionTransformer`` - ViT (Dosovitskiy et al. 2021): 16x16 patch embedding conv, class
  token, learned positions, pre-norm blocks whose attention is timm's packed-qkv
  ``F.scaled_dot_product_attention`` form, Linear-GELU-Linear MLPs.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import register


class TransformerClassifier(nn.Module):
    def __init__(self, vocab_size=30522, hidden=768, layers=12, heads=12, intermediate=3072, max_position=512,
                 num_classes=2, dropout=0.1, norm_first=False, activation='gelu', pad_id=None, eps=1e-12):
        super().__init__()
        self.pad_id = pad_id
        self.word = nn.Embedding(vocab_size, hidden)
        self.pos = nn.Embedding(max_position, hidden)
        self.ln = nn.LayerNorm(hidden, eps=eps)
        self.drop = nn.Dropout(dropout)
        layer = nn.TransformerEncoderLayer(hidden, heads, intermediate, dropout=dropout, activation=activation,
                                           layer_norm_eps=eps, batch_first=True, norm_first=norm_first)
        self.encoder = nn.TransformerEncoder(layer, layers, norm=nn.LayerNorm(hidden, eps=eps) if norm_first else None,
                                             enable_nested_tensor=False)
        self.pooler = nn.Linear(hidden, hidden)
        self.classifier = nn.Linear(hidden, num_classes)
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, 0.0, 0.02)
            if isinstance(m, nn.Linear) and m.bias is not None:
                nn.init.zeros_(m.bias)

    def forward(self, ids):
        S = ids.shape[1]
        pos = torch.arange(S, device=ids.device)
        x = self.drop(self.ln(self.word(ids) + self.pos(pos)))
        pad = (ids == self.pad_id) if self.pad_id is not None else None
        h = self.encoder(x, src_key_padding_mask=pad)
        pooled = torch.tanh(self.pooler(h[:, 0]))
        return self.classifier(self.drop(pooled))


class _Attention(nn.Module):
    def __init__(self, dim, heads, attn_drop=0.0, proj_drop=0.0):
        super().__init__()
        self.heads = heads
        self.qkv = nn.Linear(dim, dim * 3)
        self.attn_drop = attn_drop
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)

    def forward(self, x):
        B, N, C = x.shape
        qkv = self.qkv(x).reshape(B, N, 3, self.heads, C // self.heads).permute(2, 0, 3, 1, 4)
        q, k, v = qkv.unbind(0)
        x = F.scaled_dot_product_attention(q, k, v, dropout_p=self.attn_drop if self.training else 0.0)
        return self.proj_drop(self.proj(x.transpose(1, 2).reshape(B, N, C)))


class _Block(nn.Module):
    def __init__(self, dim, heads, mlp_ratio=4.0, drop=0.0):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = _Attention(dim, heads, proj_drop=drop)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        hidden = int(dim * mlp_ratio)
        self.fc1 = nn.Linear(dim, hidden)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden, dim)
        self.drop = nn.Dropout(drop)

    def forward(self, x):
        x = x + self.attn(self.norm1(x))
        return x + self.drop(self.fc2(self.act(self.fc1(self.norm2(x)))))


class VisionTransformer(nn.Module):
    def __init__(self, image_size=224, patch=16, dim=768, depth=12, heads=12, mlp_ratio=4.0, num_classes=1000,
                 drop=0.0, in_channels=3):
        super().__init__()
        self.patch_embed = nn.Conv2d(in_channels, dim, patch, patch)
        n = (image_size // patch) ** 2
        self.cls_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos_embed = nn.Parameter(torch.randn(1, n + 1, dim) * 0.02)
        self.blocks = nn.Sequential(*[_Block(dim, heads, mlp_ratio, drop) for _ in range(depth)])
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        self.head = nn.Linear(dim, num_classes)
        nn.init.normal_(self.cls_token, std=0.02)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.patch_embed(x).flatten(2).transpose(1, 2)
        x = torch.cat([self.cls_token.expand(x.shape[0], -1, -1), x], dim=1) + self.pos_embed
        x = self.norm(self.blocks(x))
        return self.head(x[:, 0])


TEXT_PRESETS = {'transformer-base': dict(),
                'transformer-small': dict(hidden=512, layers=4, heads=8, intermediate=2048),
                'transformer-tiny': dict(hidden=128, layers=2, heads=2, intermediate=512, vocab_size=1024,
                                         max_position=128)}
VIT_PRESETS = {'vit-b16': dict(dim=768, depth=12, heads=12), 'vit-s16': dict(dim=384, depth=12, heads=6),
               'vit-ti16': dict(dim=192, depth=12, heads=3)}


def _text(name, **kw):
    cfg = dict(TEXT_PRESETS[name])
    if 'num_labels' in kw:
        kw['num_classes'] = kw.pop('num_labels')
    cfg.update(kw)
    return TransformerClassifier(**cfg)


def _vit(name, **kw):
    cfg = dict(VIT_PRESETS[name])
    cfg.update(kw)
    return VisionTransformer(**cfg)


for _n in TEXT_PRESETS:
    register(_n)((lambda n: (lambda **kw: _text(n, **kw)))(_n))
for _n in VIT_PRESETS:
    register(_n)((lambda n: (lambda **kw: _vit(n, **kw)))(_n))

__all__ = ['TransformerClassifier', 'VisionTransformer', 'TEXT_PRESETS', 'VIT_PRESETS']
