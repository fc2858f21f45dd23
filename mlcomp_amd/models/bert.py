"""BERT (Devlin et al. 2019) encoder + sequence-classification head, as a plain PyTorch
module (the ``torch`` engine, CPU runs, checkpoints).  The GPU training path is
:class:`mlcomp_amd.models.native_bert.NativeBert`, which takes this module's weights.

BASELINE.json names "BERT-base fine-tune DAG" as one of the configs; the reference has no
transformer code of its own (it would come through user code / Catalyst), so the
architecture follows the published model: post-LN encoder layers, exact-erf GELU,
learned absolute positions, token-type embeddings, tanh pooler on [CLS].
"""
from __future__ import annotations

import math
from dataclasses import dataclass, asdict

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import register


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    hidden_dropout: float = 0.1
    attention_dropout: float = 0.1
    eps: float = 1e-12
    num_labels: int = 2
    init_range: float = 0.02

    @property
    def head_dim(self):
        return self.hidden // self.heads


PRESETS = {'bert-base': dict(), 'bert-large': dict(hidden=1024, layers=24, heads=16, intermediate=4096),
           'bert-small': dict(hidden=512, layers=4, heads=8, intermediate=2048),
           'bert-tiny': dict(hidden=128, layers=2, heads=2, intermediate=512, vocab_size=1024, max_position=128)}


class BertLayer(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.c = c
        self.qkv = nn.Linear(c.hidden, 3 * c.hidden)
        self.out = nn.Linear(c.hidden, c.hidden)
        self.ln1 = nn.LayerNorm(c.hidden, eps=c.eps)
        self.ffn1 = nn.Linear(c.hidden, c.intermediate)
        self.ffn2 = nn.Linear(c.intermediate, c.hidden)
        self.ln2 = nn.LayerNorm(c.hidden, eps=c.eps)

    def forward(self, x, key_bias):
        B, S, H = x.shape
        nh, dh = self.c.heads, self.c.head_dim
        q, k, v = self.qkv(x).view(B, S, 3, nh, dh).permute(2, 0, 3, 1, 4)
        mask = key_bias[:, None, None, :].to(q.dtype) if key_bias is not None else None
        a = F.scaled_dot_product_attention(q, k, v, attn_mask=mask,
                                           dropout_p=self.c.attention_dropout if self.training else 0.0)
        a = a.transpose(1, 2).reshape(B, S, H)
        x = self.ln1(x + F.dropout(self.out(a), self.c.hidden_dropout, self.training))
        f = self.ffn2(F.gelu(self.ffn1(x)))
        return self.ln2(x + F.dropout(f, self.c.hidden_dropout, self.training))


class BertForSequenceClassification(nn.Module):
    def __init__(self, config: BertConfig = None, **kw):
        super().__init__()
        c = config or BertConfig(**kw)
        self.config = c
        self.word = nn.Embedding(c.vocab_size, c.hidden)
        self.pos = nn.Embedding(c.max_position, c.hidden)
        self.tok_type = nn.Embedding(c.type_vocab, c.hidden)
        self.ln = nn.LayerNorm(c.hidden, eps=c.eps)
        self.layers = nn.ModuleList(BertLayer(c) for _ in range(c.layers))
        self.pooler = nn.Linear(c.hidden, c.hidden)
        self.classifier = nn.Linear(c.hidden, c.num_labels)
        self.apply(self._init)

    def _init(self, m):
        r = self.config.init_range
        if isinstance(m, (nn.Linear, nn.Embedding)):
            nn.init.normal_(m.weight, 0.0, r)
        if isinstance(m, nn.Linear) and m.bias is not None:
            nn.init.zeros_(m.bias)
        if isinstance(m, nn.LayerNorm):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)

    @staticmethod
    def key_bias(attention_mask):
        if attention_mask is None:
            return None
        return torch.zeros(attention_mask.shape, dtype=torch.float32, device=attention_mask.device).masked_fill(
            attention_mask == 0, float('-inf'))

    def encode(self, input_ids, token_type_ids=None, attention_mask=None):
        B, S = input_ids.shape
        pos = torch.arange(S, device=input_ids.device)
        tt = token_type_ids if token_type_ids is not None else torch.zeros_like(input_ids)
        x = self.word(input_ids) + self.pos(pos)[None] + self.tok_type(tt)
        x = F.dropout(self.ln(x), self.config.hidden_dropout, self.training)
        kb = self.key_bias(attention_mask)
        for layer in self.layers:
            x = layer(x, kb)
        return x

    def forward(self, input_ids, token_type_ids=None, attention_mask=None):
        x = self.encode(input_ids, token_type_ids, attention_mask)
        pooled = torch.tanh(self.pooler(x[:, 0]))
        return self.classifier(F.dropout(pooled, self.config.hidden_dropout, self.training))


def bert(variant: str = 'bert-base', **kw) -> BertForSequenceClassification:
    cfg = dict(PRESETS[variant])
    if 'num_classes' in kw:
        kw['num_labels'] = kw.pop('num_classes')
    cfg.update(kw)
    return BertForSequenceClassification(BertConfig(**cfg))


for _v in PRESETS:
    register(_v)((lambda v: (lambda **kw: bert(v, **kw)))(_v))

__all__ = ['BertConfig', 'BertForSequenceClassification', 'BertLayer', 'bert', 'PRESETS']
