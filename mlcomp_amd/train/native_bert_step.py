"""Native BERT fine-tuning step (the BASELINE "BERT-base fine-tune DAG" config).

embeddings+LN -> N native encoder layers -> pooler/classifier/softmax-CE -> backward
(weights' gradients straight into the flat arena, RCCL buckets all-reduced on the side
stream as they complete) -> fused AdamW per arena.  Captured into one HIP graph after
``warmup_eager`` eager steps, like the ResNet step; the dropout seed is a device scalar
advanced inside the graph.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from mlcomp_amd.models import build_model
from mlcomp_amd.models.native_bert import NativeBert
from mlcomp_amd.parallel.comm import make_comm
from mlcomp_amd.parallel.ddp import GradBucketer
from mlcomp_amd.train.graphed import GraphedStep
from mlcomp_amd.train.optim import FusedAdam, FusedSGD


class NativeBertStep(GraphedStep):
    def __init__(self, model_name='bert-base', batch=32, seq_len=128, device=None, world_size=1, use_graph=True,
                 num_labels=2, lr=2e-5, weight_decay=0.01, betas=(0.9, 0.999), eps=1e-6, seed=0, warmup_eager=2,
                 torch_model=None, dropout: Optional[float] = None, comm=None, optimizer='AdamW',
                 momentum=0.0, nesterov=False, dampening=0.0):
        self.device = torch.device(device or 'cuda')
        torch.manual_seed(seed)
        kw = {'num_labels': num_labels}
        if dropout is not None:
            kw.update(hidden_dropout=dropout, attention_dropout=dropout)
        tm = torch_model if torch_model is not None else build_model(model_name, **kw)
        self.net = NativeBert(tm, self.device, batch, seq_len)
        self.net.ctx.grad_prezeroed = True
        self.world = world_size
        self.comm = comm if comm is not None else (make_comm(self.device) if world_size > 1 else None)
        self.bucketer = GradBucketer(self.net.arena, self.comm)
        self.bucketer.broadcast_params()
        if optimizer in ('Adam', 'AdamW'):
            self.opt = FusedAdam(self.net.arena, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                 decoupled=optimizer == 'AdamW', grad_scale=1.0 / world_size)
        elif optimizer == 'SGD':
            self.opt = FusedSGD(self.net.arena, lr=lr, momentum=momentum, weight_decay=weight_decay,
                                nesterov=nesterov, dampening=dampening, grad_scale=1.0 / world_size)
        else:
            raise ValueError(f'native optimizers: SGD / Adam / AdamW, not {optimizer!r}')
        # optimizer-in-backward (MLC_OPT_IN_BWD=1): each gradient bucket is updated on the side
        # stream as soon as it is complete (and all-reduced).  Measured slower on MI355X
        # (profiles/round2_ab): the memory-bound update competes with the memory-bound
        # backward passes, so the default is one update launch per arena after backward.
        self.opt_in_bwd = os.environ.get('MLC_OPT_IN_BWD', '0') == '1'
        if self.opt_in_bwd:
            self.bucketer.attach_optimizer(self.opt)
        self.batch, self.seq_len = batch, seq_len
        rank = int(os.environ.get('RANK', '0'))
        g = torch.Generator(device=self.device)
        g.manual_seed(4321 + rank)
        c = self.net.c
        self.ids = torch.randint(0, c.vocab_size, (batch, seq_len), device=self.device, generator=g)
        self.tt = torch.zeros(batch, seq_len, dtype=torch.long, device=self.device)
        self.tt[:, seq_len // 2:] = 1
        self.key_bias = None
        self.y = torch.randint(0, num_labels, (batch,), device=self.device, generator=g)
        self.net.seed.fill_(seed * 7919 + rank)
        self.use_graph = use_graph and self.device.type == 'cuda'
        self.warmup_eager = warmup_eager
        self.graph = None
        self.calls = 0

    def _check_ids(self, ids):
        """Token ids past the vocabulary would make the embedding gather read out of bounds
        on the GPU (a device fault): refuse them while they are still on the host."""
        v = self.net.c.vocab_size
        if ids.device.type == 'cpu' and ids.numel() and (int(ids.max()) >= v or int(ids.min()) < 0):
            raise ValueError(f'token ids must be in [0, {v}) for this model (got [{int(ids.min())}, {int(ids.max())}])')

    def load_batch(self, ids, labels, token_type_ids=None, attention_mask=None):
        self._check_ids(ids)
        self.ids.copy_(ids.to(self.device, non_blocking=True))
        self.y.copy_(labels.to(self.device, non_blocking=True))
        if token_type_ids is not None:
            self.tt.copy_(token_type_ids.to(self.device, non_blocking=True))
        if attention_mask is not None:
            kb = torch.zeros(attention_mask.shape, device=self.device).masked_fill(
                attention_mask.to(self.device) == 0, float('-inf'))
            if self.key_bias is None:
                if self.graph is not None:
                    raise RuntimeError('attention masks must be enabled before the graph is captured')
                self.key_bias = kb
            else:
                self.key_bias.copy_(kb)

    def predict(self, ids, token_type_ids=None, attention_mask=None):
        """Native inference logits [B, num_labels] for one (eval) batch."""
        self._check_ids(ids)
        ids = ids.to(self.device)
        tt = token_type_ids.to(self.device) if token_type_ids is not None else torch.zeros_like(ids)
        kb = None
        if attention_mask is not None:
            kb = torch.zeros(attention_mask.shape, device=self.device).masked_fill(
                attention_mask.to(self.device) == 0, float('-inf'))
        return self.net.predict(ids, tt, kb)

    def _body(self):
        net = self.net
        net.ctx.ws.zero()
        net.arena.zero_grad()
        net.seed.add_(1)
        self.bucketer.begin()
        loss = net.loss(self.ids, self.tt, self.key_bias, self.y)
        loss.backward()
        self.bucketer.finish()
        if not self.opt_in_bwd:
            self.opt.step()

    def set_lr(self, lr):
        self.opt.set_lr(lr)

    def last_loss(self) -> float:
        return float(self.net.loss_sum().item()) / self.batch

    def accuracy(self) -> float:
        return float(self.net.correct().item()) / self.batch


__all__ = ['NativeBertStep']
