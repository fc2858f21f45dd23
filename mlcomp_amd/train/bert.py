"""BERT fine-tuning steps for the benchmark / DAG tasks: the native engine
(:class:`~mlcomp_amd.train.native_bert_step.NativeBertStep`) and the stock PyTorch-ROCm
comparison (autocast bf16, SDPA attention, fused AdamW, torch DDP over RCCL)."""
from __future__ import annotations

import os
from typing import Optional

import torch

from mlcomp_amd.models import build_model


class _TorchBertStep:
    def __init__(self, model_name, batch, seq_len, device, world_size, num_labels=2, lr=2e-5, precision='bf16'):
        torch.manual_seed(0)
        self.amp = precision != 'fp32'
        self.model = build_model(model_name, num_labels=num_labels).to(device)
        self.net = self.model
        if world_size > 1:
            from torch.nn.parallel import DistributedDataParallel as DDP
            self.net = DDP(self.model, device_ids=[device.index], gradient_as_bucket_view=True)
        decay = [p for n, p in self.model.named_parameters() if not (n.endswith('bias') or '.ln' in n or n.startswith('ln'))]
        rest = [p for n, p in self.model.named_parameters() if n.endswith('bias') or '.ln' in n or n.startswith('ln')]
        self.opt = torch.optim.AdamW([{'params': decay, 'weight_decay': 0.01}, {'params': rest, 'weight_decay': 0.0}],
                                     lr=lr, eps=1e-6, fused=True)
        rank = int(os.environ.get('RANK', '0'))
        g = torch.Generator(device=device)
        g.manual_seed(4321 + rank)
        vocab = self.model.config.vocab_size
        self.ids = torch.randint(0, vocab, (batch, seq_len), device=device, generator=g)
        self.tt = torch.zeros(batch, seq_len, dtype=torch.long, device=device)
        self.tt[:, seq_len // 2:] = 1
        self.y = torch.randint(0, num_labels, (batch,), device=device, generator=g)
        self.batch = batch
        self._loss = None

    def __call__(self):
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=self.amp):
            logits = self.net(self.ids, self.tt)
        loss = torch.nn.functional.cross_entropy(logits.float(), self.y)
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        self.opt.step()
        self._loss = loss.detach()

    def last_loss(self):
        return float(self._loss.item()) if self._loss is not None else None


def build_bert_step(model_name='bert-base', batch=32, seq_len=128, impl='native', device=None, world_size=1,
                    use_graph: Optional[bool] = None, num_labels=2, lr=2e-5, comm=None, precision='bf16'):
    device = device or torch.device('cuda')
    if impl == 'torch':
        return _TorchBertStep(model_name, batch, seq_len, device, world_size, num_labels, lr, precision)
    from .native_bert_step import NativeBertStep
    return NativeBertStep(model_name, batch=batch, seq_len=seq_len, device=device, world_size=world_size,
                          use_graph=True if use_graph is None else use_graph, num_labels=num_labels, lr=lr,
                          comm=comm)


__all__ = ['build_bert_step']
