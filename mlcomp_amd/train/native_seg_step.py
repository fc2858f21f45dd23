"""The native training step for U-Net (BASELINE config 3), LinkNet, FPN, PSPNet and DeepLab
(ResNet backbone) segmentation.

forward (fused conv+BN+ReLU nodes, fused upsample+concat) -> fused 1x1 head + BCE + Dice
-> backward (wgrad straight into the flat grad arena, bucketed RCCL all-reduce on a side
stream as buckets fill) -> one fused Adam launch per arena.  Captured into one HIP graph
after ``warmup_eager`` eager steps, exactly like :class:`NativeClassifierStep`.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from mlcomp_amd.models.native_resnet import STEM_CIN
from mlcomp_amd.models.native_deeplab import NativeDeepLab
from mlcomp_amd.models.native_fpn import NativeFPN
from mlcomp_amd.models.native_linknet import NativeLinknet
from mlcomp_amd.models.native_psp import NativePSPNet
from mlcomp_amd.models.native_unet import NativeUnet
from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.ops.layers import flatten_bn_buffers
from mlcomp_amd.parallel.comm import make_comm
from mlcomp_amd.parallel.ddp import GradBucketer
from mlcomp_amd.train.graphed import GraphedStep
from mlcomp_amd.train.optim import FusedAdam, FusedSGD


def synthetic_masks(batch, size, device, generator, classes=1):
    """Blob-shaped binary masks [batch, classes, size, size]: a smoothed random field
    thresholded at its median-ish, one independent field per class."""
    low = torch.randn(batch, classes, size // 16, size // 16, device=device, generator=generator)
    m = torch.nn.functional.interpolate(low, size=(size, size), mode='bilinear', align_corners=False)
    return (m > 0.3).float()


class NativeSegmentationStep(GraphedStep):
    def __init__(self, encoder='resnet34', batch=32, image_size=256, device=None, world_size=1, use_graph=True,
                 lr=3e-4, weight_decay=0.0, optimizer='Adam', momentum=0.9, betas=(0.9, 0.999), eps=1e-8,
                 seed=0, warmup_eager=2, torch_model=None, comm=None, classes=1, nesterov=False, dampening=0.0,
                 bce_w=1.0, dice_w=1.0, loss_eps=1e-7, arch='unet'):
        from mlcomp_amd.contrib.segmentation.models import FPN, Linknet, PSPNet, Unet
        self.device = torch.device(device or 'cuda')
        torch.manual_seed(seed)
        from mlcomp_amd.contrib.segmentation.deeplab import DeepLab
        archs = {'unet': Unet, 'linknet': Linknet, 'fpn': FPN, 'pspnet': PSPNet}
        if torch_model is None:
            if arch.lower() == 'deeplab':
                torch_model = DeepLab(backbone='resnet', num_classes=classes)
            else:
                torch_model = archs[arch.lower()](encoder_name=encoder, classes=classes)
        tm = torch_model
        engine = (NativeLinknet if isinstance(tm, Linknet) else NativeFPN if isinstance(tm, FPN)
                  else NativePSPNet if isinstance(tm, PSPNet) else NativeDeepLab if isinstance(tm, DeepLab)
                  else NativeUnet)
        self.net = engine(tm, self.device, bce_w=bce_w, dice_w=dice_w, eps=loss_eps)
        self.net.ctx.grad_prezeroed = True
        self.world = world_size
        self.comm = comm if comm is not None else (make_comm(self.device) if world_size > 1 else None)
        self.bucketer = GradBucketer(self.net.arena, self.comm)
        self.bn_buffers = flatten_bn_buffers(self.net._units())
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
        self.batch = batch
        rank = int(os.environ.get('RANK', '0'))
        g = torch.Generator(device=self.device)
        g.manual_seed(4321 + rank)
        img = torch.randn(batch, image_size, image_size, 3, device=self.device, generator=g)
        self.x = self._prep(torch.nn.functional.pad(img, (0, STEM_CIN - 3)).to(torch.bfloat16).contiguous())
        self.classes = self.net.head.K
        # targets in pixel order [N, H, W, K] (the head's NHWC layout)
        self.t = synthetic_masks(batch, image_size, self.device, g, self.classes).permute(0, 2, 3, 1).reshape(-1) \
            .contiguous()
        self.use_graph = use_graph and self.device.type == 'cuda'
        self.warmup_eager = warmup_eager
        self.graph = None
        self.calls = 0
        self._loss = None

    def _prep(self, x_nhwc):
        """The stem's space-to-depth input layout (see NativeClassifierStep._prep)."""
        if getattr(self.net.stem, 's2d', False) and x_nhwc.shape[-1] != 16:
            return Fn.stem_s2d(x_nhwc, 3)
        return x_nhwc

    def load_batch(self, images: torch.Tensor, masks: torch.Tensor):
        """Copy a batch into the static buffers: images NCHW float (or NHWC bf16 padded),
        masks [N, K, H, W] / [N, H, W] in {0, 1}."""
        x = images
        if x.dim() == 4 and x.shape[1] in (1, 3) and x.dtype != torch.bfloat16:
            x = Fn.nchw_to_nhwc(x.to(self.device, non_blocking=True).float(), pad_to=STEM_CIN)
        self.x.copy_(self._prep(x.to(self.device, non_blocking=True)))
        m = masks.to(self.device, non_blocking=True).float()
        if m.dim() == 4:               # [N, K, H, W] -> pixel order [N, H, W, K]
            m = m.permute(0, 2, 3, 1)
        self.t.copy_(m.reshape(-1))

    def _body(self):
        self.net.ctx.ws.zero()
        self.net.arena.zero_grad()
        self.bucketer.begin()
        loss = self.net.loss(self.x, self.t)
        loss.backward()
        self.bucketer.finish()
        if not self.opt_in_bwd:
            self.opt.step()
        self._end_of_step_buffers()
        self._loss = loss.detach()

    def set_lr(self, lr):
        self.opt.set_lr(lr)

    def last_loss(self) -> Optional[float]:
        return None if self._loss is None else float(self._loss.item())

    def dice(self) -> float:
        """Soft Dice of the last forward (from the head's loss sums)."""
        s = self.net.head.sums()
        return float(((2 * s[1] + 1e-7) / (s[2] + s[3] + 1e-7)).item())
