"""Native (HIP-kernel) execution of the ResNet family defined in
:mod:`mlcomp_amd.models.resnet`.

``NativeResNet(torch_model)`` lowers the module tree onto native layers
(`mlcomp_amd.ops.layers`): every ConvBNAct becomes one fused conv+BN(+residual)(+ReLU)
autograd node whose BN statistics come out of the conv epilogue, and the head fuses
avg-pool, the FC layer and softmax cross-entropy.

The stem takes the image as NHWC bf16 with channels padded 3 -> 8.  Its 7x7/2 conv runs as
a 4x4/1 conv over the 2x2 space-to-depth image (``s2d_stem``, `ops.functional.stem_s2d`:
K = 256 instead of 7x7x8 = 392 padded to 448), and BN + ReLU + 3x3/2 max-pool are one
fused pass whose backward recomputes the pool scatter inside the BN-backward passes
(``fuse_stem_pool``, `ops.layers.StemPool`, csrc/kernels/stem.hip).  Reference graph:
torchvision-style ResNet as built by the reference's classify presets
(`mlcomp/contrib/catalyst/configs/classify/resnet50.yml`).

Weights are copied into the flat arenas once; ``export_to_torch()`` writes them back
(for checkpoints in the standard PyTorch layout).
"""
from __future__ import annotations

import torch

from mlcomp_amd.ops.layers import ClassifierHead, ConvBN, MaxPool, NativeContext, ResidualBlock, StemPool
from .resnet import BasicBlock, Bottleneck, ResNet

STEM_CIN = 8


def lower_resnet_body(ctx: NativeContext, model: ResNet, prefix: str = '', s2d_stem: bool = False):
    """Lower the stem and the four residual stages of ``model`` onto native layers.
    Returns (stem ConvBN, MaxPool, [ResidualBlock], index of the last block of each stage).
    Consecutive blocks are linked (``prev``) so a block's first dgrad pre-reduces the
    previous block's output BN."""
    if model.groups != 1:
        raise NotImplementedError('native ResNet path supports groups=1 (use impl=torch)')
    stem_m = model.stem
    s2d = s2d_stem and tuple(stem_m.conv.weight.shape[1:]) == (3, 7, 7) and stem_m.conv.stride[0] == 2 \
        and stem_m.conv.padding[0] == 3
    stem = ConvBN(ctx, f'{prefix}stem', stem_m.conv, stem_m.bn, act=True, cin_pad=STEM_CIN, s2d=s2d)
    pool = MaxPool(3, 2, 1)
    blocks, ends = [], []
    for li in range(1, 5):
        for bi, blk in enumerate(getattr(model, f'layer{li}')):
            pre = f'{prefix}layer{li}.{bi}'
            units = []
            if isinstance(blk, Bottleneck):
                names = ('cb1', 'cb2', 'cb3')
            elif isinstance(blk, BasicBlock):
                names = ('cb1', 'cb2')
            else:
                raise TypeError(type(blk))
            for nm in names:
                cb = getattr(blk, nm)
                units.append(ConvBN(ctx, f'{pre}.{nm}', cb.conv, cb.bn, act=cb.act))
            down = None
            if blk.downsample is not None:
                d = blk.downsample.cb
                down = ConvBN(ctx, f'{pre}.downsample.cb', d.conv, d.bn, act=False)
            rb = ResidualBlock(units, down)
            rb.prev = blocks[-1] if blocks else None
            blocks.append(rb)
        ends.append(len(blocks) - 1)
    return stem, pool, blocks, ends


class NativeResNet:
    def __init__(self, model: ResNet, device, smoothing: float = 0.0, fuse_stem_pool: bool = True,
                 s2d_stem: bool = True):
        self.torch_model = model
        ctx = self.ctx = NativeContext()
        # split-K weight gradients with atomics, not slabs + a reduce pass: 13,264-13,318 ->
        # 13,348-13,393 img/s at 512 (interleaved, profiles/round5/wgrad_slab_ab.txt)
        ctx.default_wgrad_slab(False)
        self.stem, self.pool, self.blocks, _ = lower_resnet_body(ctx, model, s2d_stem=s2d_stem)
        # the classifier never reads the un-pooled stem activation: fuse BN+ReLU+maxpool
        self.stem_pool = StemPool(self.stem) if fuse_stem_pool else None
        self.head = ClassifierHead(ctx, 'fc', model.fc, smoothing)
        ctx.finalize(device)
        for u in self._units():
            u.load_from_torch()
        self.head.load_from_torch()
        ctx.arena.decay.refresh_mirror()

    def _units(self):
        yield self.stem
        for blk in self.blocks:
            yield from blk.units
            if blk.down is not None:
                yield blk.down

    # ------------------------------------------------------------------ execution
    def features(self, x):
        anchor = self.ctx.anchor
        if self.stem_pool is not None:
            x = self.stem_pool(x)
        else:
            x = self.stem(x)
            x = self.pool(x, anchor)
        for blk in self.blocks:
            x = blk(x)
        self.ctx.refresh_wt()    # transposed filters for the backward's dgrads
        return x

    def loss(self, x, labels):
        """Summed cross-entropy (fp32 [1] view of the workspace)."""
        return self.head(self.features(x), labels)

    def logits(self, x):
        return self.head.logits(self.features(x))

    def train(self, mode=True):
        self.ctx.training = mode
        return self

    def eval(self):
        return self.train(False)

    @property
    def arena(self):
        return self.ctx.arena

    def export_to_torch(self):
        for u in self._units():
            u.export_to_torch()
        self.head.export_to_torch()
        return self.torch_model

    def num_params(self):
        return self.ctx.arena.num_params()
