"""Generic native lowering: any ``nn.Module`` onto the HIP kernels, through torch.fx.

The reference trains whatever model an experiment returns
(`mlcomp/worker/executors/catalyst_/catalyst_.py:365-430`): its own examples' LeNet and
CIFAR nets (`examples/digit-recognizer/model.py:8-25`, `examples/cifar_simple/model.py:8-26`),
the contrib zoo (`mlcomp/contrib/model/pretrained.py`), segmentation encoders
(`mlcomp/contrib/segmentation/encoders/__init__.py:12-18`).  The hand-lowered engines cover
seven architectures; this module covers the rest:

1. ``torch.fx.symbolic_trace`` the model twice (train and eval mode: ``self.training``
   branches, dropout and drop-path are baked in at trace time).
2. Pattern-match the graph and replace each match by one native call site
   (:mod:`mlcomp_amd.ops.glayers`):

   * ``Conv2d [-> BatchNorm2d [-> + residual]] [-> activation]`` -> ``ConvBNAct``: dense
     convs on the implicit-GEMM MFMA kernels (BN statistics in the epilogue; without BN
     the bias and a ReLU in the epilogue), grouped convs on the 16x16x32 MFMA block-diagonal
     kernels, depthwise convs on the VALU kernels (``gconv.hip``); BN apply + residual +
     any of 10 activations in one pass (``normact.hip``);
   * ``BatchNorm2d / BatchNorm1d [-> + residual] [-> activation]`` -> ``BNAct``;
   * ``Linear [-> ReLU]`` -> ``LinearAct`` (bias / ReLU in the dense GEMM epilogue);
   * ``MaxPool2d`` / ``F.max_pool2d`` -> ``MaxPool``; ``AdaptiveAvgPool2d(1)`` ->
     ``GlobalAvgPool``, ``AdaptiveAvgPool2d(k > 1)`` -> ``AdaptiveAvgPool``; ``x.view`` -> ``x.reshape`` (site outputs are channels_last views).

   A fused chain needs each intermediate value to have exactly one user; every op left in
   the graph (adds, concats, upsampling, dropout, sigmoid gates, the loss ...) is a PyTorch
   tensor op on bf16 activations - no MIOpen / hipBLASLt / rocBLAS call remains, and a
   module that would need one raises :class:`NativeUnsupported` (``engine: auto`` then
   trains the stage on the torch engine and records why).
3. Every parameter lives in the flat arena: the lowered modules' weights in kernel layout
   (bf16 mirror for the GEMMs), any other parameter (a LayerNorm a torch op still uses, a
   learned scale) aliased in place - its ``.data`` and ``.grad`` become arena views - so
   one fused optimizer launch per arena and the RCCL bucketer cover the whole model.
"""
from __future__ import annotations

import operator
import os
from typing import Dict, Optional, Tuple

import torch
import torch.fx as fx
import torch.nn as nn
import torch.nn.functional as F

from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.ops.glayers import (AdaptiveAvgPool, AvgPool, BilinearUp, BNAct, BNParams, ChannelGate, Conv3dAs2d,
                                    ConvBNAct, ConvParams, DenseCat, DenseChain, Frames, GlobalAvgPool, GradAcc, LinearAct, LinearParams,
                                    MaxPool, TemporalAs2d, UpCat, VolumePool)
from mlcomp_amd.ops import gtransformer as GT
from mlcomp_amd.ops.layers import NativeContext
from mlcomp_amd.train.native_spec import NativeUnsupported

A = Fn.ACT
_ACT_MODULES = {nn.ReLU: A['relu'], nn.ReLU6: A['relu6'], nn.SiLU: A['silu'], nn.Sigmoid: A['sigmoid'],
                nn.Tanh: A['tanh'], nn.Hardswish: A['hardswish'], nn.LeakyReLU: A['leaky_relu'],
                nn.GELU: A['gelu'], nn.ELU: A['elu'], nn.Hardsigmoid: A['hardsigmoid']}
_ACT_FUNCS = {F.relu: A['relu'], torch.relu: A['relu'], torch.relu_: A['relu'], F.relu_: A['relu'],
              F.relu6: A['relu6'], F.silu: A['silu'], torch.sigmoid: A['sigmoid'], torch.tanh: A['tanh'],
              F.hardswish: A['hardswish'], F.leaky_relu: A['leaky_relu'], F.gelu: A['gelu'], F.elu: A['elu'],
              F.hardsigmoid: A['hardsigmoid']}
_ACT_METHODS = {'relu': A['relu'], 'relu_': A['relu'], 'sigmoid': A['sigmoid'], 'sigmoid_': A['sigmoid'],
                'tanh': A['tanh'], 'tanh_': A['tanh']}
_ADDS = {operator.add, operator.iadd, torch.add}


def _is_module(node, modules, types):
    return node.op == 'call_module' and isinstance(modules.get(node.target), types)


def _act_of(node: fx.Node, modules) -> Optional[Tuple[int, float]]:
    """(code, alpha) when ``node`` applies a supported activation to its first input."""
    if node.op == 'call_module':
        m = modules.get(node.target)
        code = _ACT_MODULES.get(type(m))
        if code is None:
            return None
        if isinstance(m, nn.GELU) and m.approximate != 'none':
            return None
        alpha = float(getattr(m, 'negative_slope', getattr(m, 'alpha', 0.0)))
        return code, alpha
    if node.op == 'call_function' and node.target in _ACT_FUNCS:
        extra = [a for a in node.args[1:] if isinstance(a, fx.Node)]
        if extra or any(isinstance(v, fx.Node) for v in node.kwargs.values()):
            return None
        if node.target is F.gelu and node.kwargs.get('approximate', 'none') != 'none':
            return None
        alpha = 0.0
        if node.target is F.leaky_relu:
            alpha = float(node.args[1] if len(node.args) > 1 else node.kwargs.get('negative_slope', 0.01))
        elif node.target is F.elu:
            alpha = float(node.args[1] if len(node.args) > 1 else node.kwargs.get('alpha', 1.0))
        return _ACT_FUNCS[node.target], alpha
    if node.op == 'call_method' and node.target in _ACT_METHODS and len(node.args) == 1:
        return _ACT_METHODS[node.target], 0.0
    return None


def _residual_of(node: fx.Node, cur: fx.Node) -> Optional[fx.Node]:
    """The other operand when ``node`` is ``cur + other`` (tensor + tensor, no alpha)."""
    if node.kwargs.get('alpha', 1) != 1:
        return None
    if node.op == 'call_function' and node.target in _ADDS and len(node.args) == 2:
        a, b = node.args
    elif node.op == 'call_method' and node.target in ('add', 'add_') and len(node.args) == 2:
        a, b = node.args
    else:
        return None
    if not (isinstance(a, fx.Node) and isinstance(b, fx.Node)):
        return None
    if a is cur and b is not cur:
        return b
    if b is cur and a is not cur:
        return a
    return None


def _only_user(node: fx.Node) -> Optional[fx.Node]:
    users = list(node.users)
    return users[0] if len(users) == 1 else None


def _pair(v, name):
    if isinstance(v, (tuple, list)):
        if len(set(v)) != 1:
            raise NativeUnsupported(f'{name}={tuple(v)}: the native kernels take square {name}s')
        return int(v[0])
    return int(v)


def _check_conv(name, m: nn.Conv2d):
    if m.padding_mode != 'zeros':
        raise NativeUnsupported(f'{name}: padding_mode={m.padding_mode!r}')
    if isinstance(m.padding, str):
        raise NativeUnsupported(f'{name}: padding={m.padding!r}')
    for attr in ('stride', 'dilation'):
        _pair(getattr(m, attr), f'{name}.{attr}')
    if m.groups != 1:
        _pair(m.padding, f'{name}.padding')        # grouped / depthwise kernels: one pad
    KH, KW = m.kernel_size
    if KH > 15 or KW > 15:
        raise NativeUnsupported(f'{name}: kernel {KH}x{KW} (native convs take <= 15x15)')
    Co, Cg = m.weight.shape[:2]
    if m.groups > 1:
        C = Cg * m.groups
        if m.groups == C and Co == C:
            return
        if not Fn.gconv_ok(C, Co, m.groups):
            raise NativeUnsupported(f'{name}: grouped conv {C}->{Co} x{m.groups} groups (native: channels % 8 == 0 '
                                    'and a bounded block-diagonal span)')


def _check_convT(name, m: nn.ConvTranspose2d):
    if m.padding_mode != 'zeros' or m.groups != 1:
        raise NativeUnsupported(f'{name}: ConvTranspose2d with groups={m.groups}, padding_mode={m.padding_mode!r}')
    for attr in ('stride', 'padding', 'dilation', 'output_padding'):
        _pair(getattr(m, attr), f'{name}.{attr}')
    KH, KW = m.kernel_size
    if KH > 15 or KW > 15:
        raise NativeUnsupported(f'{name}: kernel {KH}x{KW} (native convs take <= 15x15)')


def _check_conv3d(name, m):
    """nn.Conv3d / nn.Conv1d: any temporal (length) kernel, stride, padding and dilation
    (unfolded into channels); the spatial part follows the 2D rules."""
    if m.padding_mode != 'zeros' or isinstance(m.padding, str):
        raise NativeUnsupported(f'{name}: padding={m.padding!r}, padding_mode={m.padding_mode!r}')
    if isinstance(m, nn.Conv3d):
        for attr in ('stride', 'padding', 'dilation'):
            _pair(getattr(m, attr)[1:], f'{name}.{attr} (spatial)')
    _check_conv(name, Conv3dAs2d(m))


def _check_bn(name, m):
    if m.momentum is None:
        raise NativeUnsupported(f'{name}: BatchNorm momentum=None (cumulative average)')


class _Lowering:
    """One fx graph rewrite (train or eval) sharing the net's parameter sets."""

    def __init__(self, net: 'GenericNet', gm: fx.GraphModule):
        self.net, self.gm = net, gm
        self.modules = dict(gm.named_modules())
        self.erased = set()
        self.nsites = 0

    def _site_node(self, after: fx.Node, site, args):
        name = f'_native_site_{self.nsites}'
        self.nsites += 1
        self.gm.add_submodule(name, site)
        with self.gm.graph.inserting_after(after):
            return self.gm.graph.call_module(name, tuple(args))

    def _replace(self, chain, new):
        chain[-1].replace_all_uses_with(new)
        for n in reversed(chain):
            self.gm.graph.erase_node(n)
            self.erased.add(n)

    def _tail(self, cur, chain, allow_res=True):
        """Extend a chain with an optional residual add and activation: (res, act, alpha)."""
        res, act, alpha = None, 0, 0.0
        u = _only_user(cur)
        if allow_res and u is not None and _residual_of(u, cur) is not None:
            res = _residual_of(u, cur)
            chain.append(u)
            cur = u
            u = _only_user(cur)
        if u is not None:
            a = _act_of(u, self.modules)
            if a is not None:
                act, alpha = a
                chain.append(u)
        return res, act, alpha

    def conv(self, node):
        m = self.modules[node.target]
        if isinstance(m, nn.ConvTranspose2d):
            _check_convT(node.target, m)
        else:
            _check_conv(node.target, m)
        chain = [node]
        bn_node = _only_user(node)
        bn = None
        if bn_node is not None and _is_module(bn_node, self.modules, nn.BatchNorm2d):
            bm = self.modules[bn_node.target]
            if bm.num_features == m.out_channels and bm.momentum is not None:
                bn = bm
        # an image stem (7x7/2 pad 3 over <= 3 channels) reading the graph input: the
        # space-to-depth form (MLC_GENERIC_S2D=0 keeps the direct 7x7 conv)
        src = node.args[0]
        s2d = (os.environ.get('MLC_GENERIC_S2D', '1') == '1' and isinstance(src, fx.Node)
               and src.op == 'placeholder' and ConvParams.s2d_ok(m))
        if bn is not None:
            chain.append(bn_node)
            res, act, alpha = self._tail(bn_node, chain)
            cp = self.net.conv_params(node.target, m, keep_bias=False, s2d=s2d)
            bp = self.net.bn_params(bn_node.target, bn, conv_bias=m.bias)
        else:
            res, act, alpha = self._tail(node, chain, allow_res=False)
            cp = self.net.conv_params(node.target, m, keep_bias=True, s2d=s2d)
            bp = None
        site = ConvBNAct(self.net.ctx, cp, bp, act, alpha, residual=res is not None)
        new = self._site_node(chain[-1], site, [node.args[0]] + ([res] if res is not None else []))
        self._replace(chain, new)

    def conv3d(self, node):
        """Conv3d / Conv1d [-> BatchNorm3d / BatchNorm1d [-> + residual]] [-> act] -> a
        ``ConvBNAct`` over frames (temporal taps unfolded into channels), wrapped in
        ``Frames``."""
        m = self.modules[node.target]
        _check_conv3d(node.target, m)
        # purely temporal stride-1 convs run over the [N, T, H*W, C] view (no unfold copy)
        proxy = TemporalAs2d(m) if TemporalAs2d.applies(m) else Conv3dAs2d(m)
        chain = [node]
        bn_node = _only_user(node)
        bn = None
        bn_type = nn.BatchNorm3d if isinstance(m, nn.Conv3d) else nn.BatchNorm1d
        if bn_node is not None and _is_module(bn_node, self.modules, bn_type):
            bm = self.modules[bn_node.target]
            if bm.num_features == m.out_channels and bm.momentum is not None:
                bn = bm
        if bn is not None:
            chain.append(bn_node)
            res, act, alpha = self._tail(bn_node, chain)
            cp = self.net.conv_params(node.target, proxy, keep_bias=False)
            bp = self.net.bn_params(bn_node.target, bn, conv_bias=m.bias)
        else:
            res, act, alpha = self._tail(node, chain, allow_res=False)
            cp = self.net.conv_params(node.target, proxy, keep_bias=True)
            bp = None
        site = Frames(ConvBNAct(self.net.ctx, cp, bp, act, alpha, residual=res is not None), proxy, name=node.target)
        new = self._site_node(chain[-1], site, [node.args[0]] + ([res] if res is not None else []))
        self._replace(chain, new)

    def maxpool3d(self, node, m):
        k, s, p = (m.kernel_size,) * 3 if isinstance(m.kernel_size, int) else m.kernel_size, m.stride, m.padding
        s = k if s is None else ((s,) * 3 if isinstance(s, int) else s)
        p = (p,) * 3 if isinstance(p, int) else p
        d = (m.dilation,) * 3 if isinstance(m.dilation, int) else m.dilation
        if k[0] != 1 or s[0] != 1 or p[0] != 0 or d[0] != 1:
            raise NativeUnsupported(f'{node.target}: MaxPool3d with a temporal window {k[0]}/{s[0]}/{p[0]} '
                                    '(native: spatial-only 3D pooling)')
        ks, ss, ps, ds = _pair(k[1:], 'kernel_size'), _pair(s[1:], 'stride'), _pair(p[1:], 'padding'), \
            _pair(d[1:], 'dilation')
        if ds != 1 or m.return_indices or ks * ks > 255:
            raise NativeUnsupported(f'{node.target}: MaxPool3d(dilation={ds}, return_indices={m.return_indices})')
        site = Frames(MaxPool(self.net.ctx, ks, ss, ps, bool(m.ceil_mode)))
        new = self._site_node(node, site, [node.args[0]])
        self._replace([node], new)

    def bn(self, node):
        m = self.modules[node.target]
        _check_bn(node.target, m)
        chain = [node]
        res, act, alpha = self._tail(node, chain)
        site = BNAct(self.net.ctx, self.net.bn_params(node.target, m), act, alpha, residual=res is not None)
        new = self._site_node(chain[-1], site, [node.args[0]] + ([res] if res is not None else []))
        self._replace(chain, new)

    def _mlp(self, node, m) -> bool:
        """Linear -> exact GELU -> Linear [-> + residual] (each value used once) -> MlpSite."""
        g = _only_user(node)
        if g is None or _act_of(g, self.modules) != (A['gelu'], 0.0):
            return False
        n2 = _only_user(g)
        if n2 is None or not _is_module(n2, self.modules, nn.Linear) or n2.args[0] is not g or len(n2.args) != 1:
            return False
        m2 = self.modules[n2.target]
        if m.out_features % 8 or m.in_features % 8 or m2.out_features % 8 or m2.in_features != m.out_features:
            return False
        chain = [node, g, n2]
        res = None
        u = _only_user(n2)
        if u is not None and _residual_of(u, n2) is not None:
            res = _residual_of(u, n2)
            chain.append(u)
        site = GT.MlpSite(self.net.ctx, self.net.linear_params(node.target, m), self.net.linear_params(n2.target, m2),
                          residual=res is not None)
        new = self._site_node(chain[-1], site, [node.args[0]] + ([res] if res is not None else []))
        self._replace(chain, new)
        return True

    def linear(self, node):
        m = self.modules[node.target]
        if self._mlp(node, m):
            return
        chain = [node]
        u = _only_user(node)
        act = 0
        if u is not None and _act_of(u, self.modules) == (A['relu'], 0.0):
            act = 3                       # the dense epilogue's ReLU code
            chain.append(u)
        elif u is not None and _act_of(u, self.modules) == (A['gelu'], 0.0):
            # exact GELU in the GEMM epilogue, gelu' stored for the backward
            chain.append(u)
            site = GT.LinearGelu(self.net.ctx, self.net.linear_params(node.target, m))
            new = self._site_node(chain[-1], site, [node.args[0]])
            self._replace(chain, new)
            return
        res = None
        if act == 0 and m.out_features % 8 == 0 and u is not None and _residual_of(u, node) is not None:
            res = _residual_of(u, node)          # y = x W^T + b + r: the add in the epilogue
            chain.append(u)
        site = LinearAct(self.net.ctx, self.net.linear_params(node.target, m), act, residual=res is not None)
        new = self._site_node(chain[-1], site, [node.args[0]] + ([res] if res is not None else []))
        self._replace(chain, new)

    def avgpool2d(self, node, k, s, p, ceil=False, cip=True, div=None):
        """A square, floor-mode average pool without a divisor override -> ``AvgPool``
        (others stay torch ops)."""
        try:
            k, s, p = _pair(k, 'kernel_size'), _pair(s if s is not None else k, 'stride'), _pair(p, 'padding')
        except NativeUnsupported:
            return
        if ceil or div is not None or not isinstance(node.args[0], fx.Node):
            return
        new = self._site_node(node, AvgPool(self.net.ctx, k, s, p, bool(cip)), [node.args[0]])
        self._replace([node], new)

    def maxpool(self, node, k, s, p, d=1, ceil=False, ret=False):
        k, s, p, d = _pair(k, 'kernel_size'), _pair(s if s is not None else k, 'stride'), _pair(p, 'padding'), \
            _pair(d, 'dilation')
        if d != 1 or ret or k * k > 255:
            raise NativeUnsupported(f'max_pool2d(k={k}, dilation={d}, return_indices={ret})')
        src = node.args[0]
        site = self.modules.get(src.target) if isinstance(src, fx.Node) and src.op == 'call_module' else None
        if site is None and isinstance(src, fx.Node) and src.op == 'call_module':
            site = getattr(self.gm, src.target, None)
        if ((k, s, p, bool(ceil)) == (3, 2, 1, False) and isinstance(site, ConvBNAct) and site.bn is not None
                and site.act == A['relu'] and not site.residual and len(src.users) == 1
                and site.conv.Co == site.conv.Cop and Fn.stem_pool_ok(site.conv.Cop)):
            # conv -> BN -> ReLU -> 3x3/2 max-pool (a ResNet stem): one fused pass (stem.hip)
            object.__setattr__(site, 'pool3', True)
            node.replace_all_uses_with(src)
            self.gm.graph.erase_node(node)
            self.erased.add(node)
            return
        new = self._site_node(node, MaxPool(self.net.ctx, k, s, p, bool(ceil)), [node.args[0]])
        self._replace([node], new)

    def interpolate(self, node):
        """F.interpolate: nearest x2 [-> torch.cat([up, skip], 1)] -> ``UpCat`` (one NHWC pass,
        the U-Net decoder input); bilinear with align_corners=True -> ``BilinearUp``.  Other
        modes stay torch ops."""
        names = ('input', 'size', 'scale_factor', 'mode', 'align_corners', 'recompute_scale_factor', 'antialias')
        a = dict(zip(names, node.args))
        a.update(node.kwargs)
        x, size, scale = a.get('input'), a.get('size'), a.get('scale_factor')
        mode, align = a.get('mode', 'nearest'), a.get('align_corners')
        if a.get('recompute_scale_factor') or a.get('antialias') or not isinstance(x, fx.Node):
            return
        if isinstance(scale, (tuple, list)):
            scale = tuple(float(s) for s in scale) if len(set(scale)) == 1 or mode == 'bilinear' else None
        elif isinstance(scale, (int, float)):
            scale = (float(scale), float(scale))
        if mode == 'nearest' and size is None and scale == (2.0, 2.0):
            chain, skip = [node], None
            u = _only_user(node)
            if u is not None and u.op == 'call_function' and u.target is torch.cat:
                seq = u.args[0]
                dim = u.kwargs.get('dim', u.args[1] if len(u.args) > 1 else 0)
                if (dim == 1 and isinstance(seq, (list, tuple)) and len(seq) == 2 and seq[0] is node
                        and isinstance(seq[1], fx.Node) and seq[1] is not node):
                    skip = seq[1]
                    chain.append(u)
            new = self._site_node(chain[-1], UpCat(self.net.ctx), [x] + ([skip] if skip is not None else []))
            self._replace(chain, new)
        elif mode == 'bilinear' and align is True and (size is not None or scale is not None):
            if size is not None:
                new = self._site_node(node, BilinearUp(self.net.ctx), [x, size])
            else:
                new = self._site_node(node, BilinearUp(self.net.ctx, scale), [x])
            self._replace([node], new)

    def _gate_source(self, g: fx.Node, depth: int = 8):
        """The value whose global average a gate ``g`` is computed from (walking back through
        single-input sites and activations to a GlobalAvgPool site), or None."""
        for _ in range(depth):
            if not isinstance(g, fx.Node):
                return None
            if g.op == 'call_module':
                m = getattr(self.gm, g.target, None)
                if isinstance(m, GlobalAvgPool):
                    return g.args[0]
                if not (isinstance(m, (ConvBNAct, LinearAct, BNAct)) or _act_of(g, self.modules) is not None):
                    return None
                if len(g.args) != 1:
                    return None
            elif not (g.op in ('call_function', 'call_method') and _act_of(g, self.modules) is not None):
                return None
            g = g.args[0]
        return None

    def _channels(self, n: fx.Node, depth: int = 8):
        """Channel count of the value ``n`` when a native site (walking back through
        elementwise activations) says so, else None."""
        for _ in range(depth):
            if not isinstance(n, fx.Node):
                return None
            m = getattr(self.gm, n.target, None) if n.op == 'call_module' else None
            if isinstance(m, ConvBNAct):
                return m.conv.Co
            if isinstance(m, LinearAct):
                return m.lin.O
            if isinstance(m, BNAct):
                return m.bn.C
            if isinstance(m, ChannelGate) or _act_of(n, self.modules) is not None:
                n = n.args[0]
                continue
            return None
        return None

    def gate(self, node):
        """``y * g`` where g is computed from y's global average (squeeze-excitation) ->
        ChannelGate.  Only a per-channel gate lowers: g's producing site must output as many
        channels as y has (a per-sample [N, 1, 1, 1] gate is a valid torch broadcast and
        stays a torch op)."""
        if len(node.args) != 2 or node.kwargs:
            return
        a, b = node.args
        if not (isinstance(a, fx.Node) and isinstance(b, fx.Node)) or a is b:
            return
        if self._gate_source(b) is a:
            y, g = a, b
        elif self._gate_source(a) is b:
            y, g = b, a
        else:
            return
        cg, cy = self._channels(g), self._channels(y)
        if cg is None or cg != cy:
            return
        # SE-ResNeXt's block tail: (y * g) + residual -> ReLU in the same pass
        chain = [node]
        res, act, alpha = self._tail(node, chain)
        if act not in (0, A['relu']):       # another activation: gate only, the rest stays torch
            chain, res, act = [node], None, 0
        site = ChannelGate(self.net.ctx, relu=act == A['relu'], residual=res is not None)
        new = self._site_node(chain[-1], site, [y, g] + ([res] if res is not None else []))
        self._replace(chain, new)

    def avgpool(self, node):
        new = self._site_node(node, GlobalAvgPool(self.net.ctx), [node.args[0]])
        self._replace([node], new)

    def adaptive_pool(self, node, size):
        """adaptive_avg_pool2d to a fixed size > 1 (PSPNet's 2 / 3 / 6 pyramid levels)."""
        so = tuple(size) if isinstance(size, (tuple, list)) else (size, size)
        if len(so) != 2 or any(v is None for v in so):
            raise NativeUnsupported(f'{node.name}: adaptive_avg_pool2d output_size={size!r}')
        if so == (1, 1):
            return self.avgpool(node)
        new = self._site_node(node, AdaptiveAvgPool(self.net.ctx, so[0], so[1]), [node.args[0]])
        self._replace([node], new)

    def volume_pool(self, node, m):
        """AdaptiveAvgPool3d(1) / AdaptiveAvgPool1d(1) -> VolumePool; AdaptiveAvgPool1d(K) of
        ``x.reshape(N, 1, -1)`` (the ResNeXt3D head) -> VolumePool(flat_bins=K) on x."""
        out = m.output_size
        sizes = tuple(out) if isinstance(out, (tuple, list)) else (out,)
        src = node.args[0]
        if all(v == 1 for v in sizes):
            new = self._site_node(node, VolumePool(self.net.ctx), [src])
            self._replace([node], new)
            return
        if (isinstance(m, nn.AdaptiveAvgPool1d) and isinstance(src, fx.Node) and src.op == 'call_method'
                and src.target in ('reshape', 'view') and len(src.args) == 4 and src.args[2] == 1
                and src.args[3] == -1 and len(src.users) == 1):
            new = self._site_node(node, VolumePool(self.net.ctx, flat_bins=int(sizes[0])), [src.args[0]])
            self._replace([src, node], new)

    # ------------------------------------------------------------------ transformer blocks
    @staticmethod
    def _call_args(node, names):
        a = dict(zip(names, node.args))
        a.update(node.kwargs)
        return a

    def layernorm(self, node):
        """nn.LayerNorm [over ``a + b`` whose only user it is] -> LayerNormSite (the add
        fused into the normalisation pass); unsupported configurations stay torch ops."""
        m = self.modules[node.target]
        if GT.LNParams.supported(m) is not None or len(node.args) != 1:
            return
        x = node.args[0]
        lp = self.net.ln_params(node.target, m)
        chain, inputs = [node], [x]
        if isinstance(x, fx.Node) and len(x.users) == 1:
            for cand in x.args[:2] if len(x.args) >= 2 else ():
                r = _residual_of(x, cand) if isinstance(cand, fx.Node) else None
                if r is not None:
                    inputs = [cand, r]
                    chain = [x, node]
                    break
        site = GT.LayerNormSite(self.net.ctx, lp, residual=len(inputs) == 2)
        new = self._site_node(node, site, inputs)
        self._replace(chain, new)

    def _getitem_users(self, node):
        """{index: user} of a tuple-returning call whose every user is ``out[i]``; None when
        some user takes the tuple itself."""
        out = {}
        for u in node.users:
            if not (u.op == 'call_function' and u.target is operator.getitem and isinstance(u.args[1], int)):
                return None
            out.setdefault(u.args[1], []).append(u)
        return out

    def mha(self, node):
        m = self.modules[node.target]
        why = GT.mha_supported(m)
        if why:
            raise NativeUnsupported(f'{node.target}: {why}')
        a = self._call_args(node, ('query', 'key', 'value', 'key_padding_mask', 'need_weights', 'attn_mask',
                                   'average_attn_weights', 'is_causal'))
        q = a.get('query')
        if a.get('key') is not q or a.get('value') is not q:
            raise NativeUnsupported(f'{node.target}: MultiheadAttention lowers for self-attention only (q = k = v)')
        if a.get('attn_mask') is not None or a.get('is_causal'):
            raise NativeUnsupported(f'{node.target}: MultiheadAttention attn_mask / is_causal (native: a key-padding '
                                    'mask only)')
        users = self._getitem_users(node)
        if users is None or any(u.users for i, us in users.items() if i != 0 for u in us):
            raise NativeUnsupported(f'{node.target}: MultiheadAttention attention weights are used (native: the '
                                    'output only)')
        kpm = a.get('key_padding_mask')
        site = GT.MHASite(self.net.ctx, self.net.mha_params(node.target, m))
        new = self._site_node(node, site, [q] + ([kpm] if kpm is not None else []))
        for i, us in users.items():
            for u in us:
                if i == 0:
                    u.replace_all_uses_with(new)
                self.gm.graph.erase_node(u)
                self.erased.add(u)
        self.gm.graph.erase_node(node)
        self.erased.add(node)

    def encoder(self, node, layers, norm):
        """nn.TransformerEncoderLayer / nn.TransformerEncoder -> EncoderSite."""
        for i, layer in enumerate(layers):
            why = GT.encoder_layer_supported(layer)
            if why:
                raise NativeUnsupported(f'{node.target}: {why}')
        names = ('src', 'mask', 'src_key_padding_mask', 'is_causal')
        a = self._call_args(node, names)
        if a.get('src_mask') is not None or a.get('mask') is not None or a.get('is_causal'):
            raise NativeUnsupported(f'{node.target}: an attention mask / is_causal (native: a key-padding mask only)')
        if norm is not None and GT.LNParams.supported(norm) is not None:
            raise NativeUnsupported(f'{node.target}: final norm: {GT.LNParams.supported(norm)}')
        if len({bool(l.self_attn.batch_first) for l in layers}) != 1:
            raise NativeUnsupported(f'{node.target}: layers disagree on batch_first')
        single = len(layers) == 1 and isinstance(self.modules[node.target], nn.TransformerEncoderLayer)
        lps = [self.net.encoder_params(node.target if single else f'{node.target}.layers.{i}', l)
               for i, l in enumerate(layers)]
        lnp = self.net.ln_params(f'{node.target}.norm', norm) if norm is not None else None
        kpm = a.get('src_key_padding_mask')
        site = GT.EncoderSite(self.net.ctx, lps, lnp)
        new = self._site_node(node, site, [a['src']] + ([kpm] if kpm is not None else []))
        self._replace([node], new)

    def _packed_qkv(self, q, k, v):
        """timm's packed projection ``L.reshape(B, N, 3, H, D).permute(2, 0, 3, 1, 4)`` split
        into q / k / v (``unbind(0)`` or ``[0] / [1] / [2]``): (L, H, chain nodes) or None."""
        def split(n):
            if not (isinstance(n, fx.Node) and n.op == 'call_function' and n.target is operator.getitem
                    and isinstance(n.args[1], int)):
                return None
            src = n.args[0]
            if src.op in ('call_method', 'call_function') and getattr(src.target, '__name__', src.target) == 'unbind':
                dim = src.args[1] if len(src.args) > 1 else src.kwargs.get('dim', 0)
                return (src.args[0], n.args[1], src) if dim == 0 else None
            return src, n.args[1], None
        parts = [split(t) for t in (q, k, v)]
        if any(p is None for p in parts) or [p[1] for p in parts] != [0, 1, 2] or len({id(p[0]) for p in parts}) != 1:
            return None
        perm, _, unb = parts[0]
        if not (perm.op == 'call_method' and perm.target == 'permute'):
            return None
        dims = perm.args[1:] if len(perm.args) > 2 else perm.args[1]
        if tuple(dims) != (2, 0, 3, 1, 4):
            return None
        rs = perm.args[0]
        if not (rs.op == 'call_method' and rs.target in ('reshape', 'view') and len(rs.args) == 6 and rs.args[3] == 3
                and isinstance(rs.args[4], int)):
            return None
        chain = [n for n in (q, k, v)] + ([unb] if unb is not None else []) + [perm, rs]
        return rs.args[0], int(rs.args[4]), chain

    def sdpa(self, node):
        a = self._call_args(node, ('query', 'key', 'value', 'attn_mask', 'dropout_p', 'is_causal', 'scale',
                                   'enable_gqa'))
        if a.get('attn_mask') is not None or a.get('is_causal') or a.get('enable_gqa'):
            raise NativeUnsupported(f'{node.name}: scaled_dot_product_attention with a mask / is_causal / GQA '
                                    '(native: unmasked self-attention)')
        p, scale = a.get('dropout_p', 0.0), a.get('scale')
        if isinstance(p, fx.Node) or isinstance(scale, fx.Node):
            raise NativeUnsupported(f'{node.name}: scaled_dot_product_attention with a traced dropout_p / scale')
        packed = self._packed_qkv(a['query'], a['key'], a['value'])
        if packed is not None and all(len(n.users) == 1 for n in packed[2][:3]):
            # zero-copy: the projection's [B, N, 3E] output IS the kernel's qkv layout
            L, H, chain = packed
            site = GT.SDPASite(self.net.ctx, float(p or 0.0), None if scale is None else float(scale), heads=H)
            new = self._site_node(node, site, [L])
            self._replace([node], new)
            for n in chain:
                if not n.users and n not in self.erased:
                    self.gm.graph.erase_node(n)
                    self.erased.add(n)
            return
        site = GT.SDPASite(self.net.ctx, float(p or 0.0), None if scale is None else float(scale))
        new = self._site_node(node, site, [a['query'], a['key'], a['value']])
        self._replace([node], new)

    def patch_embed(self, node, m):
        """A conv with stride == kernel and no padding whose kernel is beyond the
        implicit-GEMM engine (ViT's 16x16/16 patch embedding) -> one dense GEMM."""
        k = _pair(m.kernel_size, 'kernel_size')
        if (_pair(m.stride, 'stride') != k or _pair(m.padding, 'padding') != 0 or _pair(m.dilation, 'dilation') != 1
                or m.groups != 1 or m.padding_mode != 'zeros' or (m.in_channels * k * k) % 8 or m.out_channels % 8):
            raise NativeUnsupported(f'{node.target}: kernel {m.kernel_size} (native convs take <= 15x15; larger ones '
                                    'only as a stride = kernel patch embedding)')
        d = self.net.dense_set(node.target, m.weight, m.bias)
        new = self._site_node(node, GT.PatchEmbed(self.net.ctx, d, k, m.in_channels), [node.args[0]])
        self._replace([node], new)

    def _link_residuals(self):
        """Identity residuals: a value R used exactly twice - as the input of a 2D conv site
        S1 and as the residual of a conv site S3 downstream of it - gets one gradient:
        S3's backward hands its residual gradient to S1, whose dgrad adds it in the GEMM
        epilogue (autograd would add the two branch gradients in a pass of its own).
        S3's backward runs before S1's (S3 depends on S1's output)."""
        mods = dict(self.gm.named_modules())
        for n in self.gm.graph.nodes:
            s3 = mods.get(n.target) if n.op == 'call_module' else None
            if not isinstance(s3, ConvBNAct) or not s3.residual or len(n.args) < 2:
                continue
            r = n.args[1]
            users = [u for u in r.users]
            if len(users) != 2:
                continue
            other = users[0] if users[1] is n else users[1]
            s1 = mods.get(other.target) if other.op == 'call_module' else None
            if (not isinstance(s1, ConvBNAct) or s1 is s3 or other.args[0] is not r
                    or (len(other.args) > 1 and other.args[1] is r) or s1.conv.Cip != s3.conv.Cop):
                continue
            if not self._reaches(other, n):
                continue
            object.__setattr__(s3, 'res_link', s1)

    def _fuse_drop_path(self):
        """Stochastic depth before a residual add - ``add(truediv(mul(s, mask), keep), x)`` with
        s a conv+BN site (no activation, no residual) and mask = rand_like(s[:, :1, :1, :1]) < keep
        (EfficientNet's MBConv in training): the site takes x as its residual and the mask as a
        third input and applies mask / keep to its BN output in the same pass.  The mask's
        shape source is re-pointed at the site's input (same batch), so it no longer depends
        on the site."""
        mods = dict(self.gm.named_modules())
        adds = {operator.add, torch.add}
        for n in list(self.gm.graph.nodes):
            if n.op != 'call_function' or n.target not in adds or len(n.args) != 2 or n.kwargs:
                continue
            for t, x in (n.args, n.args[::-1]):
                if not (isinstance(t, fx.Node) and isinstance(x, fx.Node) and t.op == 'call_function'
                        and t.target is operator.truediv and len(t.args) == 2 and isinstance(t.args[1], float)
                        and len(t.users) == 1):
                    continue
                m, keep = t.args
                if not (isinstance(m, fx.Node) and m.op == 'call_function' and m.target in (operator.mul, torch.mul)
                        and len(m.args) == 2 and len(m.users) == 1):
                    continue
                s_node, mask = m.args
                site = mods.get(s_node.target) if isinstance(s_node, fx.Node) and s_node.op == 'call_module' else None
                if not (isinstance(site, ConvBNAct) and site.bn is not None and site.act == 0 and not site.residual
                        and len(s_node.args) == 1 and isinstance(mask, fx.Node) and mask.op == 'call_function'
                        and mask.target is operator.lt):
                    continue
                rl = mask.args[0]
                gi = rl.args[0] if isinstance(rl, fx.Node) and rl.op == 'call_function' and rl.args else None
                while (isinstance(gi, fx.Node) and gi.op == 'call_method' and gi.target in ('float', 'to', 'double')
                       and len(gi.users) == 1):           # dtype casts of the shape source
                    gi = gi.args[0]
                if not (isinstance(gi, fx.Node) and gi.op == 'call_function' and gi.target is operator.getitem
                        and gi.args[0] is s_node and set(s_node.users) == {m, gi} and len(gi.users) == 1):
                    continue
                gi.args = (s_node.args[0],) + tuple(gi.args[1:])
                s_node.args = (s_node.args[0], x, mask)
                mask.append(s_node)              # after the mask (and x, which precedes the block)
                n.replace_all_uses_with(s_node)
                for dead in (n, t, m):
                    self.gm.graph.erase_node(dead)
                object.__setattr__(site, 'residual', True)
                object.__setattr__(site, 'drop_keep', float(keep))
                break

    def _fold_shortcut_bns(self):
        """A conv+BN site D without activation or residual whose output is only the residual
        input of a conv+BN site S (a bottleneck's downsample shortcut): S applies D's BN as
        its residual's affine in its own apply pass, so D skips its apply pass (the hand
        ResNet engine's fold; in backward the residual gradient S returns is that BN's
        output gradient, D's BN backward unchanged)."""
        mods = dict(self.gm.named_modules())
        for n in self.gm.graph.nodes:
            s = mods.get(n.target) if n.op == 'call_module' else None
            if not isinstance(s, ConvBNAct) or s.bn is None or not s.residual or len(n.args) < 2:
                continue
            r = n.args[1]
            d = mods.get(r.target) if isinstance(r, fx.Node) and r.op == 'call_module' else None
            if (not isinstance(d, ConvBNAct) or d is s or d.bn is None or d.act != 0 or d.residual
                    or len(r.users) != 1 or n.args[0] is r or d.conv.Cop != s.conv.Cop or d.conv.Co != d.conv.Cop):
                continue
            object.__setattr__(s, 'res_bn', d)
            object.__setattr__(d, 'bn_folded', True)

    def _link_dgrads(self):
        """A value that is the conv input of exactly two dense conv sites P (earlier in the
        graph) and Q (later) - a residual block's first conv and its downsample shortcut -
        where Q's backward runs before P's: Q depends on P (the shortcut site that also sums
        the block), or Q's only user is a site P reaches (once that user's backward ran, Q is
        ready no later than P and, created later, runs first: autograd's ready queue takes
        the higher sequence number).  Q hands its input gradient to P's dgrad epilogue (no
        autograd add), so P's epilogue holds the value's whole gradient (which lets the
        value's producer link its BN backward to P)."""
        mods = dict(self.gm.named_modules())
        order = {n: i for i, n in enumerate(self.gm.graph.nodes)}
        for x in self.gm.graph.nodes:
            users = sorted(x.users, key=order.get)
            if len(users) != 2:
                continue
            sites = [mods.get(u.target) if u.op == 'call_module' else None for u in users]
            if not all(isinstance(s, ConvBNAct) and s.conv.kind == 'dense' and u.args[0] is x
                       and not (len(u.args) > 1 and u.args[1] is x) for s, u in zip(sites, users)):
                continue
            (p, q), (sp, sq) = users, sites
            qu = list(q.users)
            q_first = self._reaches(p, q) or (len(qu) == 1 and self._reaches(p, qu[0]))
            if sp is sq or sp.conv.Cip != sq.conv.Cip or sq.grad_link is not None or sp.grad_expected or not q_first:
                continue
            object.__setattr__(sq, 'grad_link', sp)
            object.__setattr__(sp, 'grad_expected', True)

    def _link_frames(self):
        """The 3D residual blocks' two-branch gradients, summed in the temporal fold kernel
        instead of by autograd's add (glayers.Frames): a 5D value V used exactly twice,

        * as the unfolded input of a Conv3d site S1 and as the identity residual of a site S3
          downstream of it: S3's backward hands its residual gradient to S1 (``res_link``),
          whose fold adds it;
        * as the unfolded input of two Conv3d sites P and Q (a block's first conv and its
          shortcut conv, Q's backward first - the rule of :meth:`_link_dgrads`): Q's fold
          output is handed to P (``send_to``), whose fold adds it."""
        mods = dict(self.gm.named_modules())
        order = {n: i for i, n in enumerate(self.gm.graph.nodes)}

        def unfolding(s):
            return isinstance(s, Frames) and isinstance(s._conv, Conv3dAs2d) and isinstance(s.site, ConvBNAct)

        for v in self.gm.graph.nodes:
            users = sorted(v.users, key=order.get)
            if len(users) != 2 or not all(u.op == 'call_module' for u in users):
                continue
            (a, b), (sa, sb) = users, [mods.get(u.target) for u in users]
            if not (unfolding(sa) and unfolding(sb)) or sa is sb:
                continue
            # identity residual: one user takes V as its residual (only), the other as input
            for s1n, s1, s3n, s3 in ((a, sa, b, sb), (b, sb, a, sa)):
                if (s1n.args[0] is v and not (len(s1n.args) > 1 and s1n.args[1] is v) and len(s3n.args) > 1
                        and s3n.args[1] is v and s3n.args[0] is not v and s3.site.residual
                        and s3.site.conv.Cop == s3.site.conv.Co and s3.site.res_link is None
                        and not s1.grad_expected and self._reaches(s1n, s3n)):
                    object.__setattr__(s3.site, 'res_link', s1)
                    object.__setattr__(s1, 'grad_expected', True)
                    break
            else:
                # two sibling convs over V
                if not all(u.args[0] is v and not (len(u.args) > 1 and u.args[1] is v) for u in users):
                    continue
                qu = list(b.users)
                if not (self._reaches(a, b) or (len(qu) == 1 and self._reaches(a, qu[0]))):
                    continue
                if sb.send_to is not None or sa.grad_expected or sa.send_to is not None:
                    continue
                object.__setattr__(sb, 'send_to', sa)
                object.__setattr__(sa, 'grad_expected', True)

    def _link_fanout(self):
        """A value consumed (as their only / first input) by two or more sites that take an
        addend in their backward kernels - conv sites (dgrad epilogue), average / global
        pools, squeeze-excitation gates - and not already in a two-site hand-off: they share
        a :class:`GradAcc`, so the value's gradient is summed inside those kernels in any
        backward order (Inception's branch points: three convs and a pool per block; an SE
        block's input: its pool and its gate); other users' gradients are still added by
        autograd."""
        mods = dict(self.gm.named_modules())
        res_targets = {id(getattr(m, 'res_link', None)) for m in mods.values() if getattr(m, 'res_link', None) is not None}
        for v in self.gm.graph.nodes:
            members = []
            for u in v.users:
                s = mods.get(u.target) if u.op == 'call_module' else None
                if not u.args or u.args[0] is not v or any(a is v for a in u.args[1:]):
                    continue
                if isinstance(s, ConvBNAct):
                    if (s.grad_link is not None or s.grad_expected or id(s) in res_targets
                            or s.acc is not None):
                        members = None
                        break
                    members.append(s)
                elif isinstance(s, (AvgPool, GlobalAvgPool, ChannelGate)) and s.acc is None:
                    members.append(s)
            if not members or len(members) < 2:
                continue
            cps = {m.conv.Cip for m in members if isinstance(m, ConvBNAct)}
            if any(isinstance(m, (AvgPool, GlobalAvgPool, ChannelGate)) for m in members):
                # the pool pads channels to a multiple of 8: the convs' input width says how many
                cis = {m.conv.Ci for m in members if isinstance(m, ConvBNAct)}
                c = self._channels(v) if not cis else (cis.pop() if len(cis) == 1 else None)
                cps.add(None if c is None else -(-c // 8) * 8)
            if len(cps) != 1 or None in cps:       # one NHWC layout for the running sum
                continue
            acc = GradAcc(v.name)
            for m in members:
                object.__setattr__(m, 'acc', acc)

    def _link_cat_stats(self):
        """A BN site over ``torch.cat([a, b], 1)`` where ``a`` is also the input of an earlier
        BN site A (DenseNet: x_{i+1} = cat(x_i, layer_i(x_i)), layer_i starting with A's BN):
        the site copies a's per-channel statistics from A and reduces only b (glayers.BNAct
        .cat_prev) - each layer's statistics pass reads its 32 new channels, not the whole
        concatenation."""
        mods = dict(self.gm.named_modules())
        for n in list(self.gm.graph.nodes):
            sb = mods.get(n.target) if n.op == 'call_module' else None
            if not isinstance(sb, BNAct) or len(n.args) != 1 or n.kwargs or sb.residual:
                continue
            cat = n.args[0]
            if not (isinstance(cat, fx.Node) and cat.op == 'call_function' and cat.target is torch.cat):
                continue
            parts = cat.args[0] if cat.args else cat.kwargs.get('tensors')
            dim = cat.args[1] if len(cat.args) > 1 else cat.kwargs.get('dim', 0)
            if dim != 1 or not isinstance(parts, (list, tuple)) or len(parts) != 2:
                continue
            a, b = parts
            if not (isinstance(a, fx.Node) and isinstance(b, fx.Node)):
                continue
            prev = [u for u in a.users if u.op == 'call_module' and isinstance(mods.get(u.target), BNAct)
                    and u.args and u.args[0] is a and u is not n]
            if len(prev) != 1:
                continue
            sa = mods[prev[0].target]
            cb = self._channels(b)
            if (sa.cat_prev is sb or sa.bn.C != sa.bn.Cp or cb is None or cb % 8 or sb.bn.Cp != sa.bn.C + cb
                    or sb.bn.C != sb.bn.Cp or not self._reaches(prev[0], b)):
                continue
            object.__setattr__(sb, 'cat_prev', sa)
            n.args = (cat, b)

    def _lower_dense_cats(self):
        """``torch.cat([a, b], 1)`` where ``a``'s only other user is a BN site A that ``b``
        depends on (a DenseNet layer): a :class:`DenseCat` site, whose backward hands a's
        gradient slice to A's apply pass instead of autograd adding a strided slice to A's
        input gradient."""
        mods = dict(self.gm.named_modules())
        for cat in list(self.gm.graph.nodes):
            if cat.op != 'call_function' or cat.target is not torch.cat or cat in self.erased:
                continue
            parts = cat.args[0] if cat.args else cat.kwargs.get('tensors')
            dim = cat.args[1] if len(cat.args) > 1 else cat.kwargs.get('dim', 0)
            if dim != 1 or not isinstance(parts, (list, tuple)) or len(parts) != 2:
                continue
            a, b = parts
            if not (isinstance(a, fx.Node) and isinstance(b, fx.Node)) or a is b:
                continue
            others = [u for u in a.users if u is not cat]
            if len(others) != 1 or others[0].op != 'call_module':
                continue
            sa = mods.get(others[0].target)
            nargs = 2 if isinstance(sa, BNAct) and sa.cat_prev is not None else 1     # (x, concat tail)
            if (not isinstance(sa, BNAct) or len(others[0].args) != nargs or others[0].args[0] is not a or sa.residual
                    or sa.bn.C != sa.bn.Cp or sa.slice_expected or not self._reaches(others[0], b)):
                continue
            site = DenseCat(self.net.ctx, sa)
            new = self._site_node(cat, site, [a, b])
            self._replace([cat], new)
            object.__setattr__(sa, 'slice_expected', True)

    def _chain_dense_cats(self):
        """Runs of :class:`DenseCat` sites each over the previous one's output (a DenseNet block)
        share one concat buffer (glayers.DenseChain).  An inner concatenation's only users are
        the next DenseCat and its layer's first BN site (``_lower_dense_cats`` checked that),
        and both read the buffer's leading channels in place.  ``MLC_DENSE_CHAIN=0``: off (A/B)."""
        if os.environ.get('MLC_DENSE_CHAIN', '1') != '1':
            return
        mods = dict(self.gm.named_modules())

        def dense_cat(n):
            return isinstance(n, fx.Node) and n.op == 'call_module' and isinstance(mods.get(n.target), DenseCat)

        runs = []
        for n in self.gm.graph.nodes:
            if not dense_cat(n):
                continue
            site = mods[n.target]
            a, b = n.args[0], n.args[1]
            ca, cb = site.a_site.bn.C, self._channels(b)
            if cb is None or cb % 8 or ca % 8:
                continue
            prev = mods[a.target] if dense_cat(a) else None
            run = next((r for r in runs if prev is not None and r[-1][0] is prev), None)
            if run is not None and run[-1][1] == ca and len(a.users) == 2:     # n and its layer's BN
                run.append((site, ca + cb))
            else:
                runs.append([(site, ca + cb)])
        node_of = {mods[n.target]: n for n in self.gm.graph.nodes if dense_cat(n)}
        for run in runs:
            if len(run) < 2:
                continue
            chain = DenseChain(run[-1][1])
            for site, _ in run:
                object.__setattr__(site, 'chain', chain)
                self._cat_out(node_of[site], site)
            object.__setattr__(run[0][0], 'chain_first', True)
            object.__setattr__(run[-1][0], 'chain_last', True)

    def _split_cat_grads(self):
        """A DenseCat whose output's gradient comes from one BN site X alone (its other users
        are DenseCats, whose backward hands their first operand's gradient on instead of
        returning it): X's apply pass stores that gradient as the two operands' gradients, each
        dense (BNAct.split_to) - no strided slice of it is copied for the growth conv's
        backward.  ``MLC_DENSE_CHAIN=0``: off (A/B)."""
        if os.environ.get('MLC_DENSE_CHAIN', '1') != '1':
            return
        mods = dict(self.gm.named_modules())
        for n in self.gm.graph.nodes:
            d = mods.get(n.target) if n.op == 'call_module' else None
            if not isinstance(d, DenseCat):
                continue
            xs = [u for u in n.users if u.op == 'call_module' and isinstance(mods.get(u.target), BNAct)
                  and u.args and u.args[0] is n]
            cats = [u for u in n.users if u.op == 'call_module' and isinstance(mods.get(u.target), DenseCat)
                    and u.args[0] is n and u.args[1] is not n]
            if len(xs) != 1 or len(xs) + len(cats) != len(n.users) or xs[0].args[1:].count(n):
                continue
            x = mods[xs[0].target]
            if (x.residual or x.acc is not None or x.bn.C != x.bn.Cp or d.off % 8 or not 0 < d.off < x.bn.C
                    or x.split_to is not None):
                continue
            object.__setattr__(x, 'split_to', d)
            object.__setattr__(d, 'split_expected', True)

    def _cat_out(self, n: fx.Node, site):
        """The new segment b of chained DenseCat ``n``: a plain dense conv (no BN / bias /
        activation / residual) whose other users only take b's statistics in place (the next
        BN's concat tail) writes its output straight into the block's concat buffer."""
        b = n.args[1]
        conv = getattr(self.gm, b.target, None) if isinstance(b, fx.Node) and b.op == 'call_module' else None
        if (not isinstance(conv, ConvBNAct) or conv.bn is not None or conv.conv.kind != 'dense' or conv.conv.b is not None
                or conv.act or conv.residual or conv.epi_act or conv.conv.Co != conv.conv.Cop or len(b.args) != 1):
            return
        for u in b.users:
            m = getattr(self.gm, u.target, None) if u.op == 'call_module' else None
            if u is not n and not (isinstance(m, BNAct) and m.cat_prev is not None and len(u.args) == 2
                                   and u.args[1] is b and u.args[0] is not b):
                return
        object.__setattr__(conv, 'cat_out', site)

    def _link_bn_backward(self):
        """A conv+BN site A (ReLU or no activation, batch statistics) whose output is used
        only as the input of a dense conv site B (and, at a residual block boundary, as the
        identity residual that B's dgrad already sums): B's dgrad epilogue produces A's whole
        output gradient, so it also applies A's ReLU mask and accumulates A's BatchNorm-
        backward sums (Fn.BnBwdSpec) and A's backward skips its reduction pass."""
        mods = dict(self.gm.named_modules())
        relu = A['relu']
        for n in self.gm.graph.nodes:
            sb = mods.get(n.target) if n.op == 'call_module' else None
            if not isinstance(sb, ConvBNAct) or sb.conv.kind != 'dense' or not n.args:
                continue
            a = n.args[0]
            sa = mods.get(a.target) if isinstance(a, fx.Node) and a.op == 'call_module' else None
            if (not isinstance(sa, ConvBNAct) or sa is sb or sa.bn is None or sa.act not in (0, relu)
                    or sa.conv.Cop != sb.conv.Cip or sa.pool3 or sa.drop_keep is not None):
                continue
            others = [u for u in a.users if u is not n]
            # the only other user may be a site whose residual gradient (an identity-residual
            # link) or input gradient (a sibling-conv hand-off) B's dgrad already sums: B's
            # dgrad output is then A's whole output gradient
            o = mods.get(others[0].target) if len(others) == 1 and others[0].op == 'call_module' else None
            if others and not (o is not None and (getattr(o, 'res_link', None) is sb
                                                  or getattr(o, 'grad_link', None) is sb)):
                continue
            if len(n.args) > 1 and n.args[1] is a:
                continue
            object.__setattr__(sb, 'bn_link', sa)
            object.__setattr__(sa, 'bn_prereduced', True)
            if sa.res_bn is not None:       # its folded shortcut BN is reduced there as well
                object.__setattr__(sa.res_bn, 'bn_prereduced', True)

    @staticmethod
    def _reaches(a: fx.Node, b: fx.Node) -> bool:
        """True when node ``b`` depends on node ``a`` (so ``a``'s backward runs after ``b``'s)."""
        seen, todo = set(), [b]
        while todo:
            x = todo.pop()
            if x is a:
                return True
            for p in x.all_input_nodes:
                if p not in seen:
                    seen.add(p)
                    todo.append(p)
        return False

    def _prepass(self):
        """Before pattern matching: p = 0 dropouts and Identity modules are no ops (so they
        never split a fusable chain); float parameters that torch ops read (class tokens,
        position embeddings, layer scales) enter the graph in bf16, the engine's compute
        dtype, as autocast feeds a matmul - so the residual streams they start stay bf16."""
        g = self.gm.graph
        for node in list(g.nodes):
            if node.op == 'call_module':
                m = self.modules.get(node.target)
                if isinstance(m, (nn.Dropout, nn.Identity)) and getattr(m, 'p', 0.0) == 0.0 \
                        and len(node.args) == 1 and not node.kwargs:
                    node.replace_all_uses_with(node.args[0])
                    g.erase_node(node)
            elif node.op == 'get_attr' and os.environ.get('MLC_GENERIC_PARAM_BF16', '1') == '1':
                try:
                    t = self.gm.get_parameter(node.target)
                except AttributeError:
                    continue
                if not t.is_floating_point():
                    continue
                with g.inserting_after(node):
                    cast = g.call_method('to', (node, torch.bfloat16))
                node.replace_all_uses_with(cast)
                cast.args = (node, torch.bfloat16)

    def run(self):
        g = self.gm.graph
        self._prepass()
        for node in list(g.nodes):
            if node in self.erased:
                continue
            if node.op == 'call_module':
                m = self.modules.get(node.target)
                if isinstance(m, nn.Conv2d) and max(m.kernel_size) > 15:
                    self.patch_embed(node, m)
                elif isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
                    self.conv(node)
                elif isinstance(m, (nn.Conv3d, nn.Conv1d)):
                    self.conv3d(node)
                elif isinstance(m, (nn.BatchNorm2d, nn.BatchNorm1d, nn.BatchNorm3d)):
                    self.bn(node)
                elif isinstance(m, nn.MaxPool3d):
                    self.maxpool3d(node, m)
                elif isinstance(m, nn.Linear):
                    self.linear(node)
                elif isinstance(m, nn.MaxPool2d):
                    self.maxpool(node, m.kernel_size, m.stride, m.padding, m.dilation, m.ceil_mode, m.return_indices)
                elif isinstance(m, nn.AdaptiveAvgPool2d):
                    self.adaptive_pool(node, m.output_size)
                elif isinstance(m, nn.AvgPool2d):
                    self.avgpool2d(node, m.kernel_size, m.stride, m.padding, m.ceil_mode, m.count_include_pad,
                                   m.divisor_override)
                elif isinstance(m, (nn.AdaptiveAvgPool3d, nn.AdaptiveAvgPool1d)):
                    self.volume_pool(node, m)
                elif isinstance(m, nn.LayerNorm):
                    self.layernorm(node)
                elif isinstance(m, nn.MultiheadAttention):
                    self.mha(node)
                elif isinstance(m, nn.TransformerEncoderLayer):
                    self.encoder(node, [m], None)
                elif isinstance(m, nn.TransformerEncoder):
                    self.encoder(node, list(m.layers), m.norm)
                elif isinstance(m, (nn.ConvTranspose1d, nn.ConvTranspose3d, nn.LSTM, nn.GRU, nn.RNN,
                                    nn.TransformerDecoder, nn.TransformerDecoderLayer, nn.Transformer,
                                    nn.Bilinear, nn.InstanceNorm2d)):
                    raise NativeUnsupported(f'{node.target}: {type(m).__name__} has no native lowering')
            elif node.op == 'call_function':
                t = node.target
                if t in (F.max_pool2d, torch.max_pool2d):
                    args = list(node.args) + [None] * 6
                    kw = node.kwargs
                    self.maxpool(node, kw.get('kernel_size', args[1]), kw.get('stride', args[2]),
                                 kw.get('padding', args[3] if args[3] is not None else 0),
                                 kw.get('dilation', args[4] if args[4] is not None else 1),
                                 kw.get('ceil_mode', args[5] or False), kw.get('return_indices', args[6] or False))
                elif t in (F.avg_pool2d, torch._C._nn.avg_pool2d):
                    args = list(node.args) + [None] * 6
                    kw = node.kwargs
                    k = kw.get('kernel_size', args[1])
                    st = kw.get('stride', args[2])
                    self.avgpool2d(node, k, st if st not in (None, []) else k,
                                   kw.get('padding', args[3] if args[3] is not None else 0),
                                   kw.get('ceil_mode', args[4] or False),
                                   kw.get('count_include_pad', args[5] if args[5] is not None else True),
                                   kw.get('divisor_override', args[6]))
                elif t is F.interpolate:
                    self.interpolate(node)
                elif t in (operator.mul, torch.mul):
                    self.gate(node)
                elif t is F.adaptive_avg_pool2d:
                    self.adaptive_pool(node, node.args[1] if len(node.args) > 1 else node.kwargs['output_size'])
                elif t is F.scaled_dot_product_attention:
                    self.sdpa(node)
                elif t in (F.conv2d, torch.conv2d, F.linear, torch.matmul, torch.mm, torch.bmm, torch.addmm,
                           F.batch_norm, torch.einsum, F.conv_transpose2d, operator.matmul):
                    raise NativeUnsupported(f'{node.name}: functional {getattr(t, "__name__", t)} on module '
                                            'parameters has no native lowering (use the nn modules)')
            elif node.op == 'call_method':
                if node.target == 'view':
                    node.target = 'reshape'     # site outputs are channels_last views
                elif node.target == 'mul':
                    self.gate(node)
                elif node.target in ('matmul', 'mm', 'bmm'):
                    raise NativeUnsupported(f'{node.name}: Tensor.{node.target} has no native lowering')
        self._fuse_drop_path()
        self._fold_shortcut_bns()
        self._link_residuals()
        self._link_dgrads()
        self._link_frames()
        self._link_fanout()
        self._link_cat_stats()
        self._lower_dense_cats()
        self._chain_dense_cats()
        self._split_cat_grads()
        self._link_bn_backward()
        g.lint()
        self.gm.delete_all_unused_submodules()
        self.gm.recompile()
        return self.gm


class GenericNet:
    """A model lowered onto the native kernels: ``net(x)`` runs the train or eval graph
    (``train()`` / ``eval()``), parameters live in ``net.ctx.arena``."""

    def __init__(self, model: nn.Module, device):
        self.torch_model = model
        self.device = torch.device(device)
        ctx = self.ctx = NativeContext()
        # split-K conv weight gradients with atomics (ResNet-50 @512 12.89-12.96k -> 13.06-13.11k
        # img/s, profiles/round5/wgrad_slab_ab.txt)
        ctx.default_wgrad_slab(False)
        # MLC_GENERIC_WT=1 (default): dense convs keep a transposed, flipped filter copy for
        # their input gradients (Fn.WtTable, refreshed once per training forward), as the
        # hand engines do; 0: the dgrads read the filters directly
        ctx.wt = Fn.WtTable() if os.environ.get('MLC_GENERIC_WT', '1') == '1' else None
        ctx.grad_prezeroed = True          # the step zeroes the grad arena once
        self._params: Dict[str, object] = {}
        self._composite: Dict[str, object] = {}    # MHA / encoder-layer groupings of _params
        was = model.training
        model.to(self.device)
        try:
            model.train()
            self.train_gm = self._lower(model)
            model.eval()
            self.eval_gm = self._lower(model)
        except NativeUnsupported:
            raise
        except Exception as e:             # fx cannot trace data-dependent control flow
            raise NativeUnsupported(f'{type(model).__name__}: torch.fx tracing failed ({type(e).__name__}: '
                                    f'{str(e).splitlines()[0] if str(e) else ""})') from e
        finally:
            model.train(was)
        self._alias_residual_params(model)
        # a BatchNorm called from one site of the training graph writes dgamma / dbeta straight
        # into the (per-step zeroed) grad arena; a shared one accumulates through a scratch
        uses = {}
        for site in self.train_gm.modules():
            bn = getattr(site, 'bn', None)
            if isinstance(bn, BNParams):
                uses[id(bn)] = uses.get(id(bn), 0) + 1
        for p in self._params.values():
            if isinstance(p, BNParams):
                p.single_site = uses.get(id(p), 0) == 1
        ctx.finalize(self.device)
        # dropout seed of the kernels' counter-hash masks (transformer sites), advanced on the
        # device by every training forward, so captured replays draw fresh masks
        ctx.seed = torch.zeros(1, device=self.device, dtype=torch.int32)
        # weight gradients as one unjoined side chain, each forked before its site's input
        # gradient (BERT's and the segmentation engines' schedule).  Interleaved A/B on one
        # MI355X (profiles/round5/generic/bench_ab_defer.jsonl): ResNeXt-50 @128 7,451 ->
        # 7,721 img/s, EfficientNet-b0 @256 10,291 -> 10,925, U-Net-ResNeXt-50 @16 561 -> 580;
        # ResNet-50 @512 12,831 -> 12,750 (its long GEMMs prefer the per-site join:
        # MLC_WGRAD_DEFER=0 MLC_DGRAD_FIRST=0)
        ctx.default_wgrad_defer(True)
        ctx.default_dgrad_first(True)
        for p in self._params.values():
            p.load_from_torch()
        self._bind_residual()
        ctx.arena.decay.refresh_mirror()
        self.training = True

    # ------------------------------------------------------------------ lowering
    def _lower(self, model):
        gm = fx.symbolic_trace(model)
        return _Lowering(self, gm).run()

    def conv_params(self, name, m, keep_bias, s2d=False):
        key = f'conv:{name}:{keep_bias}:{s2d}'
        if key not in self._params:
            self._params[key] = ConvParams(self.ctx, name, m, keep_bias, s2d=s2d)
        return self._params[key]

    def bn_params(self, name, m, conv_bias=None):
        key = f'bn:{name}'
        if key not in self._params:
            p = BNParams(self.ctx, name, m)
            p.conv_bias = conv_bias        # a bias before a batch-stat BN only shifts its mean
            self._params[key] = p
        return self._params[key]

    def linear_params(self, name, m):
        key = f'linear:{name}'
        if key not in self._params:
            self._params[key] = LinearParams(self.ctx, name, m)
        return self._params[key]

    def dense_set(self, name, weight, bias):
        key = f'dense:{name}'
        if key not in self._params:
            self._params[key] = GT.DenseSet(self.ctx, name, weight, bias)
        return self._params[key]

    def ln_params(self, name, m):
        key = f'ln:{name}'
        if key not in self._params:
            self._params[key] = GT.LNParams(self.ctx, name, m)
        return self._params[key]

    def mha_params(self, name, m):
        key = f'mha:{name}'
        if key not in self._composite:
            self._composite[key] = GT.MHAParams(self.dense_set, name, m)
        return self._composite[key]

    def encoder_params(self, name, layer):
        key = f'encoder:{name}'
        if key not in self._composite:
            self._composite[key] = GT.EncoderLayerParams(self.dense_set, self.ln_params, name, layer)
        return self._composite[key]

    def _alias_residual_params(self, model):
        """Parameters no site owns (read by torch ops left in the graph) get arena slots too."""
        owned = set()
        for p in self._params.values():
            for attr in ('weight', 'bias'):
                t = getattr(p.src, attr, None)
                if isinstance(t, torch.Tensor):
                    owned.add(id(t))
        self._residual = []
        for name, t in model.named_parameters():
            if id(t) in owned or not t.requires_grad:
                continue
            slot = self.ctx.arena.vector(f'torch.{name}', tuple(t.shape))
            self._residual.append((t, slot))

    def _bind_residual(self):
        arena = self.ctx.arena
        for t, slot in self._residual:
            slot.master.copy_(t.detach().float().reshape(slot.shape))
            t.data = slot.master.view(t.shape)
            t.grad = slot.grad.view(t.shape)
            t.register_post_accumulate_grad_hook(lambda _t, s=slot: arena.mark_ready(s))

    # ------------------------------------------------------------------ run
    @property
    def arena(self):
        return self.ctx.arena

    def train(self, mode: bool = True):
        self.training = self.ctx.training = mode
        return self

    def eval(self):
        return self.train(False)

    def __call__(self, x, *rest):
        gm = self.train_gm if self.training else self.eval_gm
        # torch ops left in the graph as leaf modules (Dropout, Dropout2d, user modules) are
        # the user model's own objects, shared by both graphs: their mode is set here, on
        # every call, so the eval graph never runs a training-mode dropout
        gm.train(self.training)
        if self.training and self.ctx.wt is not None:
            self.ctx.wt.refresh()          # the weights are fixed until this step's optimizer
        if self.training and getattr(self.ctx, '_salt', None) is not None:
            self.ctx.seed.add_(1)          # fresh dropout masks for this step
        with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.device.type == 'cuda'):
            return gm(x, *rest)

    def logits(self, x):
        return self(x)

    def param_sets(self):
        return list(self._params.values())

    def _units(self):
        """BatchNorm parameter sets with running statistics (flat-buffer broadcast)."""
        return [p for p in self._params.values() if isinstance(p, BNParams) and p.track]

    def export_to_torch(self):
        for p in self._params.values():
            p.export_to_torch()
        return self.torch_model


def lower_or_none(model: nn.Module) -> Optional[str]:
    """None when ``model`` lowers (structural check on CPU, nothing allocated on a GPU),
    else the reason it does not."""
    try:
        for mode in (True, False):
            model.train(mode)
            gm = fx.symbolic_trace(model)
            probe = GenericNet.__new__(GenericNet)
            probe.ctx = NativeContext()
            probe._params = {}
            probe._composite = {}
            _Lowering(probe, gm).run()
        return None
    except NativeUnsupported as e:
        return str(e)
    except Exception as e:
        return f'torch.fx tracing failed ({type(e).__name__})'
    finally:
        model.train(True)


__all__ = ['GenericNet', 'lower_or_none']
