"""Transformer blocks on the generic native engine, on the GPU: the lowered sites run the
HIP kernels (dense MFMA GEMMs with bias / GELU epilogues, flash attention, LayerNorm) and
are compared with the fp32 PyTorch model (forward and every parameter gradient); the
``transformer-tiny`` / ``vit-ti16`` steps train with graph capture."""
import math

import pytest
import torch

from test_gtransformer_cpu import _EncClassifier, _MHANet, _ViT, _cos, _ids, _pair, _rel, _slot_pairs

pytestmark = pytest.mark.gpu


def _gpu_check(make, x_fn, cos_min=0.98, rel_max=3e-2):
    from mlcomp_amd.models.native_generic import GenericNet
    m, ref = _pair(make)
    net = GenericNet(m, 'cuda')
    ref = ref.cuda().float()
    x = x_fn().cuda()
    out = net(x)
    want = ref(x)
    assert _rel(out, want) < rel_max, _rel(out, want)
    g = torch.randn_like(want)
    (out.float() * g).sum().backward()
    (want * g).sum().backward()
    torch.cuda.synchronize()
    refp = dict(ref.named_parameters())
    worst = 1.0
    for name, got, _ in _slot_pairs(net, m):
        c = _cos(got, refp[name].grad.reshape(got.shape))
        worst = min(worst, c)
        assert c > cos_min, (name, c)
    return worst


def test_encoder_post_norm_gelu_padding_on_kernels():
    _gpu_check(_EncClassifier, _ids)


def test_encoder_pre_norm_relu_sequence_first_on_kernels():
    _gpu_check(lambda: _EncClassifier(norm_first=True, act='relu', batch_first=False), _ids)


def test_mha_module_on_kernels():
    _gpu_check(_MHANet, lambda: torch.randn(20, 4, 16))


def test_vit_style_on_kernels():
    _gpu_check(_ViT, lambda: torch.randn(2, 3, 64, 64))


@pytest.mark.parametrize('name,shape', [('transformer-tiny', 32), ('vit-ti16', 64)])
def test_generic_transformer_steps_train_with_graphs(name, shape):
    from mlcomp_amd.ops import _lib
    from mlcomp_amd.train.generic import build_generic_step
    step = build_generic_step(name, batch=8, seq_len=shape, image_size=shape, device=torch.device('cuda'),
                              num_classes=4, lr=1e-3)
    losses = []
    for _ in range(8):
        step()
        losses.append(step.last_loss())
    assert step.graph is not None, step.capture_error
    assert all(math.isfinite(v) for v in losses), losses
    assert _lib.load() is not None
