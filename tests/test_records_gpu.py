"""The GPU half of the native input pipeline: ``mlc_augment`` (csrc/kernels/augment.hip)
against its PyTorch twin for every output layout, and the CUDA RecordLoader end to end
(pinned slots, copy stream, augment kernel) against the CPU loader on the same stream."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('layout', ['s2d', 'nhwc8', 'nchw'])
def test_augment_kernel_matches_reference(layout):
    from mlcomp_amd.ops import _lib
    from mlcomp_amd.train.records import LAYOUTS, augment_reference
    torch.manual_seed(0)
    B, H, W, oh = 5, 40, 36, 24
    img = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8)
    par = torch.tensor([[0, 0, 40, 36, 0], [3, 5, 20, 17, 1], [10, 2, 30, 30, 0], [0, 20, 9, 16, 1],
                        [39, 35, 1, 1, 0]], dtype=torch.int32)
    ms = [123.7, 116.3, 103.5, 0.0, 1 / 58.4, 1 / 57.1, 1 / 57.4, 0.0]
    ref = augment_reference(img, par, oh, oh, ms, layout)
    dimg, dpar = img.cuda(), par.cuda()
    dms = torch.tensor(ms, device='cuda')
    out = torch.empty(ref.shape, dtype=ref.dtype, device='cuda')
    _lib.call('mlc_augment', _lib.ptr(dimg), _lib.ptr(dpar), _lib.ptr(dms), _lib.ptr(out), B, H, W, 3, oh, oh,
              LAYOUTS[layout], _lib.stream())
    torch.cuda.synchronize()
    tol = 2e-2 if ref.dtype == torch.bfloat16 else 1e-4
    assert torch.allclose(out.cpu().float(), ref.float(), atol=tol, rtol=tol)


def test_cuda_record_loader_matches_cpu(tmp_path):
    from mlcomp_amd.train.records import RecordLoader, write_records
    rng = np.random.default_rng(2)
    path = str(tmp_path / 'r.mlrec')
    write_records(path, rng.integers(0, 256, (40, 32, 32, 3), dtype=np.uint8), list(range(40)))
    g = RecordLoader(path, 8, out_size=24, threads=4, device='cuda', seed=5)
    c = RecordLoader(path, 8, out_size=24, threads=2, device='cpu', seed=5)
    for _ in range(2):   # two epochs
        gb, cb = list(g), list(c)
        assert len(gb) == len(cb) == 5
        for a, b in zip(gb, cb):
            assert a['features'].is_cuda and a['features'].shape == (8, 15, 15, 16)
            assert torch.equal(a['targets'].cpu(), b['targets'])
            assert torch.allclose(a['features'].cpu().float(), b['features'].float(), atol=2e-2, rtol=2e-2)
