"""The native input pipeline on CPU (`mlcomp_amd/train/records.py`, `csrc/runtime/records.cpp`):
record-file round trip, deterministic + thread-count-independent batches, epoch reshuffle,
rank sharding, the eval centre crop, the sanitizer self-tests of the C++ loader, and a
config-driven training run reading record files."""
import os
import subprocess

import numpy as np
import pytest
import torch

from mlcomp_amd.train.records import RecordFile, RecordLoader, augment_reference, write_records


@pytest.fixture
def rec(tmp_path):
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (60, 20, 24, 3), dtype=np.uint8)
    labs = list(range(100, 160))
    path = str(tmp_path / 'train.mlrec')
    assert write_records(path, imgs, labs) == 60
    return path, imgs, labs


def _all(loader):
    return [(b['features'].clone(), b['targets'].clone()) for b in loader]


def test_record_file_round_trip(rec):
    path, imgs, labs = rec
    f = RecordFile(path)
    assert len(f) == 60 and f.shape == (20, 24, 3)
    for i in (0, 17, 59):
        assert np.array_equal(f.image(i), imgs[i]) and f.label(i) == labs[i]
    with open(path, 'r+b') as fh:       # corrupt the magic: both readers refuse the file
        fh.write(b'XXXX')
    with pytest.raises(ValueError):
        RecordFile(path)
    with pytest.raises(ValueError):
        RecordLoader(path, 4, out_size=16, device='cpu')


def test_loader_is_deterministic_and_reshuffles(rec):
    path, imgs, labs = rec
    a = RecordLoader(path, 8, out_size=16, threads=1, device='cpu', seed=3)
    b = RecordLoader(path, 8, out_size=16, threads=6, device='cpu', seed=3, chunk=3)
    ea, eb = _all(a), _all(b)
    assert len(ea) == len(a) == 7                       # drop_last for training
    for (xa, ya), (xb, yb) in zip(ea, eb):
        assert torch.equal(xa, xb) and torch.equal(ya, yb)
    assert xa.shape == (8, 11, 11, 16) and xa.dtype == torch.bfloat16
    e2 = _all(a)                                          # next epoch: new order and crops
    assert not all(torch.equal(p[1], q[1]) for p, q in zip(ea, e2))
    a.set_epoch(0)
    e0 = _all(a)
    assert all(torch.equal(p[1], q[1]) and torch.equal(p[0], q[0]) for p, q in zip(ea, e0))
    seen = torch.cat([y for _, y in ea]).tolist()
    assert len(set(seen)) == len(seen) and set(seen) <= set(labs)


def test_loader_shards_ranks(rec):
    path, _, labs = rec
    got = []
    for r in range(3):
        L = RecordLoader(path, 5, out_size=16, device='cpu', rank=r, world_size=3, layout='nchw', seed=1)
        assert len(L) == 4
        got += torch.cat([y for _, y in _all(L)]).tolist()
    assert sorted(got) == sorted(labs)                  # the 3 ranks partition the epoch


def test_eval_centre_crop_matches_numpy(rec):
    path, imgs, labs = rec
    L = RecordLoader(path, 7, out_size=16, train=False, layout='nchw', device='cpu', mean=(0, 0, 0),
                     std=(1 / 255,) * 3)
    batches = _all(L)
    assert len(L) == len(batches) == 9                   # no drop_last: a short last batch
    x, y = batches[0]
    assert y.tolist() == labs[:7]
    ref = torch.from_numpy(imgs[:7, 2:18, 4:20]).permute(0, 3, 1, 2).float()
    assert torch.equal(x, ref)
    # the wrap-around rows of the last batch are dropped: every sample counted exactly once
    assert [b[1].shape[0] for b in batches] == [7] * 8 + [4]
    assert torch.cat([b[1] for b in batches]).tolist() == labs


def test_new_epoch_closes_live_iterator(rec):
    path, _, labs = rec
    L = RecordLoader(path, 8, out_size=16, device='cpu', train=False, layout='nchw')
    it = iter(L)
    next(it)                                   # a slot is in use by this iterator
    full = _all(L)                             # a second epoch starts while `it` is alive
    assert torch.cat([y for _, y in full]).tolist() == labs
    with pytest.raises(StopIteration):         # the first iterator was closed
        next(it)


def test_augment_reference_layouts():
    torch.manual_seed(0)
    img = torch.randint(0, 256, (2, 10, 12, 3), dtype=torch.uint8)
    par = torch.tensor([[1, 2, 6, 8, 1], [0, 0, 10, 12, 0]], dtype=torch.int32)
    ms = [10.0, 20.0, 30.0, 0.0, 0.5, 0.25, 0.125, 0.0]
    nchw = augment_reference(img, par, 8, 8, ms, 'nchw')
    nhwc = augment_reference(img, par, 8, 8, ms, 'nhwc8')
    s2d = augment_reference(img, par, 8, 8, ms, 's2d')
    assert nchw.shape == (2, 3, 8, 8) and nhwc.shape == (2, 8, 8, 8) and s2d.shape == (2, 7, 7, 16)
    assert torch.allclose(nhwc[..., :3].float(), nchw.permute(0, 2, 3, 1), rtol=1e-2, atol=1e-2)
    # sample 1 is the whole image resized 10x12 -> 8x8; flip of sample 0 mirrors the columns
    flipped = augment_reference(img[:1], par[:1].clone().index_fill_(1, torch.tensor([4]), 0), 8, 8, ms, 'nchw')
    assert torch.allclose(flipped.flip(-1), nchw[:1])


@pytest.mark.parametrize('san', ['tsan', 'asan'])
def test_loader_sanitizer_selftest(san, tmp_path):
    """ThreadSanitizer / AddressSanitizer+UBSan builds of the C++ loader under a consumer
    that changes thread counts, slows down and abandons epochs half way."""
    from mlcomp_amd.build import build_runtime_selftest
    binary = build_runtime_selftest(san)
    r = subprocess.run([binary, str(tmp_path)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, TSAN_OPTIONS='halt_on_error=1', ASAN_OPTIONS='detect_leaks=1'))
    assert r.returncode == 0, r.stderr[-4000:]
    assert 'records selftest ok' in r.stdout
    assert 'WARNING: ThreadSanitizer' not in r.stderr and 'ERROR: AddressSanitizer' not in r.stderr


def test_runner_trains_from_record_files(tmp_path):
    from mlcomp_amd.train.experiment import ConfigExperiment
    from mlcomp_amd.train.runner import Runner
    rng = np.random.default_rng(1)
    write_records(str(tmp_path / 'tr.mlrec'), rng.integers(0, 256, (48, 20, 20, 3), dtype=np.uint8),
                  rng.integers(0, 4, 48).tolist())
    write_records(str(tmp_path / 'va.mlrec'), rng.integers(0, 256, (16, 20, 20, 3), dtype=np.uint8),
                  rng.integers(0, 4, 16).tolist())
    cfg = {'model_params': {'model': 'SimpleCNN', 'num_classes': 4, 'width': 8},
           'args': {'logdir': str(tmp_path / 'log'), 'engine': 'torch'},
           'stages': {'data_params': {'dataset': 'records', 'path': str(tmp_path / 'tr.mlrec'),
                                      'valid_path': str(tmp_path / 'va.mlrec'), 'image_size': 16,
                                      'batch_size': 8, 'num_workers': 2},
                      'state_params': {'num_epochs': 2},
                      'criterion_params': {'criterion': 'CrossEntropyLoss'},
                      'optimizer_params': {'optimizer': 'Adam', 'lr': 0.01},
                      'callbacks_params': {'loss': {'callback': 'CriterionCallback'},
                                           'opt': {'callback': 'OptimizerCallback'},
                                           'acc': {'callback': 'AccuracyCallback'}},
                      'stage1': {}}}
    st = Runner(ConfigExperiment(cfg), device='cpu').run_experiment()
    m = st.epoch_metrics
    assert m['train_loss'] == m['train_loss'] and 'valid_accuracy01' in m


def test_contrib_pack_records_cli(tmp_path):
    from click.testing import CliRunner
    from PIL import Image
    from mlcomp_amd.contrib.__main__ import main
    rng = np.random.default_rng(3)
    for cls in ('cat', 'dog'):
        (tmp_path / 'img' / cls).mkdir(parents=True)
        for i in range(3):
            Image.fromarray(rng.integers(0, 256, (30 + i, 40, 3), dtype=np.uint8)).save(tmp_path / 'img' / cls / f'{i}.png')
    out = str(tmp_path / 'x.mlrec')
    r = CliRunner().invoke(main, ['pack-records', str(tmp_path / 'img'), out, '--size', '24'])
    assert r.exit_code == 0, r.output
    f = RecordFile(out)
    assert len(f) == 6 and f.shape == (24, 24, 3)
    assert [f.label(i) for i in range(6)] == [0, 0, 0, 1, 1, 1]
    assert open(out + '.classes').read().split() == ['cat', 'dog']
