"""Kaggle kernel submission (`mlcomp/worker/executors/kaggle.py:112-186`) against a fake
client (no network and no kaggle package here): dataset-metadata.json, the zipped
folders/files, dataset create-vs-version, kernel-metadata.json, kernels_push, status poll."""
import json
import os
import zipfile
from types import SimpleNamespace

import pytest

from mlcomp_amd.worker.executors import kaggle as K


class FakeApi:
    def __init__(self, existing=()):
        self.calls = []
        self.existing = list(existing)
        self.pushed = None

    def read_config_file(self):
        return {'username': 'alice'}

    def dataset_list(self, user):
        return [SimpleNamespace(ref=r) for r in self.existing]

    def dataset_create_new(self, folder):
        self.calls.append(('new', json.load(open(os.path.join(folder, 'dataset-metadata.json')))))
        with zipfile.ZipFile(os.path.join(folder, 'dataset.zip')) as z:
            self.zipped = sorted(z.namelist())

    def dataset_create_version(self, folder, message, **kw):
        self.calls.append(('version', message))
        return SimpleNamespace(status='ok')

    def kernels_push(self, folder):
        self.pushed = json.load(open(os.path.join(folder, 'kernel-metadata.json')))
        assert os.path.exists(os.path.join(folder, self.pushed['code_file']))
        self.calls.append(('push', self.pushed['id']))

    def kernels_status(self, ref):
        self.calls.append(('status', ref))
        return SimpleNamespace(status='complete')


@pytest.fixture
def proj(tmp_path, monkeypatch):
    monkeypatch.setenv('HOME', str(tmp_path / 'home'))
    monkeypatch.chdir(tmp_path)
    (tmp_path / 'models').mkdir()
    (tmp_path / 'models' / 'best.pth').write_bytes(b'w' * 100)
    (tmp_path / 'src').mkdir()
    (tmp_path / 'src' / 'infer.py').write_text('print(1)\n')
    (tmp_path / 'predict.ipynb').write_text('{"cells": []}')
    return tmp_path


def test_kernel_submit_creates_dataset_and_pushes(proj, monkeypatch):
    api = FakeApi()
    monkeypatch.setattr(K, '_api', lambda: api)
    s = K.Submit(competition='digit-recognizer', submit_type='kernel', folders=['models'], files=['src/infer.py'],
                 datasets=['bob/extra'], dataset_wait=0, poll_seconds=0, wait_seconds=5)
    res = s.work()
    kind, meta = api.calls[0]
    assert kind == 'new' and meta['id'] == 'alice/digit-recognizer-api-dataset'
    assert meta['competition'] == 'digit-recognizer' and meta['licenses'] == [{'name': 'CC0-1.0'}]
    assert api.zipped == ['infer.py', 'models/best.pth']
    k = api.pushed
    assert k['id'] == 'alice/digit-recognizer-api' and k['code_file'] == 'predict.ipynb'
    assert k['dataset_sources'] == ['alice/digit-recognizer-api-dataset', 'bob/extra']
    assert k['competition_sources'] == ['digit-recognizer'] and k['kernel_type'] == 'notebook'
    assert ('status', 'alice/digit-recognizer-api') in api.calls
    assert res == {'kernel': 'alice/digit-recognizer-api', 'status': 'complete'}


def test_kernel_submit_versions_an_existing_dataset_and_checks_size(proj, monkeypatch):
    api = FakeApi(existing=['alice/digit-recognizer-api-dataset'])
    monkeypatch.setattr(K, '_api', lambda: api)
    s = K.Submit(competition='digit-recognizer', submit_type='kernel', folders=['models'], message='v2',
                 dataset_wait=0, poll_seconds=0, wait_seconds=5)
    s.work()
    assert api.calls[0] == ('version', 'v2')
    big = K.Submit(competition='digit-recognizer', submit_type='kernel', folders=['models'], max_size=1e-9,
                   dataset_wait=0)
    with pytest.raises(ValueError, match='max_size'):
        big.work()


def test_missing_client_fails_clearly(monkeypatch):
    import builtins
    real = builtins.__import__

    def fake(name, *a, **k):
        if name == 'kaggle':
            raise ImportError('no kaggle')
        return real(name, *a, **k)
    monkeypatch.setattr(builtins, '__import__', fake)
    with pytest.raises(RuntimeError, match='kaggle client'):
        K._api()
