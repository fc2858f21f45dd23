"""Kaggle executors (`mlcomp/worker/executors/kaggle.py:39-196`): ``Download``
competition files and ``Submit`` a file or a kernel.  The ``kaggle`` client is an
optional dependency (not in this image, and there is no network here): the executors
register and validate their arguments, and fail with a clear message at run time when
the client is missing."""
from __future__ import annotations

import json
import os
import shutil
import time
import zipfile
from typing import List

from mlcomp_amd import config
from .base import Executor


def _api():
    try:
        from kaggle import api  # noqa: F401
    except Exception as e:  # ImportError or credential errors raised at import
        raise RuntimeError(f'the kaggle client is not available: {e}')
    return api


@Executor.register
class Download(Executor):
    def __init__(self, output: str, competition: str = None, link: str = None, type: str = 'kaggle', **kwargs):
        super().__init__(**kwargs)
        if type == 'kaggle' and not competition:
            raise ValueError('Competition is required for Kaggle')
        self.output, self.competition, self.link, self.type = output, competition, link, type

    @classmethod
    def _from_config(cls, executor, config_, additional_info):
        project = (config_.get('info') or {}).get('project', '')
        out = os.path.join(config.get().DATA_FOLDER, project, executor.get('output', '.'))
        return cls(output=out, competition=executor.get('competition'), link=executor.get('link'))

    def work(self):
        os.makedirs(self.output, exist_ok=True)
        _api().competition_download_files(self.competition, self.output)
        for f in os.listdir(self.output):
            if f.endswith('.zip'):
                shutil.unpack_archive(os.path.join(self.output, f), self.output)
        return {}


@Executor.register
class Submit(Executor):
    def __init__(self, competition: str, submit_type: str = 'file', kernel_suffix: str = 'api', message: str = '',
                 wait_seconds: int = 60 * 20, file: str = None, max_size: int = None, datasets: List[str] = (),
                 folders: List[str] = (), files: List[str] = (), model_name: str = None, suffix: str = '',
                 notebook: str = 'predict.ipynb', dataset_wait: int = 30, poll_seconds: int = 20, **kwargs):
        super().__init__(**kwargs)
        assert submit_type in ('file', 'kernel'), submit_type
        self.competition, self.submit_type, self.kernel_suffix = competition, submit_type, kernel_suffix
        self.message, self.wait_seconds, self.max_size = message, wait_seconds, max_size
        self.datasets, self.folders, self.files = list(datasets), list(folders), list(files)
        if not file and model_name:
            file = f'data/submissions/{model_name}_{suffix}.csv'
        self.file = file
        self.notebook, self.dataset_wait, self.poll_seconds = notebook, dataset_wait, poll_seconds

    def file_submit(self):
        _api().competition_submit(self.file, message=self.message, competition=self.competition)

    # ------------------------------------------------------------------ kernel submit
    def dataset_meta(self, username: str) -> dict:
        """`dataset-metadata.json` of the private dataset that carries the code / weights."""
        return {'competition': self.competition, 'id': f'{username}/{self.competition}-{self.kernel_suffix}-dataset',
                'licenses': [{'name': 'CC0-1.0'}], 'title': f'{self.competition} {self.kernel_suffix} (mlcomp)'}

    def kernel_meta(self, username: str, dataset_id: str) -> dict:
        """`kernel-metadata.json` of the notebook that runs inference over the dataset."""
        slug = f'{self.competition}-{self.kernel_suffix}'
        return {'id': f'{username}/{slug}', 'title': slug, 'code_file': os.path.basename(self.notebook),
                'language': 'python', 'kernel_type': 'notebook', 'is_private': 'true',
                'enable_gpu': 'true', 'enable_internet': 'false',
                'dataset_sources': [dataset_id] + list(self.datasets),
                'competition_sources': [self.competition], 'kernel_sources': []}

    def _size_gb(self) -> float:
        total = 0
        for f in self.folders:
            for root, _, names in os.walk(f):
                total += sum(os.path.getsize(os.path.join(root, n)) for n in names)
        total += sum(os.path.getsize(f) for f in self.files)
        return total / 2 ** 30

    def kernel_submit(self):
        """Zip the folders / files into a private dataset (created, or a new version),
        then push a notebook kernel that reads it (`mlcomp/worker/executors/kaggle.py:112-186`)
        and wait for the kernel run to finish."""
        api = _api()
        folder = os.path.expanduser(f'~/.kaggle/competitions/{self.competition}')
        shutil.rmtree(folder, ignore_errors=True)
        os.makedirs(folder, exist_ok=True)
        size = self._size_gb()
        if self.max_size and size >= self.max_size:
            raise ValueError(f'max_size = {self.max_size} GB, the submission is {size:.2f} GB')
        username = api.read_config_file()['username']
        meta = self.dataset_meta(username)
        with open(os.path.join(folder, 'dataset-metadata.json'), 'w') as f:
            json.dump(meta, f)
        self.info('kernel submit: zipping folders')
        with zipfile.ZipFile(os.path.join(folder, 'dataset.zip'), 'w', zipfile.ZIP_DEFLATED) as z:
            for d in self.folders:
                base = os.path.dirname(os.path.abspath(d).rstrip('/'))
                for root, _, names in os.walk(d):
                    for n in names:
                        p = os.path.join(root, n)
                        z.write(p, os.path.relpath(os.path.abspath(p), base))
            for p in self.files:
                z.write(p, os.path.basename(p))
        self.info('kernel submit: uploading the dataset')
        if not any(getattr(d, 'ref', None) == meta['id'] for d in api.dataset_list(user=username)):
            api.dataset_create_new(folder)
        else:
            res = api.dataset_create_version(folder, self.message or 'mlcomp submit')
            if getattr(res, 'status', '') == 'error':
                raise RuntimeError(f'dataset_create_version: {getattr(res, "error", res)}')
        time.sleep(self.dataset_wait)     # the new dataset version is processed server-side
        shutil.copy(self.notebook, os.path.join(folder, os.path.basename(self.notebook)))
        kmeta = self.kernel_meta(username, meta['id'])
        with open(os.path.join(folder, 'kernel-metadata.json'), 'w') as f:
            json.dump(kmeta, f)
        api.kernels_push(folder)
        self.info(f'kernel pushed: https://www.kaggle.com/{kmeta["id"]}')
        deadline = time.time() + self.wait_seconds
        status = None
        while time.time() < deadline:
            status = getattr(api.kernels_status(kmeta['id']), 'status', None)
            if status in ('complete', 'error', 'cancelAcknowledged'):
                break
            time.sleep(self.poll_seconds)
        if status == 'error':
            raise RuntimeError(f'kernel {kmeta["id"]} failed')
        return {'kernel': kmeta['id'], 'status': status}

    def work(self):
        if self.submit_type == 'file':
            self.file_submit()
            return {}
        return self.kernel_submit()


__all__ = ['Download', 'Submit']
