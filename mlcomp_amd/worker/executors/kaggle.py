"""Kaggle executors (`mlcomp/worker/executors/kaggle.py:39-196`): ``Download``
competition files and ``Submit`` a file or a kernel.  The ``kaggle`` client is an
optional dependency (not in this image, and there is no network here): the executors
register and validate their arguments, and fail with a clear message at run time when
the client is missing."""
from __future__ import annotations

import os
import shutil
import time
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
                 **kwargs):
        super().__init__(**kwargs)
        assert submit_type in ('file', 'kernel'), submit_type
        self.competition, self.submit_type, self.kernel_suffix = competition, submit_type, kernel_suffix
        self.message, self.wait_seconds, self.max_size = message, wait_seconds, max_size
        self.datasets, self.folders, self.files = list(datasets), list(folders), list(files)
        if not file and model_name:
            file = f'data/submissions/{model_name}_{suffix}.csv'
        self.file = file

    def file_submit(self):
        _api().competition_submit(self.file, message=self.message, competition=self.competition)

    def kernel_submit(self):
        api = _api()
        folder = os.path.expanduser(f'~/.kaggle/competitions/{self.competition}')
        shutil.rmtree(folder, ignore_errors=True)
        os.makedirs(folder, exist_ok=True)
        for f in self.folders:
            shutil.make_archive(os.path.join(folder, os.path.basename(f.rstrip('/'))), 'zip', f)
        for f in self.files:
            shutil.copy(f, folder)
        api.dataset_create_version(folder, self.message or 'mlcomp submit', dir_mode='zip')
        deadline = time.time() + self.wait_seconds
        while time.time() < deadline:
            st = api.kernel_status(f'{self.competition}-{self.kernel_suffix}')
            if getattr(st, 'status', '') in ('complete', 'error'):
                break
            time.sleep(20)

    def work(self):
        (self.file_submit if self.submit_type == 'file' else self.kernel_submit)()
        return {}


__all__ = ['Download', 'Submit']
