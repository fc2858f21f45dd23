"""File helpers (`mlcomp/utils/io.py:15-80`): YAML load/dump re-exported, zip a folder,
read a text file safely."""
from __future__ import annotations

import os
import zipfile

from .misc import yaml_dump, yaml_load  # noqa: F401


def zip_folder(folder: str, dst: str) -> str:
    with zipfile.ZipFile(dst, 'w', zipfile.ZIP_DEFLATED) as z:
        for root, _, files in os.walk(folder):
            for f in files:
                p = os.path.join(root, f)
                z.write(p, os.path.relpath(p, folder))
    return dst


def read_text(path: str, default: str = '') -> str:
    try:
        with open(path, encoding='utf-8') as f:
            return f.read()
    except (OSError, UnicodeDecodeError):
        return default


__all__ = ['zip_folder', 'read_text', 'yaml_load', 'yaml_dump']
