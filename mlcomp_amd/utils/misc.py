"""Small shared helpers: dict flatten/unflatten, smart config merge, grid expansion,
YAML io, seeding, process helpers (behaviour of `mlcomp/utils/misc.py`,
`mlcomp/utils/config.py:27-75`, `mlcomp/contrib/search/grid.py:10-62`,
`mlcomp/utils/io.py`)."""
from __future__ import annotations

import datetime
import os
import random
import sys
import re
import signal
from collections import defaultdict
from glob import glob
from itertools import product
from os.path import join
from typing import Dict, List, Optional, Tuple

import yaml


def now():
    return datetime.datetime.now()


def to_snake(name: str) -> str:
    return re.sub(r'(?<!^)(?=[A-Z])', '_', name).lower()


# ------------------------------------------------------------------ yaml / io
def yaml_load(text: str = None, file: str = None):
    if file is not None:
        with open(file) as f:
            text = f.read()
    return yaml.safe_load(text) if text else {}


def yaml_dump(data) -> str:
    return yaml.safe_dump(data, default_flow_style=False, sort_keys=False)


# ------------------------------------------------------------------ dicts
def dict_flatten(d: dict, sep: str = '/', prefix: str = '') -> dict:
    out = {}
    for k, v in d.items():
        key = f'{prefix}{sep}{k}' if prefix else str(k)
        if isinstance(v, dict) and v:
            out.update(dict_flatten(v, sep, key))
        else:
            out[key] = v
    return out


def dict_unflatten(d: dict, sep: str = '/') -> dict:
    out: dict = {}
    for k, v in d.items():
        parts = k.split(sep)
        cur = out
        for p in parts[:-1]:
            cur = cur.setdefault(p, {})
        cur[parts[-1]] = v
    return out


def merge_dicts_smart(target: dict, source: dict, sep: str = '/') -> dict:
    """Override values of ``target`` with ``source`` where a source key may be any
    *suffix* of a flattened target key (``lr`` matches ``stages/stage1/optimizer_params/lr``).
    A suffix matching several target keys is ambiguous (AssertionError).  Unknown keys
    are attached under the deepest existing parent that matches their prefix."""
    flat = dict_flatten(target, sep)
    mapping: Dict[str, List[str]] = defaultdict(list)
    hooks: Dict[str, str] = {}
    for k in flat:
        parts = k.split(sep)
        for i in range(len(parts) - 1, -1, -1):
            mapping[sep.join(parts[i:])].append(k)
            if 0 < i < len(parts) - 1:
                hooks[sep.join(parts[i:-1])] = sep.join(parts[:i + 1])
    src = {}
    for k, v in source.items():
        if isinstance(v, dict) and v:
            for kk, vv in dict_flatten(v, sep).items():
                src[f'{k}{sep}{kk}'] = vv
        else:
            src[k] = v
    for k, v in src.items():
        if not mapping.get(k):
            parts = k.split(sep)
            hook = None
            for i in range(len(parts) - 1, 0, -1):
                h = sep.join(parts[:i])
                if h in hooks:
                    hook = hooks[h] + sep + sep.join(parts[i:])
                    break
            mapping[k] = [hook or k]
        assert len(mapping[k]) == 1, f'ambiguous mapping for {k}: {mapping[k]}'
        flat[mapping[k][0]] = v
    return dict_unflatten(flat, sep)


def _parse_scalar(v: str):
    try:
        return yaml.safe_load(v)
    except yaml.YAMLError:
        return v


def dict_from_list_str(params: List[str]) -> dict:
    """``['lr:0.1', 'epochs:3']`` -> ``{'lr': 0.1, 'epochs': 3}``."""
    out = {}
    for p in params or []:
        k, v = p.split(':', 1)
        out[k] = _parse_scalar(v)
    return out


# ------------------------------------------------------------------ grid search
def cell_name(cell: dict) -> str:
    return ' '.join(f'{k}={v}' for k, v in dict_flatten(cell).items())[-300:]


def grid_cells(grid: List) -> List[Tuple[dict, str]]:
    """Cartesian product of grid rows.  Row forms: ``{key: [v1, v2]}``,
    ``{key: "a-b"}`` (inclusive int range), ``[{..}, {..}]`` (explicit cells),
    ``{_folder: dir}`` (every YAML in dir is a cell), ``{_file: [a.yml, ..]}``."""
    rows = []
    for i, row in enumerate(grid or []):
        if isinstance(row, list):
            if not row:
                raise ValueError(f'Empty list at grid row {i}')
            if not all(isinstance(c, dict) for c in row):
                raise ValueError('grid list entries must be dicts')
            rows.append(list(row))
        elif isinstance(row, dict):
            if len(row) != 1:
                raise ValueError('grid dict row must contain exactly one key')
            key, val = next(iter(row.items()))
            cells = []
            if isinstance(val, str):
                if key == '_folder':
                    cells = [yaml_load(file=f) for f in sorted(glob(join(val, '*.yml')))]
                elif re.fullmatch(r'-?\d+\s*-\s*-?\d+', val):
                    a, b = map(int, re.split(r'(?<=\d)\s*-\s*', val, maxsplit=1))
                    cells = [{key: p} for p in range(a, b + 1)]
                else:
                    raise ValueError(f'bad grid value {val!r} for {key}')
            elif isinstance(val, list):
                cells = [yaml_load(file=v) if key == '_file' else {key: v} for v in val]
            else:
                raise ValueError('grid dict value must be a list or str')
            rows.append(cells)
        else:
            raise ValueError(f'Unknown grid row type {type(row)}')
    out = []
    for combo in product(*rows):
        d = {}
        for c in combo:
            d.update(c)
        out.append((d, cell_name(d)))
    return out


# ------------------------------------------------------------------ misc
def set_global_seed(seed: int):
    random.seed(seed)
    try:
        import numpy as np
        np.random.seed(seed)
    except ImportError:
        pass
    torch = sys.modules.get('torch')   # seeded if loaded; importing it costs a task ~3 s
    if torch is not None:
        torch.manual_seed(seed)


def parse_gpu_range(gpu) -> Tuple[int, int]:
    """``2`` -> (2, 2); ``"2-4"`` -> (2, 4)."""
    if isinstance(gpu, str) and '-' in gpu:
        a, b = gpu.split('-')
        return int(a), int(b)
    g = int(gpu or 0)
    return g, g


def kill_child_processes(pid: int, sig=signal.SIGKILL) -> List[int]:
    import psutil
    killed = []
    try:
        parent = psutil.Process(pid)
    except psutil.NoSuchProcess:
        return killed
    for ch in parent.children(recursive=True):
        try:
            ch.send_signal(sig)
            killed.append(ch.pid)
        except psutil.NoSuchProcess:
            pass
    return killed


def kill_pid(pid: int, sig=signal.SIGKILL) -> bool:
    try:
        os.kill(pid, sig)
        return True
    except ProcessLookupError:
        return False


def memory_gb() -> float:
    import psutil
    return psutil.virtual_memory().total / 2 ** 30


def disk_usage(path='/') -> Tuple[float, float]:
    import shutil
    d = shutil.disk_usage(path)
    return d.used / 2 ** 30, d.total / 2 ** 30


def default_network_interface() -> Optional[str]:
    """Interface of the default IPv4 route (``/proc/net/route``), e.g. for
    NCCL_SOCKET_IFNAME (RCCL reads the same variable)."""
    try:
        with open('/proc/net/route') as f:
            for line in f.readlines()[1:]:
                parts = line.split()
                if len(parts) > 2 and parts[1] == '00000000':
                    return parts[0]
    except OSError:
        pass
    return None


__all__ = ['default_network_interface', 'now', 'to_snake', 'yaml_load', 'yaml_dump', 'dict_flatten', 'dict_unflatten',
           'merge_dicts_smart', 'dict_from_list_str', 'grid_cells', 'cell_name', 'set_global_seed',
           'parse_gpu_range', 'kill_child_processes', 'kill_pid', 'memory_gb', 'disk_usage']
