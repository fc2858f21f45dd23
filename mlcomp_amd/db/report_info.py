"""Report layout model: parse + validate layout YAML and resolve ``extend``
inheritance (behaviour of `mlcomp/db/report_info/info.py:12-132`).

A layout has ``metric`` ({name, minimize}; default loss/minimize), ``items`` (named
data items: series / img_classify / img_segment / precision_recall / f1) and
``layout`` (a tree of UI components: root, panel, blank, series, table, img_classify,
img, img_segment).  ``extend: <name>`` merges a parent's items/layout first.
"""
from __future__ import annotations

from copy import deepcopy
from dataclasses import dataclass, field
from typing import Dict, List, Optional

# component type -> {field: required}
COMPONENT_FIELDS = {
    'root': {'items': False},
    'panel': {'title': True, 'parent_cols': False, 'cols': False, 'row_height': False,
              'rows': False, 'items': False, 'expanded': False, 'table': False},
    'blank': {'cols': False, 'rows': False},
    'series': {'multi': False, 'group': False, 'source': True, 'cols': False, 'rows': False},
    'table': {'source': True, 'cols': False, 'rows': False},
    'img_classify': {'source': True, 'attrs': False, 'cols': False, 'rows': False},
    'img_segment': {'source': True, 'attrs': False, 'cols': False, 'rows': False,
                    'max_width': False, 'max_height': False},
    'img': {'source': True, 'cols': False, 'rows': False},
}

ITEM_TYPES = ('series', 'img_classify', 'img_segment', 'precision_recall', 'f1')


@dataclass
class Metric:
    name: str = 'loss'
    minimize: bool = True

    def better(self, new: float, old: Optional[float]) -> bool:
        if old is None:
            return True
        return new < old if self.minimize else new > old


@dataclass
class Item:
    name: str
    type: str
    options: dict = field(default_factory=dict)


class LayoutError(ValueError):
    pass


def check_component(c: dict, path='layout'):
    t = c.get('type')
    if t not in COMPONENT_FIELDS:
        raise LayoutError(f'{path}: unknown component type {t!r}')
    spec = COMPONENT_FIELDS[t]
    for f, req in spec.items():
        if req and f not in c:
            raise LayoutError(f'{path}: type {t} must contain field {f!r}')
    extra = set(c) - set(spec) - {'type'}
    if extra:
        raise LayoutError(f'{path}: unknown fields {sorted(extra)} for type {t}')
    for i, ch in enumerate(c.get('items', []) or []):
        check_component(ch, f'{path}.{t}[{i}]')


class ReportLayoutInfo:
    def __init__(self, data: dict):
        data = dict(data or {})
        self.data = data
        m = data.get('metric') or {'name': 'loss', 'minimize': True}
        self.metric = Metric(m.get('name', 'loss'), bool(m.get('minimize', True)))
        self.items: List[Item] = []
        for name, v in (data.get('items') or {}).items():
            t = v.get('type')
            if t not in ITEM_TYPES:
                raise LayoutError(f'item {name}: unknown type {t!r}')
            self.items.append(Item(name, t, {k: x for k, x in v.items() if k != 'type'}))
        self.layout = {'type': 'root', 'items': data.get('layout') or []}
        check_component(self.layout)

    def by_type(self, t: str) -> List[Item]:
        return [i for i in self.items if i.type == t]

    @property
    def series(self):
        return self.by_type('series')

    @property
    def img_classify(self):
        return self.by_type('img_classify')

    @property
    def img_segment(self):
        return self.by_type('img_segment')

    @property
    def precision_recall(self):
        return self.by_type('precision_recall')

    def has_classification(self) -> bool:
        return bool(self.precision_recall)

    @staticmethod
    def union(name: str, layouts: Dict[str, dict], _seen=()) -> dict:
        if name not in layouts:
            raise LayoutError(f'layout {name!r} is not in the collection')
        if name in _seen:
            raise LayoutError(f'cyclic extend through {name!r}')
        lay = deepcopy(layouts[name])
        r: dict = {}
        if lay.get('extend'):
            r = ReportLayoutInfo.union(lay['extend'], layouts, tuple(_seen) + (name,))
        if 'metric' in lay:
            r['metric'] = lay['metric']
        if 'items' in lay:
            r.setdefault('items', {}).update(lay['items'])
        if 'layout' in lay:
            r['layout'] = r.get('layout', []) + lay['layout']
        return r


def union_layouts(raw: Dict[str, dict]) -> Dict[str, dict]:
    return {n: ReportLayoutInfo.union(n, raw) for n in raw}


__all__ = ['ReportLayoutInfo', 'Metric', 'Item', 'LayoutError', 'union_layouts', 'check_component']
