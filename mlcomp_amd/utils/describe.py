"""Notebook dashboard for a DAG (`mlcomp/utils/describe.py:22-385`): task table, the DAG
graph (topological layers, coloured by status), the last log lines, computer usage history
and metric series, refreshed until every task has finished.

    from mlcomp_amd.utils.describe import describe
    describe(dag_id, metrics=['loss', 'accuracy01'])
"""
from __future__ import annotations

import datetime
import json
import time
from collections import defaultdict
from typing import List, Optional

STATUS_COLORS = {0: '#bdbdbd', 1: '#90caf9', 2: '#1e88e5', 3: '#e53935', 4: '#fb8c00', 5: '#fdd835',
                 6: '#43a047'}
STATUS_NAMES = ['not_ran', 'queued', 'in_progress', 'failed', 'stopped', 'skipped', 'success']


def _session():
    from mlcomp_amd.db.core import Session
    return Session.create_session(key='describe')


def task_table(dag_id: int):
    from mlcomp_amd.db.providers import TaskProvider
    rows = []
    for t in TaskProvider(_session()).by_dag(dag_id):
        dur = (t.finished or datetime.datetime.now()) - t.started if t.started else None
        rows.append({'id': t.id, 'name': t.name, 'status': STATUS_NAMES[t.status], 'computer': t.computer_assigned,
                     'gpu': t.gpu_assigned, 'duration': str(dur).split('.')[0] if dur else '', 'score': t.score,
                     'loss': t.loss, 'step': t.current_step,
                     'progress': f'{t.batch_index}/{t.batch_total}' if t.batch_total else ''})
    return rows


def graph_layers(dag_id: int):
    """Tasks grouped into topological layers (dependencies first)."""
    from mlcomp_amd.db.providers import TaskProvider
    tp = TaskProvider(_session())
    tasks = {t.id: t for t in tp.by_dag(dag_id)}
    deps = defaultdict(set)
    for d in tp.get_dependencies(dag_id):
        deps[d.task_id].add(d.depend_id)
    level = {}

    def lv(i):
        if i not in level:
            level[i] = 1 + max((lv(d) for d in deps[i] if d in tasks), default=-1)
        return level[i]
    for i in tasks:
        lv(i)
    layers = defaultdict(list)
    for i, l in level.items():
        layers[l].append(tasks[i])
    return [layers[k] for k in sorted(layers)], deps


def draw(dag_id: int, metrics: Optional[List[str]] = None, last_n: int = 8, fig=None):
    import matplotlib
    import matplotlib.pyplot as plt
    from mlcomp_amd.db.models import ComputerUsage, ReportSeries
    from mlcomp_amd.db.providers import LogProvider, TaskProvider
    s = _session()
    metrics = metrics or ['loss']
    fig = fig or plt.figure(figsize=(14, 4 + 3 * ((len(metrics) + 1) // 2)))
    fig.clf()
    gs = fig.add_gridspec(2 + (len(metrics) + 1) // 2, 2)
    # task table
    ax = fig.add_subplot(gs[0, 0])
    ax.axis('off')
    rows = task_table(dag_id)
    if rows:
        cols = ['id', 'name', 'status', 'duration', 'progress', 'score']
        tb = ax.table(cellText=[[str(r[c] if r[c] is not None else '') for c in cols] for r in rows],
                      colLabels=cols, loc='center', cellLoc='left')
        tb.auto_set_font_size(False)
        tb.set_fontsize(8)
    # DAG graph
    ax = fig.add_subplot(gs[0, 1])
    ax.axis('off')
    layers, deps = graph_layers(dag_id)
    pos = {}
    for x, layer in enumerate(layers):
        for y, t in enumerate(layer):
            pos[t.id] = (x, -y + len(layer) / 2)
            ax.scatter(*pos[t.id], s=600, c=STATUS_COLORS.get(t.status, '#999'), zorder=2)
            ax.annotate(t.name, pos[t.id], ha='center', va='center', fontsize=7, zorder=3)
    for i, ds in deps.items():
        for d in ds:
            if i in pos and d in pos:
                ax.annotate('', pos[i], pos[d], arrowprops=dict(arrowstyle='->', color='#555'), zorder=1)
    # last logs
    ax = fig.add_subplot(gs[1, 0])
    ax.axis('off')
    logs = LogProvider(s).last(last_n, dag=dag_id)
    ax.text(0, 1, '\n'.join(f'{l.time:%H:%M:%S} {l.message[:90]}' for l in logs) or 'no logs',
            va='top', family='monospace', fontsize=7)
    # usage history of the computers running the DAG
    ax = fig.add_subplot(gs[1, 1])
    comps = {r['computer'] for r in rows if r['computer']}
    since = datetime.datetime.now() - datetime.timedelta(minutes=30)
    for c in comps:
        us = s.query(ComputerUsage).filter(ComputerUsage.computer == c).filter(ComputerUsage.time >= since).all()
        if us:
            vals = [json.loads(u.usage) for u in us]
            ax.plot([u.time for u in us], [v.get('cpu', 0) for v in vals], label=f'{c} cpu')
            ax.plot([u.time for u in us], [v.get('memory', 0) for v in vals], label=f'{c} mem')
    ax.set_title('usage %', fontsize=8)
    if comps:
        ax.legend(fontsize=6)
    # metric series
    ids = [r['id'] for r in rows]
    for k, m in enumerate(metrics):
        ax = fig.add_subplot(gs[2 + k // 2, k % 2])
        q = s.query(ReportSeries).filter(ReportSeries.task.in_(ids)).filter(ReportSeries.name == m)
        by = defaultdict(list)
        for r in q.order_by(ReportSeries.epoch):
            by[(r.task, r.part)].append((r.epoch, r.value))
        for (t, part), pts in by.items():
            ax.plot([p[0] for p in pts], [p[1] for p in pts], marker='o', label=f'{t} {part}')
        ax.set_title(m, fontsize=8)
        if by:
            ax.legend(fontsize=6)
    fig.tight_layout()
    return fig


def describe(dag_id: int, metrics: Optional[List[str]] = None, last_n: int = 8, wait: bool = True,
             interval: float = 5.0, max_time: float = 24 * 3600):
    """Draw (and, in a notebook, keep redrawing) until every task of the DAG finished."""
    import matplotlib.pyplot as plt
    try:
        from IPython.display import clear_output, display
    except ImportError:       # plain python: draw once
        clear_output = display = None
    fig = None
    t0 = time.time()
    while True:
        fig = draw(dag_id, metrics, last_n, fig)
        if display is not None:
            clear_output(wait=True)
            display(fig)
        done = all(r['status'] in ('failed', 'stopped', 'skipped', 'success') for r in task_table(dag_id))
        if not wait or done or display is None or time.time() - t0 > max_time:
            break
        time.sleep(interval)
    plt.close(fig)
    return fig


__all__ = ['describe', 'draw', 'task_table', 'graph_layers']
