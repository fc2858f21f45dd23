"""Report plots (`mlcomp/utils/plot.py:10-185`): matplotlib figures rendered to JPEG bytes
for ``ReportImg`` rows - the per-class precision/recall/F1 heatmap (layout item ``f1``)
and precision-recall curves (layout item ``precision_recall``)."""
from __future__ import annotations

import io
from typing import List, Optional

import numpy as np


def _plt():
    import matplotlib
    matplotlib.use('Agg')
    import matplotlib.pyplot as plt
    return plt


def figure_to_bytes(fig, fmt: str = 'jpg', dpi: int = 100) -> bytes:
    buf = io.BytesIO()
    fig.savefig(buf, format='jpeg' if fmt == 'jpg' else fmt, dpi=dpi, bbox_inches='tight')
    _plt().close(fig)
    return buf.getvalue()


def classification_report_table(y_true, y_pred, num_classes: int):
    """rows = classes: precision, recall, f1, support."""
    y_true, y_pred = np.asarray(y_true), np.asarray(y_pred)
    out = []
    for c in range(num_classes):
        tp = int(((y_pred == c) & (y_true == c)).sum())
        fp = int(((y_pred == c) & (y_true != c)).sum())
        fn = int(((y_pred != c) & (y_true == c)).sum())
        p = tp / (tp + fp) if tp + fp else 0.0
        r = tp / (tp + fn) if tp + fn else 0.0
        f = 2 * p * r / (p + r) if p + r else 0.0
        out.append((p, r, f, int((y_true == c).sum())))
    return np.array(out)


def plot_classification_report(y_true, y_pred, num_classes: int, class_names: Optional[List[str]] = None) -> bytes:
    plt = _plt()
    t = classification_report_table(y_true, y_pred, num_classes)
    names = class_names or [str(i) for i in range(num_classes)]
    fig, ax = plt.subplots(figsize=(5, 0.4 * num_classes + 1.5))
    im = ax.imshow(t[:, :3], cmap='RdYlGn', vmin=0, vmax=1, aspect='auto')
    ax.set_xticks(range(3), ['precision', 'recall', 'f1'])
    ax.set_yticks(range(num_classes), [f'{n} ({int(s)})' for n, s in zip(names, t[:, 3])])
    for i in range(num_classes):
        for j in range(3):
            ax.text(j, i, f'{t[i, j]:.2f}', ha='center', va='center', fontsize=8)
    fig.colorbar(im, ax=ax)
    return figure_to_bytes(fig)


def precision_recall_curve(y_true_bin, scores):
    order = np.argsort(-np.asarray(scores))
    y = np.asarray(y_true_bin)[order]
    tp = np.cumsum(y)
    fp = np.cumsum(1 - y)
    precision = tp / np.maximum(tp + fp, 1)
    recall = tp / max(int(y.sum()), 1)
    return precision, recall


def plot_precision_recall(y_true, probs, class_names: Optional[List[str]] = None) -> bytes:
    plt = _plt()
    probs = np.asarray(probs)
    fig, ax = plt.subplots(figsize=(5, 4))
    for c in range(probs.shape[1]):
        p, r = precision_recall_curve(np.asarray(y_true) == c, probs[:, c])
        ax.plot(r, p, label=(class_names[c] if class_names else str(c)))
    ax.set_xlabel('recall')
    ax.set_ylabel('precision')
    ax.set_xlim(0, 1)
    ax.set_ylim(0, 1.02)
    ax.legend(fontsize=7)
    return figure_to_bytes(fig)


__all__ = ['figure_to_bytes', 'classification_report_table', 'plot_classification_report', 'precision_recall_curve',
           'plot_precision_recall']
