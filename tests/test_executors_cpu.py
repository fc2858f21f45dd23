"""Model tracing / model_add, equation executors (Valid / Infer) and the report
builders, on CPU against a real DB."""
import os

import numpy as np
import pytest
import torch
import yaml

from mlcomp_amd.train.experiment import ConfigExperiment
from mlcomp_amd.train.runner import Runner


def _train_cfg(logdir):
    return {'model_params': {'model': 'SimpleCNN', 'num_classes': 4, 'width': 8},
            'args': {'expdir': '.', 'logdir': str(logdir), 'engine': 'torch'},
            'stages': {'data_params': {'dataset': 'synthetic_classification', 'batch_size': 8, 'num_samples': 16,
                                       'valid_samples': 8, 'image_size': 16, 'num_classes': 4},
                       'state_params': {'num_epochs': 1},
                       'optimizer_params': {'optimizer': 'SGD', 'lr': 0.01},
                       'callbacks_params': {'loss': {'callback': 'CriterionCallback'},
                                            'opt': {'callback': 'OptimizerCallback'},
                                            'saver': {'callback': 'CheckpointCallback'}},
                       'stage1': {}}}


def test_trace_model_from_checkpoint(tmp_path):
    from mlcomp_amd.worker.executors.model import trace_model_from_checkpoint
    r = Runner(ConfigExperiment(_train_cfg(tmp_path / 'log')), device='cpu')
    r.run_experiment()
    assert (tmp_path / 'log' / 'configs' / '_config.json').exists()
    traced = trace_model_from_checkpoint(str(tmp_path / 'log'), file='last')
    x = torch.randn(3, 3, 16, 16)
    r.model.eval()
    assert torch.allclose(traced(x), r.model(x), atol=1e-5)


@pytest.fixture
def dbtask(mlc_root, monkeypatch):
    monkeypatch.setenv('MLCOMP_COMPUTER', 'exhost')
    from mlcomp_amd import broker, config
    config.reset()
    broker.set_broker(broker.InProcBroker())
    from mlcomp_amd.db.migrate import migrate
    migrate()
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.models import Dag, Task, now
    from mlcomp_amd.db.providers import ProjectProvider, TaskProvider
    s = Session.create_session(key='ex')
    p = ProjectProvider(s).add_project('pex')
    d = Dag(name='d', project=p.id, config='', created=now(), file_size=0, img_size=0, type=0)
    s.add(d)
    t = Task(name='v', dag=d.id, executor='v', status=2, type=0, gpu=0, cpu=1,
             memory=0.1, steps=1, last_activity=now())
    s.add(t)
    yield s, t, TaskProvider(s), p
    broker.set_broker(None)
    Session.cleanup()


class _Arr(torch.utils.data.Dataset):
    def __init__(self, x, y):
        self.x, self.y = x, y

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return {'features': self.x[i], 'targets': int(self.y[i])}


def _export_model(folder):
    torch.manual_seed(0)
    from mlcomp_amd.models import build_model
    m = build_model('SimpleCNN', num_classes=3, width=4).eval()
    os.makedirs(folder, exist_ok=True)
    torch.jit.save(torch.jit.trace(m, torch.randn(1, 3, 8, 8)), os.path.join(folder, 'net.pth'))
    return m


def test_valid_and_infer_equations(dbtask, tmp_path):
    from mlcomp_amd import config
    from mlcomp_amd.worker.executors.infer import Infer
    from mlcomp_amd.worker.executors.valid import Valid
    from mlcomp_amd.worker.reports import ClassificationReportBuilder
    s, task, tp, project = dbtask
    model = _export_model(os.path.join(config.get().MODEL_FOLDER, project.name))
    g = torch.Generator().manual_seed(1)
    X = torch.randn(20, 3, 8, 8, generator=g)
    with torch.no_grad():
        Y = model(X).argmax(1)      # labels = the model's own predictions -> accuracy 1.0

    class V(Valid):
        def __init__(self, **kw):
            super().__init__(layout='img_classify', plot_count=1, part_size=7, **kw)
            self.src = _Arr(X, Y)
            self.scores = []

        def create_base(self):
            self.builder = ClassificationReportBuilder(self.session, self.task, self.layout, plot_count=1)
            self.builder.create_base()

        def count(self):
            return len(self.src)

        def adjust_part(self, part):
            self.x = _Arr(X[part[0]:part[1]], Y[part[0]:part[1]])

        def score(self, preds):
            r = (preds.argmax(1) == self.x.y.numpy()).astype(np.float64)
            self.scores.extend(r)
            return r

        def score_final(self):
            return float(np.mean(self.scores))

        def plot(self, preds, scores):
            imgs = [np.zeros((8, 8, 3), np.uint8) + 100 for _ in range(len(preds))]
            self.builder.process_pred(imgs, preds, self.x.y.numpy(), scores={'accuracy': scores})

    v = V(y="torch(x, file='net.pth', batch_size=4)")
    v.session, v.task, v.task_provider = s, task, tp
    res = v.work()
    assert res['score'] == pytest.approx(1.0)
    assert task.score == pytest.approx(1.0)
    from mlcomp_amd.db.models import ReportImg
    imgs = s.query(ReportImg).filter(ReportImg.task == task.id).all()
    assert any(r.group == 'img_classify' for r in imgs)
    assert any(r.group == 'img_classify_confusion' for r in imgs)
    jpg = [r for r in imgs if r.group == 'img_classify'][0].img
    assert jpg[:2] == b'\xff\xd8'

    saved = []

    class I(Infer):
        def __init__(self, **kw):
            super().__init__(part_size=8, **kw)

        def count(self):
            return len(X)

        def adjust_part(self, part):
            self.x = _Arr(X[part[0]:part[1]], Y[part[0]:part[1]])

        def save(self, preds, folder):
            saved.append(preds)

        def save_final(self, folder):
            np.save(os.path.join(folder, 'p.npy'), np.concatenate(saved))

    inf = I(y="torch(x, file='net.pth', batch_size=8, activation='softmax')", z='y * 2')
    inf.session, inf.task, inf.task_provider = s, task, tp
    inf.work()
    allp = np.concatenate(saved)
    assert allp.shape == (20, 3) and np.allclose(allp.sum(1), 1, atol=1e-5)
    assert np.allclose(inf.solve('z', inf.part), 2 * inf.cache['y'])


def test_segmentation_report_and_rle(dbtask):
    from mlcomp_amd.contrib.transform import mask2rle, rle2mask
    from mlcomp_amd.worker.reports import SegmentationReportBuilder
    m = np.zeros((6, 5), np.uint8)
    m[1:4, 2] = 1
    m[5, 4] = 1
    assert (rle2mask(mask2rle(m), (5, 6)) == m).all()
    s, task, tp, _ = dbtask
    b = SegmentationReportBuilder(s, task, layout='img-segment', plot_count=1)
    b.create_base()
    pred = np.random.rand(2, 2, 16, 16)
    tgt = (np.random.rand(2, 2, 16, 16) > 0.5)
    b.process_pred([np.zeros((16, 16, 3), np.uint8)] * 2, pred, tgt, scores={'dice': [0.5, 0.7]})
    from mlcomp_amd.db.models import ReportImg
    rows = s.query(ReportImg).filter(ReportImg.task == task.id).all()
    assert len(rows) == 2 and rows[0].score == 0.5


def test_report_plots_and_describe(dbtask):
    from mlcomp_amd.utils.plot import classification_report_table, plot_classification_report, plot_precision_recall
    y = np.array([0, 1, 2, 1, 0, 2])
    p = np.eye(3)[[0, 1, 1, 1, 0, 2]] * 0.9 + 0.03
    t = classification_report_table(y, p.argmax(1), 3)
    assert t[2, 1] == 0.5 and t[0, 0] == 1.0
    assert plot_classification_report(y, p.argmax(1), 3)[:2] == b'\xff\xd8'
    assert plot_precision_recall(y, p)[:2] == b'\xff\xd8'
    s, task, tp, _ = dbtask
    from mlcomp_amd.utils.describe import draw, task_table
    rows = task_table(task.dag)
    assert rows and rows[0]['status'] == 'in_progress'
    fig = draw(task.dag, metrics=['loss'])
    assert fig is not None
