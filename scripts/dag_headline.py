"""The headline through the DAG path (verdict r2: "the metric is the ResNet-50 DAG train
task"): `mlcomp execute` of examples/resnet50_ddp with gpu: 1 runs the whole control
plane - DAG rows, ExecuteBuilder, the catalyst/train executor, the config-driven Runner
with its callbacks, DB progress and report series - and the throughput is read back
from the task's ``_timer/_fps`` report series (the reference's own metric,
`base_time.yml:9`).  Prints one JSON line next to what bench.py measures.

usage: python scripts/dag_headline.py [--steps 200] [--epochs 2] [--out FILE]"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--epochs', type=int, default=2)
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    work = tempfile.mkdtemp(prefix='dag_headline_')
    proj = os.path.join(work, 'resnet50_ddp')
    shutil.copytree(os.path.join(ROOT, 'examples', 'resnet50_ddp'), proj)
    cfg = yaml.safe_load(open(os.path.join(proj, 'config.yml')))
    cfg['executors']['train']['gpu'] = 1
    yaml.safe_dump(cfg, open(os.path.join(proj, 'config.yml'), 'w'))
    cat = yaml.safe_load(open(os.path.join(proj, 'catalyst.yml')))
    cat['stages']['data_params']['steps'] = a.steps
    cat['stages']['state_params']['num_epochs'] = a.epochs
    yaml.safe_dump(cat, open(os.path.join(proj, 'catalyst.yml'), 'w'))
    env = dict(os.environ, MLCOMP_ROOT=os.path.join(work, 'root'), PYTHONPATH=ROOT, MLCOMP_BROKER='inproc')
    t0 = time.time()
    subprocess.run([sys.executable, '-m', 'mlcomp_amd', 'migrate'], env=env, cwd=proj, check=True)
    r = subprocess.run([sys.executable, '-m', 'mlcomp_amd', 'execute', 'config.yml'], env=env, cwd=proj)
    wall = time.time() - t0
    os.environ.update(MLCOMP_ROOT=env['MLCOMP_ROOT'])
    sys.path.insert(0, ROOT)
    from mlcomp_amd import config
    config.reset()
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.enums import TaskStatus
    from mlcomp_amd.db.models import ReportSeries, Task
    s = Session.create_session(key='headline')
    task = s.query(Task).order_by(Task.id.desc()).first()
    series = {(x.name, x.part, x.epoch): x.value for x in s.query(ReportSeries).filter(ReportSeries.task == task.id)}
    fps = {e: series.get(('_timer/_fps', 'train', e)) for e in range(a.epochs)}
    batch = cat['stages']['data_params']['batch_size']
    res = {'metric': 'images/sec ResNet-50 DAG train task (mlcomp execute, _timer/_fps)', 'n_gpus': 1,
           'task_status': TaskStatus(task.status).name, 'exit_code': r.returncode,
           'fps_per_epoch': fps, 'steady_state_fps': fps.get(a.epochs - 1),
           'ms_per_step': 1000.0 * batch / fps[a.epochs - 1] if fps.get(a.epochs - 1) else None,
           'batch': batch, 'steps_per_epoch': a.steps, 'epochs': a.epochs, 'wall_s': round(wall, 1),
           'train_loss': {e: series.get(('loss', 'train', e)) for e in range(a.epochs)}}
    print(json.dumps(res))
    if a.out:
        os.makedirs(os.path.dirname(a.out) or '.', exist_ok=True)
        json.dump(res, open(a.out, 'w'), indent=1)
    shutil.rmtree(work, ignore_errors=True)
    return 0 if r.returncode == 0 and task.status == TaskStatus.Success.value else 1


if __name__ == '__main__':
    sys.exit(main())
