"""The shipped example DAGs on the MI355X through the whole stack (YAML -> scheduler ->
native broker -> worker pool -> task process -> Train executor -> runner): the user
experiment folder `cifar_simple` (a registered CNN) and the reference's digit-recognizer
LeNet train on the generic native engine, and the task records which engine ran."""
import pytest

from test_examples_cpu import _ids, _run_example, _wait_live
from test_lifecycle import cluster  # noqa: F401

pytestmark = pytest.mark.gpu


def _engine_info(tid):
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.models import Task
    from mlcomp_amd.utils.misc import yaml_load
    t = Session.create_session(key='eng').get(Task, tid)
    return t, (yaml_load(t.additional_info) or {}).get('engine', {})


def test_cifar_simple_example_trains_natively_through_the_dag(cluster):
    from mlcomp_amd.db.enums import TaskStatus
    ids = _ids(_run_example(cluster['tmp'], 'cifar_simple/config.yml',
                            params={'executors/train/params/stages/state_params/num_epochs': 2}))
    res = _wait_live(cluster, ids, timeout=400)
    assert all(v == TaskStatus.Success for v in res.values()), res
    t, eng = _engine_info(ids[0])
    assert eng['stage1']['engine'] == 'native' and eng['stage1']['kind'] == 'generic', eng
    assert t.score is not None and t.score > 0.3


def test_digit_recognizer_lenet_trains_natively_through_the_dag(cluster):
    from mlcomp_amd.db.enums import TaskStatus
    prep = _ids(_run_example(cluster['tmp'], 'digit-recognizer/prepare.yml'))
    assert all(v == TaskStatus.Success for v in _wait_live(cluster, prep, timeout=300).values())
    ids = _ids(_run_example(cluster['tmp'], 'digit-recognizer/train.yml',
                            params={'executors/train/params/stages/state_params/num_epochs': 2}))
    res = _wait_live(cluster, ids, timeout=400)
    assert all(v == TaskStatus.Success for v in res.values()), res
    _, eng = _engine_info(ids[0])
    assert eng['stage1']['engine'] == 'native' and eng['stage1']['kind'] == 'generic', eng


@pytest.mark.timeout(400)
def test_multi_branch_resnet50_and_bert_dag_on_one_gpu(cluster):
    """BASELINE config 5 (ResNet-50 + BERT-base train tasks in one DAG) through the whole
    stack on the box's one GPU: with one GPU per task the scheduler runs the two branches one
    after the other, both full-size models on their native engines (short epochs)."""
    from mlcomp_amd.db.enums import TaskStatus
    ids = _ids(_run_example(cluster['tmp'], 'multi_branch/config.yml', params={
        'executors/resnet50/gpu': 1, 'executors/bert/gpu': 1,
        'executors/resnet50/params/stages/data_params/steps': 20,
        'executors/resnet50/params/stages/state_params/num_epochs': 1,
        'executors/bert/params/stages/data_params/num_samples': 2048,
        'executors/bert/params/stages/data_params/valid_samples': 256,
        'executors/bert/params/stages/state_params/num_epochs': 1}))
    res = _wait_live(cluster, ids, timeout=360)
    assert all(v == TaskStatus.Success for v in res.values()), res
    engines = {}
    for tid in ids:
        t, eng = _engine_info(tid)
        if eng:
            engines[t.executor] = eng['stage1']
    assert set(engines) == {'resnet50', 'bert'}, engines
    assert all(e['engine'] == 'native' for e in engines.values()), engines


@pytest.mark.timeout(400)
def test_unet_segmentation_train_then_valid_dag_on_gpu(cluster):
    """BASELINE config 3 (U-Net segmentation DAG: train node -> traced model -> valid node)
    on the box's one GPU: the train task runs the native U-Net engine, traces the model, and
    the valid_segmentation task scores it."""
    from mlcomp_amd.db.enums import TaskStatus
    ids = _ids(_run_example(cluster['tmp'], 'unet_segmentation/config.yml', params={
        'executors/train/gpu': 1,
        'executors/train/params/stages/data_params/num_samples': 256,
        'executors/train/params/stages/data_params/valid_samples': 64,
        'executors/train/params/stages/state_params/num_epochs': 1}))
    res = _wait_live(cluster, ids, timeout=360)
    assert all(v == TaskStatus.Success for v in res.values()), res
    t, eng = _engine_info(ids[0])
    assert t.executor == 'train' and eng['stage1']['engine'] == 'native', eng


@pytest.mark.timeout(600)
def test_resnet50_dag_train_task_throughput_matches_bench(cluster):
    """The headline metric measured where the reference reports it: the ResNet-50 DAG train
    task (examples/resnet50_ddp, batch 512 per GPU, native engine) through scheduler ->
    broker -> worker -> runner, its ``_timer/_fps`` series of the warm epoch (reference:
    migration/versions/002/report_layout/base_time.yml:9) within 5 % of bench.py's bare
    step at the same config, run in the same test on the same GPU."""
    import json
    import os
    import subprocess
    import sys
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.enums import TaskStatus
    from mlcomp_amd.db.models import ReportSeries
    ids = _ids(_run_example(cluster['tmp'], 'resnet50_ddp/config.yml', params={
        'executors/train/gpu': 1,
        'executors/train/params/stages/data_params/steps': 120,
        'executors/train/params/stages/state_params/num_epochs': 2}))
    res = _wait_live(cluster, ids, timeout=480)
    assert all(v == TaskStatus.Success for v in res.values()), res
    s = Session.create_session(key='fps')
    rows = s.query(ReportSeries).filter(ReportSeries.task.in_(ids), ReportSeries.name == '_timer/_fps',
                                        ReportSeries.part == 'train').all()
    assert rows, 'no _timer/_fps series'
    dag_fps = max(rows, key=lambda r: r.epoch).value
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--steps', '30', '--warmup', '5'],
                       capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    bench = json.loads(r.stdout.strip().splitlines()[-1])
    print(f'DAG train task _timer/_fps {dag_fps:.1f} img/s (epoch {max(x.epoch for x in rows)}), '
          f'bench.py {bench["value"]:.1f} img/s')
    assert dag_fps >= 0.95 * bench['value'], (dag_fps, bench['value'])
