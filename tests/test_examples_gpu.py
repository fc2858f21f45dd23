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
