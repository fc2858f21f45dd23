"""Model registry DAGs (`create_dags/model_add.py:10-57`, `model_start.py:10-70`):
``dag_model_add`` exports a trained task's checkpoint as a ``model`` row (through a
one-executor ``model_add`` DAG on the computer that holds the checkpoint);
``dag_model_start`` instantiates a pipe of a Pipe DAG for a registered model."""
from __future__ import annotations

from mlcomp_amd.db.models import Model, now
from mlcomp_amd.db.providers import DagProvider, ModelProvider, ProjectProvider, TaskProvider
from mlcomp_amd.utils.misc import yaml_dump, yaml_load
from .standard import dag_standard


def dag_model_add(session, data: dict):
    if not data.get('task'):
        m = Model(name=data['name'], project=data['project'], equations=data.get('equations', ''),
                  created=now(), fold=data.get('fold'))
        ModelProvider(session).add(m)
        return {'model': m.id}
    tp = TaskProvider(session)
    task = tp.by_id(data['task'])
    children = tp.children(task.id)
    computer = children[0].computer_assigned if children else task.computer_assigned
    child = children[0].id if children else None
    dag = DagProvider(session).by_id(task.dag)
    project = ProjectProvider(session).by_id(dag.project)
    config = {'info': {'name': 'model_add', 'project': project.name, 'computer': computer},
              'executors': {'model_add': {'type': 'model_add', 'project': data['project'],
                                          'task': data['task'], 'name': data['name'],
                                          'file': data.get('file', 'best'), 'child_task': child,
                                          'fold': data.get('fold', 0)}}}
    return dag_standard(session, config, debug=False, upload_files=False)


def dag_model_start(session, data: dict):
    mp = ModelProvider(session)
    model = mp.by_id(data['model_id'])
    dag = DagProvider(session).by_id(data['dag'])
    project = ProjectProvider(session).by_id(dag.project)
    src = yaml_load(dag.config)
    pipe_name = data['pipe']['name']
    pipe = src['pipes'][pipe_name]
    equations = yaml_load(model.equations) or {}
    versions = data['pipe'].get('versions', [])
    if versions:
        version = data['pipe']['version']
        eq = yaml_load(version.get('equations', '')) or {}
        for v in versions:
            if v['name'] == version['name']:
                v['used'] = str(now())
        for v in pipe.values():
            v.update(eq)
    equations[pipe_name] = versions
    model.equations = yaml_dump(equations)
    for v in pipe.values():
        v['model_id'] = model.id
        v['model_name'] = model.name
    model.dag = dag.id
    mp.commit()
    config = {'info': {'name': pipe_name, 'project': project.name}, 'executors': pipe}
    return dag_standard(session, config, debug=False, upload_files=False, copy_files_from=data['dag'])


def model_start_begin(session, model_id: int) -> dict:
    """The project's Pipe DAGs (newest first, one per name) with their pipes ordered by
    the last time a version was used; feeds the UI's "start model" dialog."""
    from mlcomp_amd.db.enums import DagType
    from mlcomp_amd.db.models import Dag
    model = ModelProvider(session).by_id(model_id)
    dags = session.query(Dag).filter(Dag.type == DagType.Pipe.value).filter(
        Dag.project == model.project).order_by(Dag.id.desc()).all()
    versions = yaml_load(model.equations) or {}
    seen, res, current = set(), [], None
    for dag in dags:
        if dag.name in seen:
            continue
        seen.add(dag.name)
        cfg = yaml_load(dag.config) or {}
        pipes = []
        for name in (cfg.get('pipes') or {}):
            vs = [dict(v) for v in versions.get(name, [])]
            used = max((str(v.get('used', '')) for v in vs), default='')
            for v in vs:
                v.pop('used', None)
            pipes.append((used, {'name': name, 'versions': vs}))
        pipes.sort(key=lambda x: x[0], reverse=True)
        d = {'name': dag.name, 'id': dag.id, 'pipes': [p for _, p in pipes]}
        res.append(d)
        if dag.id == model.dag:
            current = d
    return {'dags': res, 'dag': current, 'model_id': model_id}


__all__ = ['dag_model_add', 'dag_model_start', 'model_start_begin']
