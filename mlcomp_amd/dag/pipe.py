"""Pipe DAGs: reusable inference pipelines stored as a DAG of type Pipe whose
``pipes:`` section holds executor templates; models that referenced an older pipe DAG
of the same name are re-pointed to the new one (`create_dags/pipe.py:10-36`)."""
from __future__ import annotations

import os

from mlcomp_amd.db.enums import DagType
from mlcomp_amd.db.models import Dag, Model, now
from mlcomp_amd.db.providers import ProjectProvider
from mlcomp_amd.utils.misc import yaml_dump


def dag_pipe(session, config: dict, config_text: str = None, folder: str = None):
    if 'pipes' not in config:
        raise ValueError('pipe DAG config needs a "pipes" section')
    info = config['info']
    pp = ProjectProvider(session)
    project = (pp.by_name(info['project']) or pp.add_project(info['project'])).id
    dag = Dag(config=config_text or yaml_dump(config), project=project, name=info['name'],
              docker_img=info.get('docker_img'), type=DagType.Pipe.value, created=now(),
              file_size=0, img_size=0)
    session.add(dag)
    from mlcomp_amd.worker.storage import Storage
    Storage(session).upload(folder or os.getcwd(), dag)
    old = session.query(Dag.id).filter(Dag.project == project).filter(Dag.name == info['name']).filter(
        Dag.type == DagType.Pipe.value).filter(Dag.id != dag.id)
    session.query(Model).filter(Model.dag.in_(old)).update({'dag': dag.id}, synchronize_session=False)
    session.commit()
    return {'pipe': [dag.id]}


__all__ = ['dag_pipe']
