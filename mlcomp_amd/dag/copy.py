"""DAG copy / restart with file patches (`create_dags/copy.py:16-153`).

``file_changes`` is YAML ``{path_regex: patch}``: for a matching ``.yml`` file the
patch (a mapping) is merged with :func:`merge_dicts_smart`; for other files the patch
is a list of ``[old, new]`` string replacements.  Patched content becomes a new
content-addressed ``file`` row; everything else is shared with the source DAG."""
from __future__ import annotations

import hashlib
import re

from mlcomp_amd.db.enums import TaskStatus
from mlcomp_amd.db.models import Dag, DagStorage, File, Task, TaskDependence, now
from mlcomp_amd.db.providers import DagProvider, DagStorageProvider, TaskProvider
from mlcomp_amd.utils.misc import merge_dicts_smart, yaml_dump, yaml_load


def _patch(path: str, changes: dict):
    for k, v in changes.items():
        if re.match(k, path):
            return v
    return None


def dag_copy(session, dag: int, file_changes: str = '', dag_suffix: str = '') -> int:
    src = DagProvider(session).by_id(dag)
    name = src.name + (' ' + dag_suffix if dag_suffix else '')
    new = Dag(name=name, created=now(), config=src.config, project=src.project,
              docker_img=src.docker_img, img_size=0, file_size=0, type=src.type, report=None)
    session.add(new, commit=False)
    session.flush()
    old2new = {}
    for t in TaskProvider(session).by_dag(dag):
        if t.parent:
            continue
        nt = Task(name=t.name, status=TaskStatus.NotRan.value, computer=t.computer, gpu=t.gpu,
                  gpu_max=t.gpu_max, cpu=t.cpu, executor=t.executor, memory=t.memory, steps=t.steps,
                  dag=new.id, debug=t.debug, type=t.type, continued=False,
                  additional_info=t.additional_info)
        session.add(nt, commit=False)
        session.flush()
        old2new[t.id] = nt.id
    for d in TaskProvider(session).get_dependencies(dag):
        if d.task_id in old2new and d.depend_id in old2new:
            session.add(TaskDependence(task_id=old2new[d.task_id], depend_id=old2new[d.depend_id]),
                        commit=False)
    changes = yaml_load(file_changes) if file_changes else {}
    for s, f in DagStorageProvider(session).by_dag(dag):
        fid = s.file
        rep = _patch(s.path, changes) if isinstance(changes, dict) and f is not None else None
        if rep is not None:
            content = f.content.decode('utf-8')
            if s.path.endswith(('.yml', '.yaml')):
                content = yaml_dump(merge_dicts_smart(yaml_load(content) or {}, rep))
            else:
                for old, newtxt in rep:
                    if old not in content:
                        raise ValueError(f'{old!r} is not in {s.path}')
                    content = content.replace(old, newtxt)
            data = content.encode('utf-8')
            md5 = hashlib.md5(data).hexdigest()
            nf = session.query(File).filter(File.md5 == md5).filter(File.project == new.project).first()
            if nf is None:
                nf = File(content=data, created=now(), project=new.project, md5=md5, dag=new.id)
                session.add(nf, commit=False)
                session.flush()
            fid = nf.id
        session.add(DagStorage(dag=new.id, file=fid, path=s.path, is_dir=s.is_dir), commit=False)
    session.commit()
    return new.id


__all__ = ['dag_copy']
