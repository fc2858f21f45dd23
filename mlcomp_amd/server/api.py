"""REST API + web UI (`mlcomp/server/back/app.py`).

Same contract as the reference so its front-end / scripts keep working:

* every endpoint is ``POST /api/<name>`` with a JSON body (object, or a bare id);
* ``Authorization: <TOKEN>`` header required (except ``/api/token``), 401 otherwise;
* the response is the handler's dict plus ``success`` / ``error`` (traceback text,
  HTTP 500) - SQLAlchemy errors also reset the sessions;
* list endpoints take ``paginator: {page_number, page_size, sort_column,
  sort_descending}`` and answer ``{total, data}``.

Implementation: FastAPI/uvicorn (Flask is not part of this stack) with one route table;
handlers run under a single lock because the SQLAlchemy sessions are shared - the API
is a control plane, not a hot path.  ``start_server`` also starts the scheduler thread.
The UI at ``/`` is a small self-contained dashboard (``server/static/index.html``).
"""

import hashlib
import json
import math
import os
import shutil
import threading
import traceback
from collections import OrderedDict
from typing import Callable, Dict

from mlcomp_amd import config
from mlcomp_amd.db.core import PaginatorOptions, Session
from mlcomp_amd.db.enums import ComponentType, TaskStatus
from mlcomp_amd.db.models import (DagStorage, DagTag, File, Memory, Report, ReportLayout, Space,
                                  SpaceTag, Task, now)
from mlcomp_amd.db.providers import (AuxiliaryProvider, ComputerProvider, DagProvider, DagStorageProvider,
                                     FileProvider, LogProvider, MemoryProvider, ModelProvider,
                                     ProjectProvider, ReportImgProvider, ReportLayoutProvider,
                                     ReportProvider, SpaceProvider, StepProvider, TaskProvider)
from mlcomp_amd.db.report_info import ReportLayoutInfo
from mlcomp_amd.utils.logging import create_logger
from mlcomp_amd.utils.misc import yaml_dump, yaml_load

ROUTES: Dict[str, Callable] = OrderedDict()
STATIC = os.path.join(os.path.dirname(__file__), 'static')


def route(name: str):
    def deco(fn):
        ROUTES[name] = fn
        return fn
    return deco


class Ctx:
    """Shared read/write sessions + the scheduler handle."""

    def __init__(self):
        self.lock = threading.RLock()
        self.reset()
        self.supervisor = None

    def reset(self):
        Session.cleanup('server.read')
        Session.cleanup('server.write')
        self.read = Session.create_session(key='server.read')
        self.write = Session.create_session(key='server.write')
        self.logger = create_logger(self.write, 'api')


_CTX: Ctx = None


def ctx() -> Ctx:
    global _CTX
    if _CTX is None:
        _CTX = Ctx()
    return _CTX


def _opts(data, default_sort='id') -> PaginatorOptions:
    p = (data or {}).get('paginator') or {} if isinstance(data, dict) else {}
    return PaginatorOptions(page_number=int(p.get('page_number') or 0), page_size=int(p.get('page_size') or 0),
                            sort_column=p.get('sort_column') or default_sort,
                            sort_descending=str(p.get('sort_descending', True)).lower() in ('true', '1'))


def _id(data):
    return int(data['id']) if isinstance(data, dict) else int(data)


def _clean(o):
    """JSON-safe: NaN/inf -> None, datetimes -> isoformat."""
    if isinstance(o, float):
        return None if math.isnan(o) or math.isinf(o) else o
    if isinstance(o, dict):
        return {k: _clean(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_clean(v) for v in o]
    if hasattr(o, 'isoformat'):
        return o.isoformat()
    return o


def dispatch(name: str, data, token: str):
    """Run one API call; returns (status, body dict). Used by the HTTP layer and tests."""
    c = ctx()
    s = config.get()
    if name != 'token' and (token is None or str(token).strip() != s.TOKEN):
        return 401, {'success': False, 'error': 'Could not verify your access level for that URL.'}
    fn = ROUTES.get(name)
    if fn is None:
        return 404, {'success': False, 'error': f'unknown endpoint {name}'}
    with c.lock:
        try:
            res = fn(data)
            if isinstance(res, tuple):   # (status, body) from token()
                return res
            res = dict(res or {}) if isinstance(res, dict) or res is None else {'data': res}
            res.update(success=True, error='')
            return 200, _clean(res)
        except Exception as e:  # noqa: BLE001  - the envelope carries it
            tb = traceback.format_exc()
            if Session.sqlalchemy_error(e):
                c.reset()
            try:
                c.logger.error(f'Requested Url: /api/{name}\n\n{tb}', ComponentType.API)
            except Exception:
                pass
            return 500, {'success': False, 'error': tb}


# ---------------------------------------------------------------------------- auth
@route('token')
def token(data):
    if str((data or {}).get('token', '')).strip() != config.get().TOKEN:
        return 401, {'success': False, 'reason': 'invalid token'}
    return 200, {'success': True}


# ---------------------------------------------------------------------------- computers
@route('computers')
def computers(data):
    """Computers with current usage, dockers and ``usage_history`` since
    ``usage_min_time`` (default: the last day) in the reference's shape
    {time: [...], mean: [{name: cpu|memory|disk|gpu_<i>, value: [...]}]}
    (`mlcomp/db/providers/computer.py:71-103`), thinned to at most 300 points."""
    import datetime
    from mlcomp_amd.db.providers import parse_time
    o = _opts(data, 'name')
    o.sort_column = 'name'
    data = data if isinstance(data, dict) else {}
    cp = ComputerProvider(ctx().read)
    res = cp.get(data, o)
    since = parse_time(data['usage_min_time']) if data.get('usage_min_time') else now() - datetime.timedelta(days=1)
    for item in res['data']:
        rows = cp.usage_history(item['name'], since)
        step = max(1, len(rows) // 300)
        rows = rows[::step]
        mean = OrderedDict((k, []) for k in ('cpu', 'memory', 'disk'))
        for r in rows:
            for k in ('cpu', 'memory', 'disk'):
                mean[k].append(r.get(k))
            for i, g in enumerate(r.get('gpu') or []):
                mean.setdefault(f'gpu_{i}', []).append(g.get('load'))
        item['usage_history'] = {'time': [r['time'] for r in rows],
                                 'mean': [{'name': k, 'value': v} for k, v in mean.items()]}
    return res


@route('computer_sync_start')
def computer_sync_start(data):
    return {'data': [{'id': p['id'], 'name': p['name'], 'sync_folders': p.get('sync_folders'),
                      'ignore_folders': p.get('ignore_folders')}
                     for p in ProjectProvider(ctx().read).get({}, None)['data']],
            'computers': [c.name for c in ComputerProvider(ctx().read).all()]}


@route('computer_sync_end')
def computer_sync_end(data):
    cp = ComputerProvider(ctx().write)
    for c in cp.all():
        if data.get('computer') and data['computer'] != c.name:
            continue
        meta = yaml_load(c.meta) or {}
        meta['manual_sync'] = {'project': data['id'], 'sync_folders': yaml_load(data.get('sync_folders')),
                               'ignore_folders': yaml_load(data.get('ignore_folders'))}
        c.meta = yaml_dump(meta)
    cp.commit()


# ---------------------------------------------------------------------------- projects
@route('projects')
def projects(data):
    return ProjectProvider(ctx().read).get(data, _opts(data))


@route('project/add')
def project_add(data):
    ProjectProvider(ctx().write).add_project(data['name'], yaml_load(data.get('class_names')) or {},
                                             data.get('sync_folders') or '', data.get('ignore_folders') or '')


@route('project/edit')
def project_edit(data):
    pp = ProjectProvider(ctx().write)
    p = pp.by_id(data['id']) if data.get('id') else pp.by_name(data['name'])
    fields = {k: data[k] for k in ('class_names', 'sync_folders', 'ignore_folders') if k in data}
    if 'class_names' in fields and not isinstance(fields['class_names'], str):
        fields['class_names'] = yaml_dump(fields['class_names'])
    if data.get('new_name'):
        fields['name'] = data['new_name']
    pp.edit(p.id, **fields)


@route('project/remove')
def project_remove(data):
    ProjectProvider(ctx().write).remove(_id(data))


@route('project/stop_all_dags')
def stop_all_dags(data):
    tp = TaskProvider(ctx().write)
    ts = tp.by_status(TaskStatus.InProgress, TaskStatus.Queued, TaskStatus.NotRan, project=data['project'])
    for t in ts:
        info = yaml_load(t.additional_info) or {}
        info['stopped'] = True
        t.additional_info = yaml_dump(info)
    tp.commit()
    _supervisor().stop_tasks(ts)


@route('project/remove_all_dags')
def remove_all_dags(data):
    dp = DagProvider(ctx().write)
    from mlcomp_amd.db.models import Dag
    ids = [d.id for d in dp.query(Dag).filter(Dag.project == data['project']).all()]
    for i in ids:
        _remove_dag(i)


# ---------------------------------------------------------------------------- dags
@route('dags')
def dags(data):
    return DagProvider(ctx().read).get(data, _opts(data))


@route('config')
def dag_config(data):
    return {'data': DagProvider(ctx().read).config(_id(data))}


@route('graph')
def graph(data):
    return DagProvider(ctx().read).graph(_id(data))


@route('dag/stop')
def dag_stop(data):
    i = _id(data)
    ts = TaskProvider(ctx().write).by_dag(i)
    _supervisor().stop_tasks(ts)
    res = DagProvider(ctx().read).get({'id': i}, None)['data']
    return {'dag': res[0] if res else None}


@route('dag/start')
def dag_start(data):
    _supervisor().start_dag(_id(data))


@route('dag/restart')
def dag_restart(data):
    from mlcomp_amd.dag.copy import dag_copy
    return {'dag': dag_copy(ctx().write, int(data['dag']), data.get('file_changes') or '')}


def _remove_dag(i: int):
    from mlcomp_amd.worker.tasks import remove_dag_files
    remove_dag_files(ctx().write, i)
    DagProvider(ctx().write).remove(i)


@route('dag/remove')
def dag_remove(data):
    _remove_dag(_id(data))


@route('dag/tags')
def dag_tags(data):
    return {'data': DagProvider(ctx().read).tags((data or {}).get('name', ''))}


@route('dag/tag_add')
def dag_tag_add(data):
    DagProvider(ctx().write).add_tag(int(data['dag']), data['tag'])


@route('dag/tag_remove')
def dag_tag_remove(data):
    DagProvider(ctx().write).remove_tag(int(data['dag']), data['tag'])


@route('dag/toogle_report')
def dag_toggle_report(data):
    rp = ReportProvider(ctx().write)
    ids = [t.id for t in TaskProvider(ctx().write).by_dag(int(data['id']))]
    for t in ids:
        (rp.remove_task if data.get('remove') else rp.add_task)(int(data['report']), t)
    return {'report_full': not data.get('remove')}


# ---------------------------------------------------------------------------- code
@route('code')
def code(data):
    did = _id(data)
    roots, dirs = [], {}
    rows = DagStorageProvider(ctx().read).by_dag(did)
    for st, f in rows:
        path = st.path.strip().strip('/')
        if not path:
            continue
        parent, name = os.path.dirname(path), os.path.basename(path)
        if st.is_dir:
            node = {'name': name, 'children': [], 'id': st.id, 'dag': did, 'storage': st.id}
            dirs[path] = node
        else:
            try:
                content = f.content.decode('utf-8') if f is not None else ''
            except UnicodeDecodeError:
                content = ''
            node = {'name': name, 'id': f.id if f else None, 'dag': did, 'storage': st.id, 'content': content}
        (dirs[parent]['children'] if parent in dirs else roots).append(node)

    def key(n):
        return ('_____' if n.get('children') else '') + n['name']

    def sort(nodes):
        nodes.sort(key=key)
        for n in nodes:
            if n.get('children'):
                sort(n['children'])
    sort(roots)
    return {'items': roots}


@route('update_code')
def update_code(data):
    fp = FileProvider(ctx().write)
    f = fp.by_id(data['file_id'])
    content = data['content'].encode('utf-8')
    md5 = hashlib.md5(content).hexdigest()
    if md5 == f.md5:
        return {'file': f.id}
    if f.dag != data['dag']:
        nf = File(md5=md5, content=content, project=f.project, dag=data['dag'], created=now(), size=len(content))
        fp.add(nf)
        st = DagStorageProvider(ctx().write).by_id(data['storage'])
        st.file = nf.id
        fp.commit()
        return {'file': nf.id}
    f.content, f.md5 = content, md5
    fp.commit()
    return {'file': f.id}


@route('code_download')
def code_download(data):
    """Zip of the DAG's stored code, base64 in ``content`` (GET /api/code_download?id=
    streams the file itself)."""
    import base64
    return {'file_name': f'{_id(data)}.zip', 'content': base64.b64encode(_code_zip(_id(data))).decode()}


def _code_zip(did: int) -> bytes:
    from mlcomp_amd.worker.storage import Storage
    s = config.get()
    folder = os.path.join(s.TMP_FOLDER, f'code_{did}_{os.getpid()}')
    try:
        Storage(ctx().read).download_dag(did, folder)
        base = shutil.make_archive(folder, 'zip', folder)
        with open(base, 'rb') as f:
            out = f.read()
        os.remove(base)
        return out
    finally:
        shutil.rmtree(folder, ignore_errors=True)


# ---------------------------------------------------------------------------- tasks
@route('tasks')
def tasks(data):
    return TaskProvider(ctx().read).get(data, _opts(data))


@route('task/stop')
def task_stop(data):
    tp = TaskProvider(ctx().write)
    t = tp.by_id(_id(data))
    _supervisor().stop_tasks([t] + tp.children(t.id))


@route('task/info')
def task_info(data):
    t = TaskProvider(ctx().read).by_id(_id(data))
    return {'pid': t.pid, 'worker_index': t.worker_index, 'gpu_assigned': t.gpu_assigned,
            'celery_id': t.celery_id, 'additional_info': t.additional_info or '', 'result': t.result or '',
            'id': t.id}


@route('task/steps')
def task_steps(data):
    return StepProvider(ctx().read).get(_id(data))


@route('task/toogle_report')
def task_toggle_report(data):
    rp = ReportProvider(ctx().write)
    (rp.remove_task if data.get('remove') else rp.add_task)(int(data['report']), int(data['id']))
    return {'report_full': not data.get('remove')}


@route('logs')
def logs(data):
    return LogProvider(ctx().read).get(data, _opts(data))


@route('auxiliary')
def auxiliary(data):
    return AuxiliaryProvider(ctx().read).get()


# ---------------------------------------------------------------------------- reports
@route('reports')
def reports(data):
    return ReportProvider(ctx().read).get(data, _opts(data))


@route('report')
def report(data):
    return ReportProvider(ctx().read).detail(_id(data))


@route('report/add_start')
def report_add_start(data):
    return {'projects': ProjectProvider(ctx().read).get({}, None)['data'],
            'layouts': ReportLayoutProvider(ctx().read).get()['data']}


@route('report/add_end')
def report_add_end(data):
    layouts = ReportLayoutProvider(ctx().write).all()
    ReportProvider(ctx().write).add(Report(name=data['name'], project=data['project'], layout=data['layout'],
                                           config=yaml_dump(layouts[data['layout']]), time=now()))


@route('report/update_layout_start')
def report_update_layout_start(data):
    r = ReportProvider(ctx().read).by_id(_id(data))
    return {'id': r.id, 'layout': r.layout, 'layouts': list(ReportLayoutProvider(ctx().read).all())}


@route('report/update_layout_end')
def report_update_layout_end(data):
    rp = ReportProvider(ctx().write)
    r = rp.by_id(int(data['id']))
    layouts = ReportLayoutProvider(ctx().write).all()
    r.layout = data['layout']
    r.config = yaml_dump(layouts[data['layout']])
    rp.commit()
    return rp.detail(r.id)


@route('layouts')
def layouts(data):
    return ReportLayoutProvider(ctx().read).get(data, _opts(data))


@route('layout/add')
def layout_add(data):
    ReportLayoutProvider(ctx().write).add(ReportLayout(name=data['name'], content=data.get('content', ''),
                                                       last_modified=now()))


@route('layout/edit')
def layout_edit(data):
    lp = ReportLayoutProvider(ctx().write)
    lay = lp.by_name(data['name'])
    lay.last_modified = now()
    if data.get('content') is not None:
        ReportLayoutInfo(yaml_load(data['content']) or {})   # validate before storing
        lay.content = data['content']
    if data.get('new_name'):
        lay.name = data['new_name']
    lp.commit()


@route('layout/remove')
def layout_remove(data):
    lp = ReportLayoutProvider(ctx().write)
    lp.query(ReportLayout).filter(ReportLayout.name == data['name']).delete(synchronize_session=False)
    lp.commit()


@route('img_classify')
def img_classify(data):
    return ReportImgProvider(ctx().read).get(data, _opts(data))


@route('img_segment')
def img_segment(data):
    return ReportImgProvider(ctx().read).get(data, _opts(data))


@route('remove_imgs')
def remove_imgs(data):
    from mlcomp_amd.db.models import ReportImg
    p = ReportImgProvider(ctx().write)
    q = p.query(ReportImg)
    for k in ('dag', 'task', 'project'):
        if data.get(k) is not None:
            q = q.filter(getattr(ReportImg, k) == data[k])
    n = q.delete(synchronize_session=False)
    p.commit()
    return {'removed': n}


@route('remove_files')
def remove_files(data):
    p = FileProvider(ctx().write)
    q = p.query(File)
    for k in ('dag', 'project'):
        if data.get(k) is not None:
            q = q.filter(getattr(File, k) == data[k])
    n = q.delete(synchronize_session=False)
    p.commit()
    return {'removed': n}


# ---------------------------------------------------------------------------- models
@route('models')
def models(data):
    return ModelProvider(ctx().read).get(data, _opts(data))


@route('model/add')
def model_add(data):
    from mlcomp_amd.dag.model import dag_model_add
    dag_model_add(ctx().write, data)


@route('model/remove')
def model_remove(data):
    mp = ModelProvider(ctx().write)
    m = mp.by_id(_id(data))
    s = config.get()
    proj = ProjectProvider(ctx().read).by_id(m.project)
    for suffix in ('.pth', '_weight.pth'):
        path = os.path.join(s.MODEL_FOLDER, proj.name if proj else '', m.name + suffix)
        if os.path.exists(path):
            os.remove(path)
    mp.remove(m.id)


@route('model/start_begin')
def model_start_begin(data):
    from mlcomp_amd.dag.model import model_start_begin as _begin
    return _begin(ctx().read, int(data['model_id']))


@route('model/start_end')
def model_start_end(data):
    from mlcomp_amd.dag.model import dag_model_start
    dag_model_start(ctx().write, data)


# ---------------------------------------------------------------------------- spaces / memory
@route('spaces')
def spaces(data):
    o = _opts(data, 'name')
    if o.sort_column == 'id':
        o.sort_column = 'name'
    return SpaceProvider(ctx().read).get(data, o)


def _space_fields(sp: Space, data: dict):
    content = data.get('content', '') or ''
    yaml_load(content)
    sp.name = data['name']
    sp.content = content
    sp.created = sp.created or now()
    sp.changed = now()
    return sp


@route('space/add')
def space_add(data):
    SpaceProvider(ctx().write).add(_space_fields(Space(), data))


@route('space/copy')
def space_copy(data):
    sp = SpaceProvider(ctx().write)
    new = _space_fields(Space(), data['space'])
    sp.add(new)
    for c in sp.related(data['old_space']):
        sp.add_relation(new.name, c.name)


@route('space/edit')
def space_edit(data):
    sp = SpaceProvider(ctx().write)
    _space_fields(sp.by_name(data['name']), data)
    sp.commit()


@route('space/remove')
def space_remove(data):
    sp = SpaceProvider(ctx().write)
    sp.query(Space).filter(Space.name == data['name']).delete(synchronize_session=False)
    sp.commit()


@route('space/relation_append')
def space_relation_append(data):
    SpaceProvider(ctx().write).add_relation(data['parent'], data['child'])


@route('space/relation_remove')
def space_relation_remove(data):
    SpaceProvider(ctx().write).remove_relation(data['parent'], data['child'])


@route('space/tag_add')
def space_tag_add(data):
    SpaceProvider(ctx().write).add_tag(data['space'], data['tag'])


@route('space/tag_remove')
def space_tag_remove(data):
    SpaceProvider(ctx().write).remove_tag(data['space'], data['tag'])


@route('space/tags')
def space_tags(data):
    sp = SpaceProvider(ctx().read)
    q = sp.query(SpaceTag.tag).distinct()
    if data.get('name'):
        q = q.filter(SpaceTag.tag.like(f"%{data['name']}%"))
    return {'data': [t[0] for t in q.limit(20)]}


@route('space/names')
def space_names(data):
    sp = SpaceProvider(ctx().read)
    q = sp.query(Space.name)
    if data.get('name'):
        q = q.filter(Space.name.like(f"%{data['name']}%"))
    return {'data': [t[0] for t in q.limit(20)]}


def _merge_lists(d: dict, d2: dict) -> dict:
    """Space merge: lists concatenate, dicts update, other type clashes are errors."""
    res = {}
    for k in set(d) | set(d2):
        if k in d and k in d2:
            a, b = d[k], d2[k]
            if isinstance(a, list) and isinstance(b, list):
                res[k] = a + b
            elif isinstance(a, dict) and isinstance(b, dict):
                res[k] = dict(a, **b)
            else:
                raise ValueError(f'Types are different: {type(a)}, {type(b)}')
        else:
            res[k] = d[k] if k in d else d2[k]
    return res


@route('space/run')
def space_run(data):
    """AND-spaces merge into one patch set; every OR-space (and its related spaces)
    yields one copied DAG (`app.py:503-560`)."""
    from mlcomp_amd.dag.copy import dag_copy
    sp = SpaceProvider(ctx().write)
    changes = yaml_load(data.get('file_changes') or '') or {}
    suffix = []
    for s in data['spaces']:
        if s['logic'] == 'and':
            space = sp.by_name(s['value'])
            if space.content:
                changes = _merge_lists(changes, yaml_load(space.content) or {})
                suffix.append(space.name)
    created = []
    for s in data['spaces']:
        if s['logic'] != 'or':
            continue
        space = sp.by_name(s['value'])
        rel = sp.related(space.name) + ([space] if space.content else [])
        for r in rel:
            d = _merge_lists(changes, yaml_load(r.content) or {})
            created.append(dag_copy(ctx().write, int(data['dag']), file_changes=yaml_dump(d),
                                    dag_suffix=' '.join(suffix + [r.name])))
    if not any(s['logic'] == 'or' for s in data['spaces']):
        created.append(dag_copy(ctx().write, int(data['dag']), file_changes=yaml_dump(changes),
                                dag_suffix=' '.join(suffix)))
    return {'dags': created}


@route('memories')
def memories(data):
    return MemoryProvider(ctx().read).get(data, _opts(data))


def _memory_fields(m: Memory, data: dict):
    m.model = data['model']
    m.memory = float(data['memory'])
    m.batch_size = int(data['batch_size'])
    m.variant = data.get('variant')
    m.num_classes = int(data['num_classes']) if data.get('num_classes') else None
    m.img_size = int(data['img_size']) if data.get('img_size') else None
    return m


@route('memory/add')
def memory_add(data):
    MemoryProvider(ctx().write).add(_memory_fields(Memory(), data))


@route('memory/edit')
def memory_edit(data):
    mp = MemoryProvider(ctx().write)
    _memory_fields(mp.by_id(int(data['id'])), data)
    mp.commit()


@route('memory/remove')
def memory_remove(data):
    MemoryProvider(ctx().write).remove(_id(data))


# ---------------------------------------------------------------------------- server
@route('stop')
def stop(data):
    return {}


@route('shutdown')
def shutdown(data):
    srv = getattr(ctx(), 'server', None)
    if srv is not None:
        srv.should_exit = True
    return {'message': 'Server shutting down...'}


def _supervisor():
    from mlcomp_amd.server.supervisor import SupervisorBuilder, get_supervisor
    sup = ctx().supervisor or get_supervisor()
    if sup is None:   # API used without the scheduler thread (tests, read-only site)
        sup = ctx().supervisor = SupervisorBuilder(session_key='api-supervisor')
    return sup


# ---------------------------------------------------------------------------- HTTP
def create_app():
    from fastapi import FastAPI, Request
    from fastapi.responses import FileResponse, HTMLResponse, JSONResponse, Response

    app = FastAPI(title='mlcomp_amd', docs_url=None, redoc_url=None)

    @app.post('/api/{name:path}')
    async def api(name: str, request: Request):
        body = await request.body()
        try:
            data = json.loads(body) if body else {}
        except ValueError:
            data = {}
        status, res = dispatch(name, data, request.headers.get('Authorization'))
        return JSONResponse(res, status_code=status)

    @app.get('/api/code_download')
    def code_download_get(id: int, request: Request):
        if str(request.headers.get('Authorization', '')).strip() != config.get().TOKEN:
            return JSONResponse({'success': False}, status_code=401)
        with ctx().lock:
            blob = _code_zip(id)
        return Response(blob, media_type='application/zip',
                        headers={'Content-Disposition': f'attachment; filename="{id}.zip"'})

    @app.get('/{path:path}')
    def static(path: str):
        p = os.path.join(STATIC, path)
        if path and os.path.isfile(p) and os.path.abspath(p).startswith(STATIC):
            return FileResponse(p)
        return HTMLResponse(open(os.path.join(STATIC, 'index.html')).read())

    return app


def start_server(host: str = None, port: int = None, scheduler: bool = True):
    import uvicorn
    s = config.get()
    c = ctx()
    c.logger.info(f'Server TOKEN = {s.TOKEN}', ComponentType.API)
    if scheduler:
        from mlcomp_amd.server.supervisor import register_supervisor
        c.supervisor = register_supervisor()
    cfg = uvicorn.Config(create_app(), host=host or s.WEB_HOST, port=int(port or s.WEB_PORT), log_level='warning')
    c.server = uvicorn.Server(cfg)
    c.server.run()


def stop_server(port: int = None):
    import requests
    s = config.get()
    requests.post(f'http://127.0.0.1:{port or s.WEB_PORT}/api/shutdown', headers={'Authorization': s.TOKEN},
                  timeout=10)


__all__ = ['ROUTES', 'dispatch', 'create_app', 'start_server', 'stop_server']
