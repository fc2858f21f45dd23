"""Web UI (`mlcomp_amd/server/static/`): the assets are served, every endpoint the pages
call exists in the API route table, the scripts parse, and the pure layout logic (DAG
layering, report `_other` series) behaves - under node when it is installed."""
import json
import os
import re
import shutil
import subprocess

import pytest

STATIC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'mlcomp_amd', 'server', 'static')
JS = ['core.js', 'pages.js']


def test_pages_only_call_existing_endpoints():
    from mlcomp_amd.server.api import ROUTES
    called = set()
    for f in JS:
        called |= set(re.findall(r"\bapi\('([\w/]+)'", open(os.path.join(STATIC, f)).read()))
    assert len(called) > 40
    missing = sorted(c for c in called if c not in ROUTES)
    assert not missing, missing
    # the reference UI's page groups are all there (app-routing.module.ts:12-67)
    pages = open(os.path.join(STATIC, 'pages.js')).read()
    for view in ('projects', 'computers', 'dags', 'dag', 'tasks', 'task', 'models', 'reports', 'report',
                 'skynet', 'logs', 'auxiliary'):
        assert f"App.register('{view}'" in pages, view


def test_assets_are_served(mlc_root):
    from fastapi.testclient import TestClient
    from mlcomp_amd.server.api import create_app
    c = TestClient(create_app())
    for path, needle in [('/', 'App.boot()'), ('/core.js', 'function layoutDag'), ('/pages.js', "App.register('report'"),
                         ('/app.css', '.st-success'), ('/dag/3', 'App.boot()')]:
        r = c.get(path)
        assert r.status_code == 200 and needle in r.text, path


NODE = shutil.which('node')


@pytest.mark.skipif(NODE is None, reason='node not installed')
def test_scripts_parse_and_layout_logic(tmp_path):
    for f in JS:
        subprocess.run([NODE, '--check', os.path.join(STATIC, f)], check=True)
    harness = tmp_path / 'h.js'
    harness.write_text("""
const vm = require('vm'), fs = require('fs');
const ctx = {console, setTimeout, clearTimeout, setInterval, clearInterval, URLSearchParams,
  localStorage: {getItem: () => null}, window: {addEventListener() {}}, location: {hash: ''}};
vm.createContext(ctx);
for (const f of ['core.js', 'pages.js']) vm.runInContext(fs.readFileSync(process.argv[2] + '/' + f, 'utf8'), ctx, {filename: f});
const out = vm.runInContext(`(() => {
  const nodes = [1, 2, 3, 4, 5].map(id => ({id}));
  const edges = [{from: 1, to: 2}, {from: 1, to: 3}, {from: 2, to: 4}, {from: 3, to: 4}, {from: 4, to: 5}, {from: 1, to: 5}];
  const L = layoutDag(nodes, edges);
  const layout = {items: {acc: {type: 'series', key: 'accuracy01'}}, layout: [
    {type: 'panel', items: [{type: 'table', source: ['loss']}, {type: 'series', source: 'acc'}, {type: 'series', source: '_other'}]}]};
  return {layer: L.layer, nlayers: L.layers.length, views: Object.keys(App.views).sort(),
          mapped: [...mappedSeries(layout, layout.layout, new Set())].sort(), nz: [nz(0, 5), nz(null, 5)]};
})()`, ctx);
console.log(JSON.stringify(out));
""")
    res = subprocess.run([NODE, str(harness), STATIC], check=True, capture_output=True, text=True)
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out['layer'] == {'1': 0, '2': 1, '3': 1, '4': 2, '5': 3}   # longest-path layering
    assert out['nlayers'] == 4
    assert out['mapped'] == ['accuracy01', 'loss']                   # _other = everything else
    assert out['nz'] == [0, 5]
    assert {'projects', 'dag', 'report', 'skynet', 'auxiliary'} <= set(out['views'])


def test_computers_endpoint_has_usage_history(mlc_root):
    import datetime
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.migrate import migrate
    from mlcomp_amd.db.models import Computer, ComputerUsage, now
    from mlcomp_amd.server import api
    migrate()
    s = Session.create_session(key='ui-test')
    s.add(Computer(name='n1', gpu=2, cpu=8, memory=1024))
    for i in range(5):
        s.add(ComputerUsage(computer='n1', time=now() - datetime.timedelta(minutes=5 - i), usage=json.dumps(
            {'cpu': 10.0 * i, 'memory': 20.0, 'disk': 30.0, 'gpu': [{'load': 50.0, 'memory': 10.0}, {'load': 5.0}]})))
    s.commit()
    api._CTX = None
    from mlcomp_amd import config
    status, body = api.dispatch('computers', {'usage_min_time': (now() - datetime.timedelta(minutes=3.5)).isoformat()},
                                config.get().TOKEN)
    assert status == 200, body
    h = body['data'][0]['usage_history']
    assert len(h['time']) == 3
    by = {m['name']: m['value'] for m in h['mean']}
    assert by['cpu'] == [20.0, 30.0, 40.0] and by['gpu_0'] == [50.0] * 3 and by['gpu_1'] == [5.0] * 3
    api._CTX = None


DOM_SHIM = r"""
class FakeNode {
  constructor(tag) { this.tag = tag; this.children = []; this.attrs = {}; this.style = {}; this.dataset = {};
    this.classList = {toggle() {}, add() {}, remove() {}, contains() { return false; }}; this.value = ''; this.textContent = ''; }
  append(...c) { for (const x of c) { if (x instanceof FakeNode) this.children.push(x); else { const t = new FakeNode('#text');
    t.textContent = String(x); this.children.push(t); } } }   // like the DOM: non-nodes become text
  prepend(...c) { this.children.unshift(...c); }
  setAttribute(k, v) { this.attrs[k] = v; } addEventListener() {} replaceChildren(...c) { this.children = c; }
  replaceWith() {} get childNodes() { return this.children; } querySelector() { return null; }
  querySelectorAll() { return []; } remove() {} focus() {} click() {} insertAdjacentHTML() {}
  text() { return this.tag === '#text' ? this.textContent : this.children.map(c => c.text ? c.text() : '').join(' '); }
}
"""


def _ui_fixture(tmp):
    """Real API answers for every endpoint the pages read, from a populated DB."""
    import datetime
    from mlcomp_amd import config
    from mlcomp_amd.dag.standard import dag_standard
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.migrate import migrate
    from mlcomp_amd.db.models import (Computer, ComputerUsage, Docker, Log, Memory, Model, Report, ReportImg,
                                      ReportSeries, ReportTasks, Space, Step, now)
    from mlcomp_amd.server import api
    migrate()
    s = Session.create_session(key='ui-fix')
    s.add(Computer(name='n1', gpu=2, cpu=8, memory=1024, usage=json.dumps(
        {'cpu': 10, 'memory': 20, 'disk': 30, 'gpu': [{'index': 0, 'load': 50, 'memory': 10}]})))
    s.add(Docker(name='default', computer='n1', last_activity=now(), ports='29500-29510'))
    s.add(ComputerUsage(computer='n1', time=now(), usage=json.dumps({'cpu': 1, 'memory': 2, 'disk': 3, 'gpu': [{'load': 4}]})))
    cfg = {'info': {'name': 'uidag', 'project': 'uiproj', 'layout': 'img-classify'},
           'executors': {'a': {'type': 'bash', 'command': 'true'}, 'b': {'type': 'bash', 'command': 'true', 'depends': 'a'}}}
    ids = dag_standard(s, cfg, upload_files=False, control_reqs=False)
    ta, tb = ids['a'][0], ids['b'][0]
    st = Step(task=ta, level=0, name='main', started=now(), index=0)
    s.add(st)
    s.commit()
    s.add(Log(message='hello', time=now(), level=20, component=2, task=ta, step=st.id))
    rep = s.query(Report).first()
    for e in range(3):
        for part in ('train', 'valid'):
            s.add(ReportSeries(task=ta, part=part, name='accuracy', epoch=e, value=0.5 + 0.1 * e, time=now(), stage='s1'))
            s.add(ReportSeries(task=ta, part=part, name='loss', epoch=e, value=1.0 - 0.1 * e, time=now(), stage='s1'))
    if rep is not None and not s.query(ReportTasks).filter(ReportTasks.task == ta).count():
        s.add(ReportTasks(report=rep.id, task=ta))
    s.add(ReportImg(group='img_classify', epoch=0, task=ta, dag=1, project=1, img=b'\xff\xd8', y=1, y_pred=0, score=0.3,
                    part='valid'))
    s.add(ReportImg(group='img_classify_confusion', epoch=0, task=ta, dag=1, project=1, img=b'[[3, 1], [2, 5]]',
                    part='valid'))
    s.add(Model(name='m1', project=1, created=now()))
    s.add(Memory(model='resnet50', batch_size=256, memory=60.0))
    s.add(Space(name='sp1', content='a: 1', created=now(), changed=now()))
    s.commit()
    api._CTX = None
    tok = config.get().TOKEN
    calls = {'projects': {}, 'dags': {}, 'graph': 1, 'config': 1, 'code': 1, 'tasks': {}, 'task/info': ta,
             'task/steps': ta, 'logs': {}, 'computers': {}, 'computer_sync_start': {}, 'reports': {},
             'report': rep.id if rep else 1, 'img_classify': {'group': 'img_classify'},
             'img_segment': {}, 'models': {}, 'memories': {}, 'spaces': {}, 'auxiliary': {}, 'layouts': {},
             'report/add_start': {}, 'report/update_layout_start': rep.id if rep else 1}
    out = {}
    for name, body in calls.items():
        status, res = api.dispatch(name, body, tok)
        assert status == 200, (name, res)
        out[name] = res
    conf = api.dispatch('img_classify', {'group': 'img_classify_confusion'}, tok)[1]
    api._CTX = None
    return out, conf, ta


@pytest.mark.skipif(NODE is None, reason='node not installed')
def test_every_page_renders_real_api_payloads(mlc_root, tmp_path):
    """Each view renders the real API answers without throwing (a DOM shim under node)."""
    fix, conf, ta = _ui_fixture(tmp_path)
    (tmp_path / 'fix.json').write_text(json.dumps({'fix': fix, 'conf': conf}))
    harness = tmp_path / 'pages.js'
    harness.write_text(DOM_SHIM + """
const vm = require('vm'), fs = require('fs');
const F = JSON.parse(fs.readFileSync(process.argv[3], 'utf8'));
const errors = [];
const doc = {createElement: t => new FakeNode(t), createElementNS: (ns, t) => new FakeNode(t),
  createTextNode: s => { const n = new FakeNode('#text'); n.textContent = s; return n; },
  getElementById: id => doc.ids[id] || (doc.ids[id] = new FakeNode('div')), ids: {},
  querySelectorAll: () => [], querySelector: () => null, body: new FakeNode('body'), hidden: false};
const ctx = {console: {log: console.log, error: (...a) => errors.push(a.map(String).join(' '))}, setTimeout, clearTimeout,
  setInterval: () => 0, clearInterval() {}, URLSearchParams, Node: FakeNode, Element: FakeNode, document: doc, atob: s => Buffer.from(s, 'base64').toString('binary'),
  localStorage: {getItem: () => 'tok'}, window: {addEventListener() {}}, location: {hash: ''}};
vm.createContext(ctx);
for (const f of ['core.js', 'pages.js']) vm.runInContext(fs.readFileSync(process.argv[2] + '/' + f, 'utf8'), ctx, {filename: f});
ctx.FIX = F;
vm.runInContext(`api = async (name, body) => {
  if (name === 'img_classify' && body && String(body.group).endsWith('_confusion')) return FIX.conf;
  if (!(name in FIX.fix)) throw new Error('no fixture for ' + name);
  return FIX.fix[name];
};`, ctx);
const hashes = ['#/projects', '#/computers', '#/dags', '#/dag/1', '#/dag/1/tasks', '#/dag/1/config', '#/dag/1/code',
  '#/tasks', '#/task/' + process.argv[4], '#/logs', '#/models', '#/reports', '#/report/' + (F.fix.report.id || 1),
  '#/reports/layouts', '#/skynet', '#/skynet/memory', '#/auxiliary'];
(async () => {
  const sizes = {};
  for (const h of hashes) {
    ctx.location.hash = h;
    await vm.runInContext('App.render()', ctx);
    const main = doc.ids.main;
    const txt = main.text();
    if (/^\\s*loading/.test(txt) || (main.children[0] && main.children[0].attrs && main.children[0].attrs.class === 'err')
        || /\\bnull\\b|\\[object /.test(txt))
      errors.push(h + ': ' + txt.slice(0, 300));
    sizes[h] = txt.length;
  }
  console.log(JSON.stringify({errors, sizes}));
})();
""")
    res = subprocess.run([NODE, '--unhandled-rejections=strict', str(harness), STATIC, str(tmp_path / 'fix.json'), str(ta)],
                         capture_output=True,
                         text=True, timeout=60)
    assert res.returncode == 0, res.stderr
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert not out['errors'], out['errors']
    assert all(n > 20 for n in out['sizes'].values()), out['sizes']
