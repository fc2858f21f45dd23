// mlcomp_amd UI pages (the reference Angular app's routes, `app-routing.module.ts:12-67`):
// projects, computers (usage gauges + history, sync), dags (list, detail: graph / config /
// code viewer-editor / tasks), tasks (list, detail: info, step tree, logs, rank tasks),
// models (add / start), reports (list, layout renderer: panel / table / series / _other /
// img_classify with confusion matrix / img_segment / img; layouts editor), skynet
// (memory table, spaces), logs and the scheduler snapshot (auxiliary).
'use strict';

// ================================================================== projects
App.register('projects', {
  async render(m, args, q, st) {
    st.p = st.p || {page: 0, size: 50, col: 'id', desc: true};
    const r = await api('projects', {paginator: pag(st.p.page, st.p.size, st.p.col, st.p.desc), name: st.name || ''});
    const rerender = () => App.render(true);
    m.append(el('h2', {}, 'Projects'),
      el('div', {class: 'toolbar'},
        el('input', {placeholder: 'name filter', value: st.name || '', onchange: e => { st.name = e.target.value; rerender(); }}),
        el('button', {class: 'primary', onclick: () => projectDialog()}, 'Add project')),
      grid(r.data, [
        {title: 'id', sort: 'id', render: p => p.id},
        {title: 'name', sort: 'name', render: p => el('a', {href: `#/dags?project=${p.id}`}, p.name)},
        {title: 'dags', render: p => nz(p.dag_count, '')},
        {title: 'last activity', render: p => fmt.time(p.last_activity)},
        {title: 'sync folders', render: p => p.sync_folders || ''},
        {title: 'ignore folders', render: p => p.ignore_folders || ''},
        {title: '', render: p => el('span', {},
          el('button', {class: 'small', onclick: () => projectDialog(p)}, 'edit'), ' ',
          el('button', {class: 'small', onclick: () => confirmDo(`Stop every DAG of ${p.name}?`, () => api('project/stop_all_dags', {project: p.id}))}, 'stop dags'), ' ',
          el('button', {class: 'small danger', onclick: () => confirmDo(`Remove every DAG of ${p.name}?`, () => api('project/remove_all_dags', {project: p.id}))}, 'remove dags'), ' ',
          el('button', {class: 'small danger', onclick: () => confirmDo(`Remove project ${p.name}?`, () => api('project/remove', {id: p.id}).then(rerender))}, 'remove'))},
      ], {state: st.p, onChange: rerender, onClick: p => App.go(`#/dags?project=${p.id}`)}),
      pager(r.total, st.p, rerender));
  },
}, 'Projects');

function projectDialog(p) {
  const f = form([
    {name: 'name', value: p ? p.name : ''},
    {name: 'class_names', label: 'class names (YAML)', type: 'textarea', rows: 4, value: p ? (p.class_names || '') : ''},
    {name: 'sync_folders', label: 'sync folders', value: p ? (p.sync_folders || '') : ''},
    {name: 'ignore_folders', label: 'ignore folders', value: p ? (p.ignore_folders || '') : ''},
  ]);
  dialog(p ? `Edit project ${p.name}` : 'Add project', f, [{label: 'Cancel'}, {label: 'Save', cls: 'primary', action: async () => {
    const v = f.values();
    if (p) await api('project/edit', {id: p.id, new_name: v.name !== p.name ? v.name : undefined, class_names: v.class_names,
      sync_folders: v.sync_folders, ignore_folders: v.ignore_folders});
    else await api('project/add', v);
    App.render(true);
  }}]);
}

// ================================================================== computers
App.register('computers', {
  async render(m, args, q, st) {
    st.window = st.window || 60;
    const since = new Date(Date.now() - st.window * 60000).toISOString().slice(0, 19);
    const r = await api('computers', {usage_min_time: since});
    m.append(el('h2', {}, 'Computers'), el('div', {class: 'toolbar'},
      el('label', {}, 'usage history'),
      el('select', {onchange: e => { st.window = +e.target.value; App.render(true); }},
        [[30, '30 min'], [60, '1 hour'], [360, '6 hours'], [1440, '1 day']].map(([v, t]) => el('option', {value: v, selected: v === st.window}, t))),
      el('button', {onclick: () => syncDialog()}, 'Sync data…')));
    const cards = el('div', {class: 'cards'});
    for (const c of r.data) {
      const u = c.usage || {};
      const alive = (c.dockers || []).map(d => {
        const age = (Date.now() - Date.parse(d.last_activity + (String(d.last_activity).endsWith('Z') ? '' : 'Z'))) / 1000;
        return el('span', {class: 'tag', style: {background: age < 15 ? '#d9f2e3' : '#fde2e1'}}, `${d.name} ${age < 15 ? 'alive' : 'silent ' + fmt.time(d.last_activity)} ports ${d.ports}`);
      });
      const gpus = (u.gpu || []).map(g => el('tr', {},
        el('td', {}, 'GPU ' + (nz(g.index, ''))), el('td', {style: {width: '35%'}}, loadBar(g.load)), el('td', {class: 'muted'}, fmt.num(g.load, 0) + '% load'),
        el('td', {style: {width: '35%'}}, loadBar(g.memory)), el('td', {class: 'muted'}, fmt.num(g.memory, 0) + '% mem' + (g.power ? ` ${g.power.toFixed(0)} W` : ''))));
      const h = c.usage_history || {time: [], mean: []};
      const series = (h.mean || []).map(s => ({label: s.name, x: h.time, y: s.value}));
      cards.append(el('div', {class: 'card'},
        el('h3', {style: {marginTop: 0}}, c.name, ' ', el('span', {class: 'muted'}, `${c.gpu} GPU · ${c.cpu} CPU · ${fmt.gb(c.memory)} · ${c.ip || ''}`)),
        el('div', {}, alive),
        el('div', {class: 'gauges'}, gauge(u.cpu, 'CPU'), gauge(u.memory, 'memory'), gauge(u.disk, 'disk')),
        gpus.length ? el('table', {class: 'grid'}, gpus) : null,
        lineChart(series, {title: 'usage history (mean %)', width: 490, height: 170, yMin: 0, yMax: 100}),
        c.meta && c.meta.manual_sync ? el('div', {class: 'muted'}, 'pending manual sync: ' + JSON.stringify(c.meta.manual_sync)) : null));
    }
    m.append(cards);
  },
}, 'Computers');

async function syncDialog() {
  const r = await api('computer_sync_start', {});
  const f = form([
    {name: 'id', label: 'project', type: 'select', options: r.data.map(p => [p.id, p.name])},
    {name: 'computer', type: 'select', options: [['', '(all)']].concat(r.computers.map(c => [c, c]))},
    {name: 'sync_folders', label: 'sync folders (YAML list)', type: 'textarea', rows: 3, value: (r.data[0] || {}).sync_folders || ''},
    {name: 'ignore_folders', label: 'ignore folders (YAML list)', type: 'textarea', rows: 3, value: (r.data[0] || {}).ignore_folders || ''},
  ]);
  dialog('Synchronise project folders', f, [{label: 'Cancel'}, {label: 'Sync', cls: 'primary', action: async () => {
    const v = f.values(); v.id = +v.id; await api('computer_sync_end', v); toast('sync scheduled');
  }}]);
}

// ================================================================== dags
App.register('dags', {
  async render(m, args, q, st) {
    st.p = st.p || {page: 0, size: 50, col: 'id', desc: true};
    const filt = {paginator: pag(st.p.page, st.p.size, st.p.col, st.p.desc), project: q.project ? +q.project : undefined,
      name: st.name || '', tags: st.tag ? [st.tag] : undefined};
    const r = await api('dags', filt);
    const rerender = () => App.render(true);
    m.append(el('h2', {}, 'DAGs', q.project ? el('span', {class: 'muted'}, ` · project ${q.project} `) : '', q.project ? el('a', {href: '#/dags'}, '(all)') : ''),
      el('div', {class: 'toolbar'},
        el('input', {placeholder: 'name filter', value: st.name || '', onchange: e => { st.name = e.target.value; rerender(); }}),
        el('input', {placeholder: 'tag', value: st.tag || '', onchange: e => { st.tag = e.target.value; rerender(); }})),
      grid(r.data, [
        {title: 'id', sort: 'id', render: d => d.id},
        {title: 'name', sort: 'name', render: d => el('a', {href: `#/dag/${d.id}`}, d.name)},
        {title: 'project', render: d => d.project ? d.project.name : ''},
        {title: 'type', render: d => d.type},
        {title: 'tasks', render: d => statusCounts(d.task_statuses)},
        {title: 'created', sort: 'created', render: d => fmt.time(d.created)},
        {title: 'last activity', render: d => fmt.time(d.last_activity)},
        {title: 'tags', render: d => el('span', {}, (d.tags || []).map(t => el('span', {class: 'tag'}, t,
          el('a', {onclick: () => api('dag/tag_remove', {dag: d.id, tag: t}).then(rerender)}, '×'))),
          el('a', {onclick: () => promptText('Add tag', '', tag => api('dag/tag_add', {dag: d.id, tag}).then(rerender))}, '+tag'))},
        {title: '', render: d => dagButtons(d, rerender)},
      ], {state: st.p, onChange: rerender, onClick: d => App.go(`#/dag/${d.id}`)}),
      pager(r.total, st.p, rerender));
  },
}, 'DAGs');

function dagButtons(d, after) {
  return el('span', {},
    el('button', {class: 'small', onclick: () => api('dag/stop', {id: d.id}).then(after)}, 'stop'), ' ',
    el('button', {class: 'small', onclick: () => api('dag/start', {id: d.id}).then(after)}, 'start'), ' ',
    el('button', {class: 'small', onclick: () => restartDialog(d)}, 'restart…'), ' ',
    el('button', {class: 'small danger', onclick: () => confirmDo(`Remove DAG ${d.id} ${d.name}?`, () => api('dag/remove', {id: d.id}).then(after))}, 'remove'));
}

function restartDialog(d) {
  const f = form([{name: 'file_changes', label: 'file changes (YAML: path regex -> patch)', type: 'textarea', rows: 10, value: ''}]);
  dialog(`Restart DAG ${d.id} as a copy`, f, [{label: 'Cancel'}, {label: 'Restart', cls: 'primary', action: async () => {
    const res = await api('dag/restart', {dag: d.id, file_changes: f.values().file_changes});
    toast('created DAG ' + JSON.stringify(res.dag));
    App.render(true);
  }}]);
}

function promptText(title, value, fn) {
  const i = el('input', {value, style: {width: '100%'}});
  dialog(title, i, [{label: 'Cancel'}, {label: 'OK', cls: 'primary', action: () => fn(i.value)}]);
  setTimeout(() => i.focus(), 0);
}

App.register('dag', {
  nav: 'dags',
  static: args => args[1] === 'code',
  async render(m, args, q, st) {
    const id = +args[0], tab = args[1] || 'graph';
    const info = (await api('dags', {id, paginator: pag(0, 1)})).data[0];
    if (!info) { m.append(el('div', {class: 'err'}, `DAG ${id} not found`)); return; }
    m.append(el('h2', {}, `DAG ${id} · ${info.name} `, el('span', {class: 'muted'}, info.project ? info.project.name : ''), ' ', statusCounts(info.task_statuses)),
      el('div', {class: 'toolbar'}, dagButtons(info, () => App.render(true)),
        el('button', {class: 'small', onclick: () => apiDownload(`/api/code_download?id=${id}`, `${id}.zip`)}, 'download code')),
      el('div', {class: 'tabs'}, ['graph', 'tasks', 'config', 'code'].map(t => el('a', {class: t === tab ? 'on' : null, href: `#/dag/${id}/${t}`}, t))));
    if (tab === 'graph') {
      const g = await api('graph', id);
      m.append(dagGraph(g, n => App.go(`#/task/${n.id}`)),
        el('div', {class: 'muted', style: {marginTop: '6px'}}, Object.entries(STATUS_COLORS).map(([k, c]) => el('span', {class: 'tag', style: {background: c, color: '#fff'}}, k))));
    } else if (tab === 'config') {
      const c = await api('config', id);
      m.append(el('pre', {class: 'code'}, c.data || ''));
    } else if (tab === 'tasks') {
      await taskTable(m, {dag: id}, st);
    } else if (tab === 'code') {
      await codeView(m, id, st);           // an editor: not refreshed in the background
    }
  },
});

async function codeView(m, dag, st) {
  const r = await api('code', dag);
  st.open = st.open || new Set();
  const pane = el('div');
  const show = n => {
    if (n.children) return;
    st.file = n;
    const ta = el('textarea', {rows: 32, spellcheck: 'false'}, n.content || '');
    pane.replaceChildren(el('div', {class: 'toolbar'}, el('b', {}, n.name),
      el('button', {class: 'primary small', onclick: async () => {
        const res = await api('update_code', {file_id: n.id, dag, storage: n.storage, content: ta.value});
        n.content = ta.value; n.id = res.file; toast('saved (file ' + res.file + ')');
      }}, 'save')), ta);
  };
  const t = tree(r.items, n => n.name, show, {open: st.open, key: n => n.storage});
  m.append(el('div', {class: 'split'}, t, pane));
  if (st.file) show(st.file); else pane.append(el('div', {class: 'muted'}, 'select a file'));
}

// ================================================================== tasks
async function taskTable(m, filter, st) {
  st.p = st.p || {page: 0, size: 50, col: 'id', desc: true};
  st.status = st.status || {};
  const rerender = () => App.render(true);
  const r = await api('tasks', Object.assign({paginator: pag(st.p.page, st.p.size, st.p.col, st.p.desc), status: st.status,
    name: st.name || ''}, filter));
  m.append(el('div', {class: 'toolbar'},
    el('input', {placeholder: 'name filter', value: st.name || '', onchange: e => { st.name = e.target.value; rerender(); }}),
    STATUSES.map(s => el('label', {}, el('input', {type: 'checkbox', checked: !!st.status[s], onchange: e => { st.status[s] = e.target.checked; rerender(); }}), ' ', s.replace('_', ' ')))),
  grid(r.data, [
    {title: 'id', sort: 'id', render: t => t.id},
    {title: 'name', sort: 'name', render: t => el('a', {href: `#/task/${t.id}`}, t.name)},
    {title: 'dag', render: t => t.dag_rel ? el('a', {href: `#/dag/${t.dag}`}, `${t.dag} ${t.dag_rel.name}`) : t.dag},
    {title: 'status', sort: 'status', render: t => statusBadge(t.status)},
    {title: 'executor', render: t => t.executor},
    {title: 'computer / gpu', render: t => [t.computer_assigned || '', t.gpu_assigned ? ` [${t.gpu_assigned}]` : '']},
    {title: 'progress', render: t => [progressBar(t.batch_index, t.batch_total), t.loader_name ? el('span', {class: 'muted'}, ' ' + t.loader_name) : '']},
    {title: 'step', render: t => t.current_step || ''},
    {title: 'duration', render: t => t.duration || ''},
    {title: 'score', sort: 'score', render: t => fmt.num(t.score)},
    {title: 'loss', render: t => fmt.num(t.loss)},
    {title: '', render: t => el('button', {class: 'small', onclick: () => api('task/stop', {id: t.id}).then(rerender)}, 'stop')},
  ], {state: st.p, onChange: rerender, onClick: t => App.go(`#/task/${t.id}`)}),
  pager(r.total, st.p, rerender));
}

App.register('tasks', {
  async render(m, args, q, st) {
    m.append(el('h2', {}, 'Tasks'));
    await taskTable(m, {dag: q.dag ? +q.dag : undefined, project: q.project ? +q.project : undefined}, st);
  },
}, 'Tasks');

App.register('task', {
  nav: 'tasks',
  async render(m, args, q, st) {
    const id = +args[0];
    const t = (await api('tasks', {id, paginator: pag(0, 1), type: ['User', 'Train', 'Service']})).data[0];
    if (!t) { m.append(el('div', {class: 'err'}, `task ${id} not found`)); return; }
    const info = await api('task/info', id);
    const steps = await api('task/steps', id);
    st.levels = st.levels || {debug: false, info: true, warning: true, error: true};
    const logs = await api('logs', {task: id, step: st.step || undefined, levels: LEVELS.filter(l => st.levels[l]), paginator: pag(0, 300)});
    const kids = (await api('tasks', {parent: id, paginator: pag(0, 64, 'id', false), type: ['User', 'Train', 'Service']})).data;
    m.append(el('h2', {}, `Task ${id} · ${t.name} `, statusBadge(t.status), ' ',
      el('button', {class: 'small', onclick: () => api('task/stop', {id}).then(() => App.render(true))}, 'stop')),
      el('div', {class: 'cards'},
        el('div', {class: 'card'}, kvTable({dag: el('a', {href: `#/dag/${t.dag}`}, `${t.dag} ${t.dag_rel ? t.dag_rel.name : ''}`),
          executor: t.executor, computer: t.computer_assigned, gpu: info.gpu_assigned, pid: info.pid, worker: info.worker_index,
          started: fmt.time(t.started), finished: fmt.time(t.finished), duration: t.duration, step: t.current_step,
          progress: progressBar(t.batch_index, t.batch_total), score: fmt.num(t.score), loss: fmt.num(t.loss)})),
        el('div', {class: 'card'}, el('h3', {style: {marginTop: 0}}, 'steps'),
          tree(steps.data || steps, s => [s.name, ' ', el('span', {class: 'muted'}, fmt.time(s.started)), ' ',
            ...(s.log_statuses || []).filter(x => x.count).map(x => el('span', {class: 'lvl-' + x.name}, ` ${x.name}:${x.count}`))],
          s => { st.step = st.step === s.id ? null : s.id; App.render(true); }, {cls: 'steps', expandAll: true, selected: st.step}))),
      kids.length ? [el('h3', {}, 'rank / child tasks'), grid(kids, [
        {title: 'id', render: k => el('a', {href: `#/task/${k.id}`}, k.id)},
        {title: 'status', render: k => statusBadge(k.status)},
        {title: 'computer / gpu', render: k => `${k.computer_assigned || ''} [${k.gpu_assigned || ''}]`},
        {title: 'progress', render: k => progressBar(k.batch_index, k.batch_total)},
        {title: 'duration', render: k => k.duration || ''}])] : null,
      el('h3', {}, 'additional info'), el('pre', {class: 'plain'}, info.additional_info || ''),
      info.result ? [el('h3', {}, 'result'), el('pre', {class: 'plain'}, info.result)] : null,
      el('h3', {}, 'logs', st.step ? el('span', {class: 'muted'}, ` (step ${st.step})`) : ''),
      el('div', {class: 'toolbar'}, LEVELS.map(l => el('label', {}, el('input', {type: 'checkbox', checked: !!st.levels[l],
        onchange: e => { st.levels[l] = e.target.checked; App.render(true); }}), ' ', l))),
      logTable(logs.data));
  },
});

function logTable(rows) {
  return grid(rows, [
    {title: 'time', render: l => fmt.time(l.time)},
    {title: 'level', render: l => el('span', {class: 'lvl-' + l.level}, l.level)},
    {title: 'component', render: l => nz(COMPONENTS[l.component], l.component)},
    {title: 'computer', render: l => l.computer || ''},
    {title: 'task', render: l => l.task ? el('a', {href: `#/task/${l.task}`}, l.task) : ''},
    {title: 'step', render: l => l.step_name || ''},
    {title: 'message', render: l => el('pre', {class: 'plain', style: {maxHeight: '140px', border: 0, padding: 0}}, l.message)},
  ]);
}

// ================================================================== logs
App.register('logs', {
  async render(m, args, q, st) {
    st.p = st.p || {page: 0, size: 100, col: 'id', desc: true};
    st.levels = st.levels || {debug: false, info: true, warning: true, error: true};
    st.comps = st.comps || {};
    const rerender = () => App.render(true);
    const comps = COMPONENTS.map((c, i) => i).filter(i => st.comps[i]);
    const r = await api('logs', {paginator: pag(st.p.page, st.p.size), levels: LEVELS.filter(l => st.levels[l]),
      components: comps.length ? comps : undefined, computer: st.computer || undefined, message: st.message || undefined,
      task: st.task ? +st.task : undefined});
    m.append(el('h2', {}, 'Logs'), el('div', {class: 'toolbar'},
      LEVELS.map(l => el('label', {}, el('input', {type: 'checkbox', checked: !!st.levels[l], onchange: e => { st.levels[l] = e.target.checked; rerender(); }}), ' ', l)),
      ' | ', COMPONENTS.map((c, i) => el('label', {}, el('input', {type: 'checkbox', checked: !!st.comps[i], onchange: e => { st.comps[i] = e.target.checked; rerender(); }}), ' ', c)),
      el('input', {placeholder: 'computer', value: st.computer || '', onchange: e => { st.computer = e.target.value; rerender(); }}),
      el('input', {placeholder: 'task id', value: st.task || '', size: 7, onchange: e => { st.task = e.target.value; rerender(); }}),
      el('input', {placeholder: 'message contains', value: st.message || '', onchange: e => { st.message = e.target.value; rerender(); }})),
    logTable(r.data), pager(r.total, st.p, rerender));
  },
}, 'Logs');

// ================================================================== models
App.register('models', {
  async render(m, args, q, st) {
    st.p = st.p || {page: 0, size: 50, col: 'id', desc: true};
    const rerender = () => App.render(true);
    const r = await api('models', {paginator: pag(st.p.page, st.p.size), name: st.name || '', project: q.project ? +q.project : undefined});
    m.append(el('h2', {}, 'Models'), el('div', {class: 'toolbar'},
      el('input', {placeholder: 'name filter', value: st.name || '', onchange: e => { st.name = e.target.value; rerender(); }}),
      el('button', {class: 'primary', onclick: () => modelAddDialog()}, 'Add model')),
    grid(r.data, [
      {title: 'id', render: x => x.id},
      {title: 'name', render: x => x.name},
      {title: 'project', render: x => x.project ? x.project.name : ''},
      {title: 'dag', render: x => x.dag ? el('a', {href: `#/dag/${x.dag}`}, x.dag) : ''},
      {title: 'fold', render: x => nz(x.fold, '')},
      {title: 'score local', render: x => fmt.num(x.score_local)},
      {title: 'score public', render: x => fmt.num(x.score_public)},
      {title: 'created', render: x => fmt.time(x.created)},
      {title: '', render: x => el('span', {},
        el('button', {class: 'small', onclick: () => modelStartDialog(x)}, 'start…'), ' ',
        el('button', {class: 'small danger', onclick: () => confirmDo(`Remove model ${x.name} (and its files)?`, () => api('model/remove', {id: x.id}).then(rerender))}, 'remove'))},
    ]), pager(r.total, st.p, rerender));
  },
}, 'Models');

async function modelAddDialog() {
  const projects = (await api('projects', {paginator: pag(0, 500)})).data;
  const f = form([
    {name: 'name'},
    {name: 'project', type: 'select', options: projects.map(p => [p.id, p.name])},
    {name: 'task', label: 'train task id (empty: register only)', type: 'number'},
    {name: 'file', label: 'checkpoint', type: 'select', options: ['best', 'last']},
    {name: 'fold', type: 'number', value: 0},
    {name: 'equations', label: 'equations (YAML)', type: 'textarea', rows: 4},
  ]);
  dialog('Add model', f, [{label: 'Cancel'}, {label: 'Add', cls: 'primary', action: async () => {
    const v = f.values(); v.project = +v.project; if (!v.task) delete v.task;
    await api('model/add', v); toast('model add scheduled'); App.render(true);
  }}]);
}

async function modelStartDialog(model) {
  const r = await api('model/start_begin', {model_id: model.id});
  if (!r.dags.length) { dialog('Start model', el('p', {}, 'the project has no Pipe DAGs (info.type: pipe)')); return; }
  const dagSel = el('select', {}, r.dags.map(d => el('option', {value: d.id, selected: r.dag && r.dag.id === d.id}, `${d.id} ${d.name}`)));
  const pipeSel = el('select'), verSel = el('select'), eq = el('textarea', {rows: 6});
  const cur = () => r.dags.find(d => d.id === +dagSel.value);
  const pipe = () => (cur().pipes || []).find(p => p.name === pipeSel.value);
  const fillVer = () => {
    const p = pipe();
    verSel.replaceChildren(el('option', {value: ''}, '(new version)'), ...(p ? p.versions : []).map(v => el('option', {value: v.name}, v.name)));
    eq.value = '';
  };
  const fillPipe = () => { pipeSel.replaceChildren(...(cur().pipes || []).map(p => el('option', {value: p.name}, p.name))); fillVer(); };
  dagSel.onchange = fillPipe; pipeSel.onchange = fillVer;
  verSel.onchange = () => { const v = (pipe().versions || []).find(x => x.name === verSel.value); eq.value = v ? (v.equations || '') : ''; };
  fillPipe();
  const name = el('input', {placeholder: 'version name'});
  dialog(`Start model ${model.name}`, el('div', {class: 'form'},
    el('label', {}, 'pipe DAG'), dagSel, el('label', {}, 'pipe'), pipeSel, el('label', {}, 'version'), verSel,
    el('label', {}, 'new version name'), name, el('label', {}, 'equations (YAML)'), eq),
  [{label: 'Cancel'}, {label: 'Start', cls: 'primary', action: async () => {
    const p = pipe();
    const versions = (p.versions || []).slice();
    let vname = verSel.value || name.value || ('v' + (versions.length + 1));
    if (!verSel.value) versions.push({name: vname, equations: eq.value});
    await api('model/start_end', {model_id: model.id, dag: +dagSel.value,
      pipe: {name: p.name, versions, version: {name: vname, equations: eq.value}}});
    toast('pipe started'); App.render(true);
  }}]);
}

// ================================================================== reports
App.register('reports', {
  static: args => args[0] === 'layouts',
  async render(m, args, q, st) {
    if (args[0] === 'layouts') return layoutsView(m, st);
    st.p = st.p || {page: 0, size: 50, col: 'id', desc: true};
    const rerender = () => App.render(true);
    const r = await api('reports', {paginator: pag(st.p.page, st.p.size), project: q.project ? +q.project : undefined});
    m.append(el('h2', {}, 'Reports'), el('div', {class: 'toolbar'},
      el('button', {class: 'primary', onclick: () => reportAddDialog()}, 'Add report'),
      el('a', {href: '#/reports/layouts'}, 'layouts')),
    grid(r.data, [
      {title: 'id', render: x => x.id},
      {title: 'name', render: x => el('a', {href: `#/report/${x.id}`}, x.name)},
      {title: 'project', render: x => x.project ? x.project.name : ''},
      {title: 'layout', render: x => x.layout},
      {title: 'tasks', render: x => x.tasks},
      {title: 'time', render: x => fmt.time(x.time)},
    ], {onClick: x => App.go(`#/report/${x.id}`)}), pager(r.total, st.p, rerender));
  },
}, 'Reports');

async function reportAddDialog() {
  const r = await api('report/add_start', {});
  const f = form([{name: 'name'}, {name: 'project', type: 'select', options: r.projects.map(p => [p.id, p.name])},
    {name: 'layout', type: 'select', options: r.layouts.map(l => l.name)}]);
  dialog('Add report', f, [{label: 'Cancel'}, {label: 'Add', cls: 'primary', action: async () => {
    const v = f.values(); v.project = +v.project; await api('report/add_end', v); App.render(true);
  }}]);
}

// ---------------------------------------------------------------- report layout renderer
// data: {series name: [{task, task_name, part, stage, x, y}]}; layout components:
// panel / table / series / img / img_classify / img_segment / blank; series source
// "_other" = every series no other series component of the layout shows
function layoutKey(layout, source) {
  const it = (layout.items || {})[source];
  return it && it.key ? it.key : source;
}

function mappedSeries(layout, comps, out) {
  for (const c of comps || []) {
    if (c.type === 'panel') mappedSeries(layout, c.items, out);
    else if (c.type === 'series' && c.source !== '_other') out.add(layoutKey(layout, c.source));
    else if (c.type === 'table') (Array.isArray(c.source) ? c.source : [c.source]).forEach(s => out.add(layoutKey(layout, s)));
  }
  return out;
}

function seriesCharts(name, list, multi, height) {
  const label = s => `${s.task_name || ''}#${s.task} ${s.part || ''}${s.stage ? ' ' + s.stage : ''}`;
  if (multi || new Set(list.map(s => s.task)).size <= 1)
    return [lineChart(list.map(s => ({label: label(s), x: s.x, y: s.y})), {title: name, height})];
  const byTask = {};
  list.forEach(s => { (byTask[s.task] = byTask[s.task] || []).push(s); });
  return Object.values(byTask).map(l => lineChart(l.map(s => ({label: label(s), x: s.x, y: s.y})), {title: `${name} · ${l[0].task_name || ''}#${l[0].task}`, height}));
}

function metricTable(report, data, sources, layout) {
  const names = (Array.isArray(sources) ? sources : [sources]).map(s => layoutKey(layout, s));
  const val = (task, name) => {
    const l = (data[name] || []).filter(s => s.task === task.id);
    const pick = l.find(s => s.part === 'valid') || l[0];
    return pick && pick.y.length ? pick.y[pick.y.length - 1] : null;
  };
  return grid(report.tasks, [{title: 'task', render: t => el('a', {href: `#/task/${t.id}`}, `${t.id} ${t.name}`)},
    {title: 'status', render: t => statusBadge(t.status)}, {title: 'score', render: t => fmt.num(t.score)},
    ...names.map(n => ({title: n, render: t => fmt.num(val(t, n))}))]);
}

async function imagesFor(kind, report, group, st, extra) {
  const out = [];
  for (const t of report.tasks) {
    const r = await api(kind, Object.assign({task: t.id, group, paginator: pag(st.page || 0, 24, 'id', false)}, extra || {}));
    out.push(...r.data.map(x => Object.assign(x, {task_name: t.name})));
  }
  return out;
}

function imgFigure(x, caption) {
  return el('figure', {}, x.content ? el('img', {src: 'data:image/jpeg;base64,' + x.content}) : el('div', {class: 'muted'}, 'no image'),
    el('figcaption', {}, caption));
}

async function imgClassify(report, comp, st) {
  const key = 'ic_' + comp.source;
  const s = st[key] = st[key] || {page: 0};
  const box = el('div', {class: 'card'}, el('h3', {style: {marginTop: 0}}, comp.source));
  // confusion matrix: ReportImg group "<source>_confusion", JSON bytes
  const cms = await imagesFor('img_classify', report, comp.source + '_confusion', {page: 0});
  for (const cm of cms) {
    let mat = null;
    try { mat = JSON.parse(atob(cm.content)); } catch (e) { /* not a matrix */ }
    if (!Array.isArray(mat)) continue;
    const mx = Math.max(1, ...mat.flat());
    box.append(el('div', {class: 'muted'}, `confusion matrix · task ${cm.task} (rows: y, columns: y_pred; click a cell to filter)`),
      el('table', {class: 'cm'}, el('tr', {}, el('th', {}, ''), mat[0].map((_, j) => el('th', {}, j))),
        mat.map((row, i) => el('tr', {}, el('th', {}, i), row.map((v, j) => el('td', {
          style: {background: `rgba(29,95,191,${0.08 + 0.92 * v / mx})`, color: v / mx > 0.5 ? '#fff' : '#1f2933'},
          title: `y=${i} y_pred=${j}: ${v}`, onclick: () => { s.y = i; s.y_pred = j; s.page = 0; App.render(true); }}, v))))));
  }
  const filt = {y: nz(s.y, undefined), y_pred: nz(s.y_pred, undefined),
    score_min: nz(s.score_min, undefined), score_max: nz(s.score_max, undefined)};
  const imgs = await imagesFor('img_classify', report, comp.source, s, filt);
  const num = (k, ph) => el('input', {type: 'number', step: 'any', placeholder: ph, value: nz(s[k], ''), style: {width: '80px'},
    onchange: e => { s[k] = e.target.value === '' ? null : +e.target.value; s.page = 0; App.render(true); }});
  box.append(el('div', {class: 'toolbar'}, 'y', num('y', 'any'), 'y_pred', num('y_pred', 'any'), 'score', num('score_min', 'min'), num('score_max', 'max'),
    el('button', {class: 'small', onclick: () => { s.page = Math.max(0, s.page - 1); App.render(true); }}, '‹'), `page ${s.page + 1}`,
    el('button', {class: 'small', onclick: () => { s.page++; App.render(true); }}, '›')),
  el('div', {class: 'imgs'}, imgs.map(x => imgFigure(x, `#${x.task} y=${nz(x.y, '')} pred=${nz(x.y_pred, '')} score=${fmt.num(x.score, 3)}`))));
  return box;
}

async function imgGrid(kind, report, comp, st) {
  const key = 'ig_' + comp.source;
  const s = st[key] = st[key] || {page: 0};
  const imgs = await imagesFor(kind, report, comp.source, s);
  return el('div', {class: 'card'}, el('h3', {style: {marginTop: 0}}, comp.source),
    el('div', {class: 'toolbar'},
      el('button', {class: 'small', onclick: () => { s.page = Math.max(0, s.page - 1); App.render(true); }}, '‹'), `page ${s.page + 1}`,
      el('button', {class: 'small', onclick: () => { s.page++; App.render(true); }}, '›')),
    el('div', {class: 'imgs'}, imgs.map(x => imgFigure(x, `#${x.task} ${x.part || ''} score=${fmt.num(x.score, 3)}`))));
}

async function renderComponents(comps, report, data, layout, st, ctx) {
  const out = [];
  for (const c of comps || []) {
    if (c.type === 'panel') {
      const key = 'panel_' + (c.title || '');
      const closed = st[key] === undefined ? c.expanded === false : st[key];
      const body = el('div', {class: 'pb', style: {gridTemplateColumns: `repeat(${c.parent_cols || 1}, minmax(0, 1fr))`}},
        await renderComponents(c.items, report, data, layout, st, Object.assign({}, ctx, {height: c.row_height ? Math.min(420, c.row_height - 60) : undefined})));
      const p = el('div', {class: 'panel' + (closed ? ' closed' : '')},
        el('div', {class: 'ph', onclick: () => { st[key] = !p.classList.contains('closed'); p.classList.toggle('closed'); }}, c.title || 'panel'), body);
      out.push(p);
    } else if (c.type === 'table') {
      out.push(metricTable(report, data, c.source, layout));
    } else if (c.type === 'series') {
      if (c.source === '_other') {
        const used = mappedSeries(layout, layout.layout, new Set());
        Object.keys(data).filter(k => !used.has(k)).sort().forEach(k => out.push(...seriesCharts(k, data[k], c.multi, ctx.height)));
      } else {
        const k = layoutKey(layout, c.source);
        if (data[k]) out.push(...seriesCharts(k, data[k], c.multi, ctx.height));
      }
    } else if (c.type === 'img_classify') {
      out.push(await imgClassify(report, c, st));
    } else if (c.type === 'img_segment' || c.type === 'img') {
      out.push(await imgGrid(c.type === 'img' ? 'img_classify' : 'img_segment', report, c, st));
    } else if (c.type === 'blank') {
      out.push(el('div'));
    }
  }
  return out;
}

App.register('report', {
  nav: 'reports',
  async render(m, args, q, st) {
    const r = await api('report', +args[0]);
    const data = {};
    r.series.forEach(s => { (data[s.name] = data[s.name] || []).push(s); });
    const layout = r.layout || {layout: [{type: 'series', source: '_other'}]};
    m.append(el('h2', {}, `Report ${r.id} · ${r.name} `, el('span', {class: 'muted'}, `layout ${r.layout_name}`)),
      el('div', {class: 'toolbar'}, el('button', {class: 'small', onclick: () => layoutChangeDialog(r)}, 'change layout…'),
        layout.metric ? el('span', {class: 'muted'}, `metric ${layout.metric.name} (${layout.metric.minimize ? 'min' : 'max'})`) : ''),
      await renderComponents(layout.layout, r, data, layout, st, {}));
  },
});

async function layoutChangeDialog(r) {
  const s = await api('report/update_layout_start', r.id);
  const f = form([{name: 'layout', type: 'select', options: s.layouts, value: s.layout}]);
  dialog('Report layout', f, [{label: 'Cancel'}, {label: 'Apply', cls: 'primary', action: async () => {
    await api('report/update_layout_end', {id: r.id, layout: f.values().layout}); App.render(true);
  }}]);
}

async function layoutsView(m, st) {
  const r = await api('layouts', {});
  st.sel = st.sel || (r.data[0] && r.data[0].name);
  const cur = r.data.find(l => l.name === st.sel);
  const ta = el('textarea', {rows: 30, spellcheck: 'false'}, cur ? cur.content : '');
  m.append(el('h2', {}, 'Report layouts'), el('div', {class: 'toolbar'},
    el('button', {class: 'primary', onclick: () => promptText('New layout name', '', async name => {
      await api('layout/add', {name, content: 'extend: base\nlayout: []\n'}); st.sel = name; App.render(true);
    })}, 'Add layout')),
  el('div', {class: 'split'},
    el('div', {class: 'tree'}, r.data.map(l => el('div', {class: 'node file' + (l.name === st.sel ? ' on' : ''), style: '--d:0',
      onclick: () => { st.sel = l.name; App.render(true); }}, l.name, ' ', el('span', {class: 'muted'}, fmt.time(l.last_modified))))),
    cur ? el('div', {},
      el('div', {class: 'toolbar'}, el('b', {}, cur.name),
        el('button', {class: 'primary small', onclick: async () => { await api('layout/edit', {name: cur.name, content: ta.value}); toast('saved'); }}, 'save'),
        el('button', {class: 'small', onclick: () => promptText('Rename layout', cur.name, async n => { await api('layout/edit', {name: cur.name, new_name: n}); st.sel = n; App.render(true); })}, 'rename'),
        el('button', {class: 'small danger', onclick: () => confirmDo(`Remove layout ${cur.name}?`, async () => { await api('layout/remove', {name: cur.name}); st.sel = null; App.render(true); })}, 'remove')),
      ta, el('div', {class: 'muted'}, 'components: panel (title, expanded, parent_cols, row_height, items) · table (source: [series]) · series (source, multi; _other) · img_classify (source, attrs) · img_segment · img · blank; items: {name: {type, key}}; metric: {name, minimize}; extend: <layout>')) : el('div')));
}

// ================================================================== skynet (memory table, spaces)
App.register('skynet', {
  async render(m, args, q, st) {
    const tab = args[0] || 'spaces';
    m.append(el('h2', {}, 'Skynet'), el('div', {class: 'tabs'}, ['spaces', 'memory'].map(t => el('a', {class: t === tab ? 'on' : null, href: `#/skynet/${t}`}, t))));
    if (tab === 'memory') return memoryView(m);
    return spacesView(m, st);
  },
}, 'Skynet');

async function memoryView(m) {
  const r = await api('memories', {});
  const edit = x => {
    const f = form([{name: 'model', value: x ? x.model : ''}, {name: 'variant', value: x ? x.variant || '' : ''},
      {name: 'num_classes', type: 'number', value: x ? x.num_classes : ''}, {name: 'img_size', type: 'number', value: x ? x.img_size : ''},
      {name: 'batch_size', type: 'number', value: x ? x.batch_size : ''}, {name: 'memory', label: 'memory (GB)', type: 'number', value: x ? x.memory : ''}]);
    dialog(x ? 'Edit memory row' : 'Add memory row', f, [{label: 'Cancel'}, {label: 'Save', cls: 'primary', action: async () => {
      const v = f.values(); if (x) v.id = x.id; await api(x ? 'memory/edit' : 'memory/add', v); App.render(true);
    }}]);
  };
  m.append(el('div', {class: 'toolbar'}, el('button', {class: 'primary', onclick: () => edit(null)}, 'Add row'),
    el('span', {class: 'muted'}, 'batch sizes the training executor picks by the GPU memory they need (catalyst_.py:247-265)')),
  grid(r.data, [{title: 'id', render: x => x.id}, {title: 'model', render: x => x.model}, {title: 'variant', render: x => x.variant || ''},
    {title: 'classes', render: x => nz(x.num_classes, '')}, {title: 'img size', render: x => nz(x.img_size, '')},
    {title: 'batch', render: x => x.batch_size}, {title: 'memory GB', render: x => fmt.num(x.memory, 1)},
    {title: '', render: x => el('span', {}, el('button', {class: 'small', onclick: () => edit(x)}, 'edit'), ' ',
      el('button', {class: 'small danger', onclick: () => confirmDo('Remove this row?', () => api('memory/remove', {id: x.id}).then(() => App.render(true)))}, 'remove'))}]));
}

async function spacesView(m, st) {
  const r = await api('spaces', {name: st.name || '', parent: st.parent || undefined});
  const rerender = () => App.render(true);
  const edit = x => {
    const f = form([{name: 'name', value: x ? x.name : ''}, {name: 'content', label: 'content (YAML patch)', type: 'textarea', rows: 14, value: x ? x.content || '' : ''}]);
    dialog(x ? `Edit space ${x.name}` : 'Add space', f, [{label: 'Cancel'}, {label: 'Save', cls: 'primary', action: async () => {
      await api(x ? 'space/edit' : 'space/add', f.values()); rerender();
    }}]);
  };
  m.append(el('div', {class: 'toolbar'},
    el('input', {placeholder: 'name filter', value: st.name || '', onchange: e => { st.name = e.target.value; rerender(); }}),
    st.parent ? el('span', {class: 'tag'}, 'children of ' + st.parent, el('a', {onclick: () => { st.parent = null; rerender(); }}, '×')) : '',
    el('button', {class: 'primary', onclick: () => edit(null)}, 'Add space'),
    el('button', {onclick: () => spaceRunDialog(r.data)}, 'Run on a DAG…')),
  grid(r.data, [
    {title: 'name', render: x => x.name},
    {title: 'tags', render: x => el('span', {}, (x.tags || []).map(t => el('span', {class: 'tag'}, t,
      el('a', {onclick: () => api('space/tag_remove', {space: x.name, tag: t}).then(rerender)}, '×'))),
      el('a', {onclick: () => promptText('Add tag', '', tag => api('space/tag_add', {space: x.name, tag}).then(rerender))}, '+tag'))},
    {title: 'content', render: x => el('pre', {class: 'plain', style: {maxHeight: '90px'}}, x.content || '')},
    {title: 'changed', render: x => fmt.time(x.changed)},
    {title: '', render: x => el('span', {},
      el('button', {class: 'small', onclick: () => edit(x)}, 'edit'), ' ',
      el('button', {class: 'small', onclick: () => { st.parent = x.name; rerender(); }}, 'children'), ' ',
      el('button', {class: 'small', onclick: () => promptText(`Add child space of ${x.name}`, '', c => api('space/relation_append', {parent: x.name, child: c}).then(rerender))}, '+child'), ' ',
      st.parent ? el('button', {class: 'small', onclick: () => api('space/relation_remove', {parent: st.parent, child: x.name}).then(rerender)}, 'unlink') : '', ' ',
      el('button', {class: 'small', onclick: () => promptText('Copy as', x.name + '_copy', n => api('space/copy', {space: {name: n, content: x.content}, old_space: x.name}).then(rerender))}, 'copy'), ' ',
      el('button', {class: 'small danger', onclick: () => confirmDo(`Remove space ${x.name}?`, () => api('space/remove', {name: x.name}).then(rerender))}, 'remove'))},
  ]));
}

function spaceRunDialog(spaces) {
  const rows = el('div');
  const addRow = () => rows.append(el('div', {class: 'toolbar'},
    el('select', {class: 'logic'}, ['and', 'or'].map(l => el('option', {value: l}, l))),
    el('select', {class: 'space'}, spaces.map(s => el('option', {value: s.name}, s.name)))));
  addRow();
  const dag = el('input', {type: 'number', placeholder: 'DAG id'});
  const fc = el('textarea', {rows: 5, placeholder: 'extra file changes (YAML)'});
  dialog('Run spaces on a DAG (AND-spaces merge; one copy per OR-space)', el('div', {},
    el('div', {class: 'form'}, el('label', {}, 'DAG'), dag, el('label', {}, 'file changes'), fc),
    el('h3', {}, 'spaces'), rows, el('button', {class: 'small', onclick: addRow}, '+ space')),
  [{label: 'Cancel'}, {label: 'Run', cls: 'primary', action: async () => {
    const sp = [...rows.children].map(r => ({logic: r.querySelector('.logic').value, value: r.querySelector('.space').value}));
    const res = await api('space/run', {dag: +dag.value, spaces: sp, file_changes: fc.value});
    toast('created DAGs ' + JSON.stringify(res.dags));
  }}]);
}

// ================================================================== auxiliary (scheduler snapshot)
App.register('auxiliary', {
  async render(m) {
    const r = await api('auxiliary', {});
    const sup = r.supervisor || {};
    m.append(el('h2', {}, 'Scheduler'), el('div', {class: 'muted'}, `tick at ${sup.time || '?'} · ${fmt.num(sup.duration, 3)} s`),
      el('h3', {}, 'live queues'), el('div', {}, (sup.queues || []).map(qn => el('span', {class: 'tag'}, qn))),
      el('h3', {}, 'resource ledger'), grid(sup.computers || [], [
        {title: 'computer', render: c => c.name}, {title: 'free cpu', render: c => `${c.cpu} / ${c.cpu_total}`},
        {title: 'free memory', render: c => `${fmt.gb(c.memory)} / ${fmt.gb(c.memory_total)}`},
        {title: 'gpus (owner task)', render: c => (c.gpu || []).map((g, i) => el('span', {class: 'tag', style: {background: g ? '#fde2e1' : '#d9f2e3'}}, `${i}:${g || 'free'}`))},
        {title: 'master ports', render: c => (c.ports || []).join(', ')}]),
      el('h3', {}, 'placement of the first tasks'), grid(sup.process_tasks || [], [
        {title: 'task', render: t => el('a', {href: `#/task/${t.id}`}, `${t.id} ${t.name}`)},
        {title: 'not valid', render: t => t.not_valid || ''},
        {title: 'computers', render: t => (t.computers || []).map(c => el('div', {}, `${c.name}: ${c.error || 'ok'}`))}]),
      el('h3', {}, 'parent tasks'), el('pre', {class: 'plain'}, JSON.stringify(sup.parent_tasks_stats || [], null, 1)),
      el('h3', {}, 'everything'), el('pre', {class: 'plain'}, JSON.stringify(r, null, 1)));
  },
}, 'Scheduler');
