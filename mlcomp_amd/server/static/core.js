// mlcomp_amd UI core: API client, hash router, DOM helpers and the reusable widgets
// (tables with paging/sorting, status badges, SVG line charts and gauges, the DAG graph,
// trees, dialogs).  Plain ES2017, no build step; pages.js registers the views.
'use strict';

const STATUSES = ['not_ran', 'queued', 'in_progress', 'failed', 'stopped', 'skipped', 'success'];
const LEVELS = ['debug', 'info', 'warning', 'error'];
const COMPONENTS = ['API', 'Supervisor', 'Worker', 'WorkerSupervisor', 'Client'];
const PALETTE = ['#1d7bd8', '#d64545', '#2f9e5b', '#e08a1e', '#7c5cd6', '#0fa3b1', '#c2185b', '#6b8e23', '#8d6e63', '#455a64'];

// ------------------------------------------------------------------ API
class AuthError extends Error {}

async function api(name, body) {
  const r = await fetch('/api/' + name, {
    method: 'POST',
    headers: {'Authorization': localStorage.getItem('token') || '', 'Content-Type': 'application/json'},
    body: JSON.stringify(body === undefined ? {} : body),
  });
  if (r.status === 401) { App.showLogin(); throw new AuthError('auth'); }
  const j = await r.json();
  if (!j.success) { toast(firstLine(j.error || 'request failed'), true); throw new Error(j.error); }
  return j;
}

async function apiDownload(path, filename) {
  const r = await fetch(path, {headers: {'Authorization': localStorage.getItem('token') || ''}});
  if (!r.ok) { toast('download failed', true); return; }
  const url = URL.createObjectURL(await r.blob());
  const a = el('a', {href: url, download: filename});
  document.body.append(a); a.click(); a.remove();
  setTimeout(() => URL.revokeObjectURL(url), 5000);
}

const nz = (v, d) => (v === null || v === undefined) ? d : v;
const firstLine = s => String(s).trim().split('\n').slice(-1)[0].slice(0, 300);
const pag = (page = 0, size = 50, col = 'id', desc = true) =>
  ({page_number: page, page_size: size, sort_column: col, sort_descending: desc});

// ------------------------------------------------------------------ DOM
function el(tag, attrs, ...kids) {
  const e = document.createElement(tag);
  for (const [k, v] of Object.entries(attrs || {})) {
    if (v === undefined || v === null || v === false) continue;
    if (k.startsWith('on')) e.addEventListener(k.slice(2), v);
    else if (k === 'html') e.innerHTML = v;
    else if (k === 'style' && typeof v === 'object') Object.assign(e.style, v);
    else e.setAttribute(k, v === true ? '' : v);
  }
  for (const c of kids.flat(Infinity)) {
    if (c === null || c === undefined || c === false) continue;
    e.append(c instanceof Node ? c : document.createTextNode(String(c)));
  }
  return e;
}
const svgEl = (tag, attrs, ...kids) => {
  const e = document.createElementNS('http://www.w3.org/2000/svg', tag);
  for (const [k, v] of Object.entries(attrs || {})) {
    if (k.startsWith('on')) e.addEventListener(k.slice(2), v); else if (v !== undefined) e.setAttribute(k, v);
  }
  for (const c of kids.flat()) if (c !== null && c !== undefined) e.append(c instanceof Node ? c : document.createTextNode(String(c)));
  return e;
};
const fmt = {
  time: s => s ? String(s).replace('T', ' ').slice(0, 19) : '',
  num: (v, d = 4) => (v === null || v === undefined || v === '') ? '' : (typeof v === 'number' ? (Number.isInteger(v) ? String(v) : v.toFixed(d)) : String(v)),
  gb: mb => mb ? (mb / 1024).toFixed(0) + ' GB' : '',
};

let toastTimer = null;
function toast(msg, bad) {
  const t = document.getElementById('toast');
  t.textContent = msg; t.className = 'show' + (bad ? ' bad' : '');
  clearTimeout(toastTimer); toastTimer = setTimeout(() => { t.className = ''; }, bad ? 6000 : 2500);
}

function statusBadge(s) {
  const name = typeof s === 'number' ? STATUSES[s] : s;
  return el('span', {class: 'st st-' + name}, String(name).replace('_', ' '));
}

function statusCounts(list) {   // [{name, count}] -> badges of the non-zero ones
  return el('span', {class: 'counts'}, (list || []).filter(x => x.count).map(x => el('span', {}, statusBadge(x.name), ' ', x.count)));
}

function progressBar(a, b) {
  if (!b) return '';
  const p = Math.min(100, 100 * a / b);
  return el('div', {}, el('div', {class: 'bar'}, el('div', {style: {width: p + '%'}})), el('span', {class: 'muted'}, `${a}/${b}`));
}

function loadBar(pct) {
  const v = Math.max(0, Math.min(100, +pct || 0));
  return el('div', {class: 'bar' + (v > 90 ? ' hot' : v > 70 ? ' warn' : ''), title: v.toFixed(0) + '%'}, el('div', {style: {width: v + '%'}}));
}

// ------------------------------------------------------------------ table with paging / sorting
// cols: [{title, render(row) -> node|string, sort: 'column'}]; state: {page, size, col, desc}
function grid(rows, cols, opts = {}) {
  const head = el('tr', {}, cols.map(c => {
    const th = el('th', {class: c.sort ? 'sort' : null}, c.title);
    if (c.sort && opts.state) {
      if (opts.state.col === c.sort) th.append(opts.state.desc ? ' ▾' : ' ▴');
      th.onclick = () => { const s = opts.state; s.desc = s.col === c.sort ? !s.desc : true; s.col = c.sort; opts.onChange(); };
    }
    return th;
  }));
  const body = rows.map(r => {
    const tr = el('tr', {class: opts.onClick ? 'click' : null}, cols.map(c => el('td', {}, c.render(r))));
    if (opts.onClick) tr.onclick = ev => { if (!ev.target.closest('button,a,input,select')) opts.onClick(r); };
    return tr;
  });
  return el('table', {class: 'grid'}, head, body);
}

function pager(total, state, onChange) {
  const pages = Math.max(1, Math.ceil(total / state.size));
  return el('div', {class: 'pager'},
    el('button', {class: 'small', disabled: state.page <= 0, onclick: () => { state.page--; onChange(); }}, '‹'),
    `page ${state.page + 1} / ${pages} (${total})`,
    el('button', {class: 'small', disabled: state.page >= pages - 1, onclick: () => { state.page++; onChange(); }}, '›'),
    el('select', {onchange: e => { state.size = +e.target.value; state.page = 0; onChange(); }},
      [20, 50, 100, 500].map(n => el('option', {value: n, selected: n === state.size}, n + ' / page'))));
}

// ------------------------------------------------------------------ charts
// series: [{label, x: [], y: [], color?}]; time-valued x (ISO strings) are plotted by time
function lineChart(series, opts = {}) {
  const W = opts.width || 520, H = opts.height || 220, L = 46, R = 10, T = 10, B = 24;
  const wrap = el('div', {class: 'chart'}, opts.title ? el('div', {class: 'title'}, opts.title) : null);
  const pts = series.filter(s => s.x && s.x.length);
  if (!pts.length) { wrap.append(el('div', {class: 'muted'}, 'no data')); return wrap; }
  const isTime = typeof pts[0].x[0] === 'string';
  const xv = v => isTime ? Date.parse(String(v).replace(' ', 'T') + (String(v).endsWith('Z') ? '' : 'Z')) : +v;
  const xs = pts.flatMap(s => s.x.map(xv)), ys = pts.flatMap(s => s.y.filter(v => v !== null && isFinite(v)));
  let x0 = Math.min(...xs), x1 = Math.max(...xs), y0 = Math.min(...ys), y1 = Math.max(...ys);
  if (opts.yMin !== undefined) y0 = opts.yMin;
  if (opts.yMax !== undefined) y1 = opts.yMax;
  if (x1 === x0) { x1 = x0 + 1; } if (y1 === y0) { y1 = y0 + Math.abs(y0 || 1) * 0.1; y0 -= Math.abs(y0 || 1) * 0.1; }
  const sx = x => L + (W - L - R) * (x - x0) / (x1 - x0), sy = y => H - B - (H - T - B) * (y - y0) / (y1 - y0);
  const svg = svgEl('svg', {width: W, height: H});
  for (let i = 0; i <= 4; i++) {
    const y = y0 + (y1 - y0) * i / 4;
    svg.append(svgEl('line', {x1: L, x2: W - R, y1: sy(y), y2: sy(y), stroke: '#edf0f4'}),
      svgEl('text', {x: 2, y: sy(y) + 3}, Math.abs(y) >= 1000 ? y.toExponential(2) : +y.toPrecision(4)));
  }
  const xlab = v => isTime ? new Date(v).toISOString().slice(11, 16) : +(+v).toPrecision(4);
  for (let i = 0; i <= 4; i++) {
    const x = x0 + (x1 - x0) * i / 4;
    svg.append(svgEl('text', {x: sx(x) - 10, y: H - 6}, xlab(x)));
  }
  pts.forEach((s, i) => {
    const c = s.color || PALETTE[i % PALETTE.length];
    const p = s.x.map((x, j) => (s.y[j] === null || !isFinite(s.y[j])) ? null : [sx(xv(x)), sy(s.y[j])]).filter(Boolean);
    svg.append(svgEl('polyline', {fill: 'none', stroke: c, 'stroke-width': 1.8, points: p.map(q => q.join(',')).join(' ')}));
    if (p.length <= 60) p.forEach((q, j) => svg.append(svgEl('circle', {cx: q[0], cy: q[1], r: 2.4, fill: c},
      svgEl('title', {}, `${s.label}: ${fmt.num(s.y[j], 5)} @ ${isTime ? fmt.time(s.x[j]) : s.x[j]}`))));
  });
  wrap.append(svg);
  wrap.append(el('div', {}, pts.map((s, i) => el('span', {class: 'tag', style: {background: 'transparent', color: s.color || PALETTE[i % PALETTE.length]}},
    '■ ' + s.label + (s.y.length ? ' = ' + fmt.num(s.y[s.y.length - 1], 4) : '')))));
  return wrap;
}

function gauge(pct, label) {
  const v = Math.max(0, Math.min(100, +pct || 0)), r = 30, c = Math.PI * r;
  const col = v > 90 ? '#d64545' : v > 70 ? '#e0a030' : '#2f9e5b';
  const arc = `M ${40 - r} 40 A ${r} ${r} 0 0 1 ${40 + r} 40`;
  return el('div', {class: 'gauge'},
    svgEl('svg', {width: 80, height: 48},
      svgEl('path', {d: arc, fill: 'none', stroke: '#e3e8ee', 'stroke-width': 8}),
      svgEl('path', {d: arc, fill: 'none', stroke: col, 'stroke-width': 8, 'stroke-dasharray': `${c * v / 100} ${c}`}),
      svgEl('text', {x: 40, y: 38, 'text-anchor': 'middle', style: 'font-size:12px;fill:#1f2933;font-weight:600'}, v.toFixed(0) + '%')),
    el('div', {class: 'lbl'}, label));
}

// ------------------------------------------------------------------ DAG graph
// Layered layout: longest-path layering from the sources, then barycentric ordering
// sweeps inside each layer; edges are cubic curves coloured by their source's status.
const STATUS_COLORS = {not_ran: '#9aa5b1', queued: '#7c5cd6', in_progress: '#1d7bd8', failed: '#d64545',
  stopped: '#c8811a', skipped: '#b8a038', success: '#2f9e5b'};

function layoutDag(nodes, edges) {
  const ids = nodes.map(n => n.id), preds = {}, succs = {};
  ids.forEach(i => { preds[i] = []; succs[i] = []; });
  edges.forEach(e => { if (preds[e.to] && succs[e.from]) { preds[e.to].push(e.from); succs[e.from].push(e.to); } });
  const layer = {}, seen = {};
  const depth = i => {
    if (layer[i] !== undefined) return layer[i];
    if (seen[i]) return 0;           // a cycle (not expected in a DAG): cut it
    seen[i] = true;
    layer[i] = preds[i].length ? 1 + Math.max(...preds[i].map(depth)) : 0;
    return layer[i];
  };
  ids.forEach(depth);
  const layers = [];
  ids.forEach(i => { (layers[layer[i]] = layers[layer[i]] || []).push(i); });
  const pos = {};
  const setPos = () => layers.forEach(l => l.forEach((i, k) => { pos[i] = k; }));
  setPos();
  for (let sweep = 0; sweep < 4; sweep++) {
    const down = sweep % 2 === 0;
    const order = down ? layers.slice(1) : layers.slice(0, -1).reverse();
    order.forEach(l => {
      const bc = i => { const nb = down ? preds[i] : succs[i]; return nb.length ? nb.reduce((s, j) => s + pos[j], 0) / nb.length : pos[i]; };
      l.sort((a, b) => bc(a) - bc(b));
      l.forEach((i, k) => { pos[i] = k; });
    });
  }
  return {layer, pos, layers};
}

function dagGraph(g, onNode) {
  const NW = 150, NH = 34, GX = 60, GY = 26;
  const {layer, pos, layers} = layoutDag(g.nodes, g.edges);
  const maxRows = Math.max(1, ...layers.map(l => l.length));
  const W = Math.max(300, layers.length * (NW + GX) + GX), H = maxRows * (NH + GY) + GY;
  const xy = i => [GX / 2 + layer[i] * (NW + GX), GY + pos[i] * (NH + GY) + (maxRows - layers[layer[i]].length) * (NH + GY) / 2];
  const svg = svgEl('svg', {class: 'dag', width: W, height: H},
    svgEl('defs', {}, svgEl('marker', {id: 'arr', viewBox: '0 0 10 10', refX: 10, refY: 5, markerWidth: 7, markerHeight: 7, orient: 'auto'},
      svgEl('path', {d: 'M0,0 L10,5 L0,10 z', fill: '#8a97a5'}))));
  g.edges.forEach(e => {
    if (layer[e.from] === undefined || layer[e.to] === undefined) return;
    const [x1, y1] = xy(e.from), [x2, y2] = xy(e.to);
    const a = [x1 + NW, y1 + NH / 2], b = [x2, y2 + NH / 2], m = (a[0] + b[0]) / 2;
    svg.append(svgEl('path', {d: `M${a} C${m},${a[1]} ${m},${b[1]} ${b}`, fill: 'none', 'marker-end': 'url(#arr)',
      stroke: STATUS_COLORS[e.status] || '#8a97a5', 'stroke-width': 1.6}));
  });
  g.nodes.forEach(n => {
    const [x, y] = xy(n.id);
    const label = (n.label || n.name || String(n.id));
    svg.append(svgEl('g', {class: 'n', onclick: () => onNode && onNode(n)},
      svgEl('rect', {x, y, width: NW, height: NH, rx: 6, fill: STATUS_COLORS[n.status] || '#9aa5b1', stroke: '#17212b', 'stroke-opacity': .25}),
      svgEl('text', {x: x + 8, y: y + 14}, label.length > 22 ? label.slice(0, 21) + '…' : label),
      svgEl('text', {x: x + 8, y: y + 27, style: 'font-size:10px;fill:#f1f5f9'}, String(n.status).replace('_', ' ')),
      svgEl('title', {}, `${label}\n${n.status}`)));
  });
  return el('div', {style: {overflow: 'auto'}}, svg);
}

// ------------------------------------------------------------------ trees
// nodes: [{..., children: []}]; label(node) -> node|string; onSelect(node)
function tree(nodes, label, onSelect, opts = {}) {
  const box = el('div', {class: 'tree' + (opts.cls ? ' ' + opts.cls : '')});
  const open = opts.open || new Set();
  const walk = (list, d) => list.forEach(n => {
    const dir = n.children && n.children.length;
    const key = opts.key ? opts.key(n) : n.id;
    const row = el('div', {class: 'node ' + (dir ? 'dir' + (open.has(key) || opts.expandAll ? ' open' : '') : 'file') +
      (opts.selected === key ? ' on' : ''), style: `--d:${d}`}, label(n));
    row.onclick = () => {
      if (dir && !opts.expandAll) { open.has(key) ? open.delete(key) : open.add(key); box.replaceWith(tree(nodes, label, onSelect, Object.assign(opts, {open}))); }
      if (onSelect) onSelect(n);
    };
    box.append(row);
    if (dir && (open.has(key) || opts.expandAll)) walk(n.children, d + 1);
  });
  walk(nodes, 0);
  return box;
}

// ------------------------------------------------------------------ dialogs and forms
function dialog(title, body, buttons) {
  const m = el('div', {class: 'modal'});
  const close = () => m.remove();
  const btns = (buttons || [{label: 'Close'}]).map(b => el('button', {class: b.cls || '', onclick: async () => {
    try { if (b.action && (await b.action()) === false) return; close(); } catch (e) { if (!(e instanceof AuthError)) toast(firstLine(e.message || e), true); }
  }}, b.label));
  m.append(el('div', {class: 'box'}, el('h3', {}, title), body, el('div', {class: 'actions'}, btns)));
  m.addEventListener('mousedown', e => { if (e.target === m) close(); });
  document.body.append(m);
  return close;
}

// fields: [{name, label, type: text|number|textarea|select|checkbox, value, options}]
function form(fields) {
  const inputs = {};
  const f = el('div', {class: 'form'}, fields.map(fl => {
    let inp;
    if (fl.type === 'textarea') inp = el('textarea', {rows: fl.rows || 8}, nz(fl.value, ''));
    else if (fl.type === 'select') inp = el('select', {}, (fl.options || []).map(o => {
      const [v, t] = Array.isArray(o) ? o : [o, o];
      return el('option', {value: v, selected: String(v) === String(fl.value)}, t);
    }));
    else if (fl.type === 'checkbox') inp = el('input', {type: 'checkbox', checked: !!fl.value});
    else inp = el('input', {type: fl.type || 'text', value: nz(fl.value, ''), placeholder: fl.placeholder || ''});
    inputs[fl.name] = inp;
    return [el('label', {}, fl.label || fl.name), inp];
  }));
  f.values = () => Object.fromEntries(Object.entries(inputs).map(([k, i]) =>
    [k, i.type === 'checkbox' ? i.checked : (i.type === 'number' ? (i.value === '' ? null : +i.value) : i.value)]));
  return f;
}

function confirmDo(text, fn) {
  dialog('Confirm', el('p', {}, text), [{label: 'Cancel'}, {label: 'OK', cls: 'danger', action: fn}]);
}

function kvTable(obj) {
  return el('table', {class: 'grid kv'}, Object.entries(obj).map(([k, v]) =>
    el('tr', {}, el('td', {}, k), el('td', {}, v instanceof Node ? v : (typeof v === 'object' && v !== null ? el('pre', {class: 'plain'}, JSON.stringify(v, null, 1)) : String(nz(v, '')))))));
}

// ------------------------------------------------------------------ router
const App = {
  views: {}, current: null, timer: null, nav: [],
  register(name, view, navTitle) { this.views[name] = view; if (navTitle) this.nav.push([name, navTitle]); },
  parse() {
    const h = location.hash.replace(/^#\/?/, '');
    const [path, query] = h.split('?');
    const parts = path.split('/').filter(Boolean);
    const q = Object.fromEntries(new URLSearchParams(query || ''));
    return {name: parts[0] || 'projects', args: parts.slice(1), q};
  },
  go(hash) { if (location.hash === hash) this.render(); else location.hash = hash; },
  async render(refresh) {
    const r = this.parse();
    const view = this.views[r.name] || this.views.projects;
    document.querySelectorAll('header a[data-v]').forEach(a => a.classList.toggle('on', a.dataset.v === (view.nav || r.name)));
    const main = document.getElementById('main');
    if (!refresh || !this.current || this.current.view !== view) {
      this.current = {view, state: {}};
      main.replaceChildren(el('div', {class: 'muted'}, 'loading…'));
    }
    if (refresh && view.static && view.static(r.args)) return;   // editors: no background refresh
    const tmp = el('div');
    // views append nested arrays / optional (null) parts: flatten and drop them here, as
    // el() does for its children (a native append() would stringify them)
    tmp.append = (...kids) => Element.prototype.append.apply(tmp, kids.flat(Infinity).filter(k => k !== null && k !== undefined && k !== false));
    try {
      await view.render(tmp, r.args, r.q, this.current.state);
      if (this.current.view === view) main.replaceChildren(...tmp.childNodes);
    } catch (e) {
      if (!(e instanceof AuthError)) { console.error(e); if (!refresh) main.replaceChildren(el('div', {class: 'err'}, String(e.message || e))); }
    }
  },
  showLogin() {
    document.getElementById('login').hidden = false;
    document.getElementById('hdr').hidden = true;
    document.getElementById('main').hidden = true;
    clearInterval(this.timer);
  },
  async login() {
    const t = document.getElementById('tok').value.trim();
    const r = await fetch('/api/token', {method: 'POST', body: JSON.stringify({token: t})});
    if (r.status === 200) { localStorage.setItem('token', t); this.start(); }
    else document.getElementById('lerr').textContent = 'invalid token';
  },
  start() {
    document.getElementById('login').hidden = true;
    document.getElementById('hdr').hidden = false;
    document.getElementById('main').hidden = false;
    const nav = document.getElementById('nav');
    nav.replaceChildren(...this.nav.map(([v, t]) => el('a', {'data-v': v, href: '#/' + v}, t)));
    this.render();
    clearInterval(this.timer);
    this.timer = setInterval(() => { if (!document.querySelector('.modal') && !document.hidden) this.render(true); }, 3000);
  },
  boot() {
    window.addEventListener('hashchange', () => this.render());
    document.getElementById('tok').addEventListener('keydown', e => { if (e.key === 'Enter') this.login(); });
    localStorage.getItem('token') ? this.start() : this.showLogin();
  },
};
