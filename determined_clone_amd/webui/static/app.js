// Single-page UI over the master's /api/v1 REST surface. No build step, no dependencies.
"use strict";

// ------------------------------------------------------------------------------------ api
const api = {
  get token() { return localStorage.getItem("det_token"); },
  async call(method, path, body) {
    const headers = { "Content-Type": "application/json" };
    if (this.token) headers.Authorization = "Bearer " + this.token;
    const res = await fetch(path, { method, headers, body: body === undefined ? undefined : JSON.stringify(body) });
    let data = {};
    try { data = await res.json(); } catch (e) { /* empty body */ }
    if (res.status === 401 && !path.endsWith("/auth/login")) {
      localStorage.removeItem("det_token");
      location.hash = "#/login?next=" + encodeURIComponent(location.hash);
      throw new Error("unauthenticated");
    }
    if (!res.ok) throw new Error(data.error || res.status + " " + res.statusText);
    return data;
  },
  get(p) { return this.call("GET", p); },
  post(p, b) { return this.call("POST", p, b || {}); },
  patch(p, b) { return this.call("PATCH", p, b || {}); },
  del(p, b) { return this.call("DELETE", p, b); },
};

// ------------------------------------------------------------------------------------ dom helpers
function h(tag, attrs, ...kids) {
  const el = document.createElement(tag);
  for (const [k, v] of Object.entries(attrs || {})) {
    if (v === undefined || v === null || v === false) continue;
    if (k.startsWith("on")) el.addEventListener(k.slice(2), v);
    else if (k === "class") el.className = v;
    else el.setAttribute(k, v === true ? "" : v);
  }
  for (const kid of kids.flat(Infinity)) {
    if (kid === undefined || kid === null || kid === false) continue;
    el.appendChild(kid instanceof Node ? kid : document.createTextNode(String(kid)));
  }
  return el;
}
const badge = (s) => h("span", { class: "badge " + (s || "") }, (s || "-").replace(/^STATE_/, ""));
const link = (href, text) => h("a", { href }, text);
function fmtTime(t) {
  if (t === null || t === undefined || t === "") return "-";
  const d = typeof t === "number" ? new Date(t * 1000) : new Date(t);
  return isNaN(d) ? String(t) : d.toLocaleString();
}
function fmtDur(a, b) {
  if (!a) return "-";
  const s = Math.max(0, Math.round(((b || Date.now() / 1000) - a)));
  return s < 90 ? s + "s" : s < 5400 ? Math.round(s / 60) + "m" : (s / 3600).toFixed(1) + "h";
}
function fmtNum(v) {
  if (typeof v !== "number") return v === undefined || v === null ? "-" : String(v);
  return Math.abs(v) >= 1e4 || (Math.abs(v) < 1e-3 && v !== 0) ? v.toExponential(3) : +v.toPrecision(5) + "";
}
function progressBar(p) {
  const pct = Math.max(0, Math.min(1, p || 0)) * 100;
  return h("div", { class: "progress", title: pct.toFixed(0) + "%" }, h("div", { style: `width:${pct}%` }));
}
const errBox = (e) => h("div", { class: "err" }, String(e.message || e));
async function act(fn, after) {
  try { await fn(); if (after) after(); else render(); } catch (e) { alert(e.message || e); }
}

// sortable table: cols = [{key, label, render?(row), sort?(row)}]
function table(cols, rows, opts) {
  opts = opts || {};
  let sortKey = opts.sortKey, desc = opts.desc !== false;
  const tbody = h("tbody");
  const fill = () => {
    tbody.innerHTML = "";
    const col = cols.find((c) => c.key === sortKey);
    const data = rows.slice();
    if (col) {
      const f = col.sort || ((r) => r[col.key]);
      data.sort((a, b) => {
        const x = f(a), y = f(b);
        const c = x === y ? 0 : x === undefined || x === null ? 1 : y === undefined || y === null ? -1 : x < y ? -1 : 1;
        return desc ? -c : c;
      });
    }
    if (!data.length) tbody.appendChild(h("tr", {}, h("td", { colspan: cols.length, class: "muted" }, opts.empty || "nothing here")));
    for (const r of data) tbody.appendChild(h("tr", {}, cols.map((c) => h("td", {}, c.render ? c.render(r) : fmtNum(r[c.key])))));
  };
  const head = h("tr", {}, cols.map((c) => h("th", {
    onclick: () => { desc = sortKey === c.key ? !desc : true; sortKey = c.key; fill(); },
  }, c.label)));
  fill();
  return h("table", {}, h("thead", {}, head), tbody);
}

// ------------------------------------------------------------------------------------ charts
const PALETTE = ["#c8102e", "#1f77b4", "#2ca02c", "#ff7f0e", "#9467bd", "#8c564b", "#e377c2", "#17becf", "#7f7f7f", "#bcbd22"];
function niceTicks(lo, hi, n) {
  if (lo === hi) { lo -= 1; hi += 1; }
  const step0 = (hi - lo) / n, mag = Math.pow(10, Math.floor(Math.log10(step0)));
  const step = [1, 2, 5, 10].map((m) => m * mag).find((s) => s >= step0);
  const out = [];
  for (let v = Math.ceil(lo / step) * step; v <= hi + step * 1e-9; v += step) out.push(+v.toPrecision(12));
  return out;
}
// series: [{name, points: [[x, y], ...]}]
function lineChart(title, series, xlabel, opts) {
  opts = opts || {};
  const NS = "http://www.w3.org/2000/svg";
  const W = 460, H = 240, L = 58, R = 12, T = 10, B = 34;
  const pts = series.flatMap((s) => s.points).filter((p) => isFinite(p[0]) && isFinite(p[1]));
  const svg = document.createElementNS(NS, "svg");
  svg.setAttribute("viewBox", `0 0 ${W} ${H}`);
  const mk = (tag, attrs, text) => {
    const e = document.createElementNS(NS, tag);
    for (const [k, v] of Object.entries(attrs)) e.setAttribute(k, v);
    if (text !== undefined) e.textContent = text;
    svg.appendChild(e);
    return e;
  };
  if (!pts.length) {
    mk("text", { x: W / 2, y: H / 2, "text-anchor": "middle", fill: "#6b7685", "font-size": 12 }, "no data");
  } else {
    let x0 = Math.min(...pts.map((p) => p[0])), x1 = Math.max(...pts.map((p) => p[0]));
    let y0 = Math.min(...pts.map((p) => p[1])), y1 = Math.max(...pts.map((p) => p[1]));
    if (x0 === x1) { x0 -= 1; x1 += 1; }
    if (y0 === y1) { y0 -= Math.abs(y0) * 0.1 || 1; y1 += Math.abs(y1) * 0.1 || 1; }
    const sx = (x) => L + ((x - x0) / (x1 - x0)) * (W - L - R), sy = (y) => H - B - ((y - y0) / (y1 - y0)) * (H - T - B);
    for (const t of niceTicks(y0, y1, 5)) {
      if (t < y0 || t > y1) continue;
      mk("line", { x1: L, x2: W - R, y1: sy(t), y2: sy(t), stroke: "#eef0f3" });
      mk("text", { x: L - 6, y: sy(t) + 4, "text-anchor": "end", "font-size": 10, fill: "#6b7685" }, fmtNum(t));
    }
    for (const t of niceTicks(x0, x1, 6)) {
      if (t < x0 || t > x1) continue;
      mk("text", { x: sx(t), y: H - B + 14, "text-anchor": "middle", "font-size": 10, fill: "#6b7685" }, fmtNum(t));
    }
    mk("line", { x1: L, x2: L, y1: T, y2: H - B, stroke: "#9aa6b4" });
    mk("line", { x1: L, x2: W - R, y1: H - B, y2: H - B, stroke: "#9aa6b4" });
    if (xlabel) mk("text", { x: (L + W - R) / 2, y: H - 4, "text-anchor": "middle", "font-size": 10, fill: "#6b7685" }, xlabel);
    series.forEach((s, i) => {
      const p = s.points.filter((q) => isFinite(q[0]) && isFinite(q[1])).sort((a, b) => a[0] - b[0]);
      if (!p.length) return;
      const color = PALETTE[i % PALETTE.length];
      if (!opts.scatter) mk("polyline", { points: p.map((q) => sx(q[0]) + "," + sy(q[1])).join(" "), fill: "none", stroke: color, "stroke-width": 1.6 });
      if (opts.scatter || p.length < 40) p.forEach((q) => mk("circle", { cx: sx(q[0]), cy: sy(q[1]), r: opts.scatter ? 3.2 : 2.2, fill: color, "fill-opacity": opts.scatter ? 0.75 : 1 }));
    });
  }
  const legend = h("div", { class: "legend" }, series.length > 1 ? series.map((s, i) =>
    h("span", {}, h("i", { style: `background:${PALETTE[i % PALETTE.length]}` }), s.name)) : null);
  return h("div", { class: "card chart" }, h("div", { class: "title" }, title), svg, legend);
}

// metric rows [{group, steps_completed, metrics}] -> one chart per metric name, one series per group
function metricCharts(rowsBySeries) {
  const names = new Set();
  for (const s of rowsBySeries) for (const r of s.rows) for (const [k, v] of Object.entries(r.metrics || {})) if (typeof v === "number") names.add(k);
  return h("div", { class: "charts" }, [...names].sort().map((name) => lineChart(name, rowsBySeries.map((s) => ({
    name: s.name,
    points: s.rows.filter((r) => typeof (r.metrics || {})[name] === "number").map((r) => [r.steps_completed, r.metrics[name]]),
  })), "batches")));
}

// Parallel coordinates (reference ExperimentVisualization HpParallelCoordinates): one vertical
// axis per hyperparameter plus the searcher metric, one polyline per trial, coloured from best
// (red) to worst (blue) on the metric. Categorical / string hparams get evenly spaced categories.
function hpAxes(trials, keys) {
  return keys.map((k) => {
    const vals = trials.map((t) => (t.hparams || {})[k]);
    const numeric = vals.every((v) => typeof v === "number");
    if (numeric) {
      const lo = Math.min(...vals), hi = Math.max(...vals);
      const log = lo > 0 && hi / lo > 50;
      const f = (v) => (log ? Math.log10(v) : v);
      const a = f(lo), b = f(hi);
      return { key: k, pos: (v) => (b === a ? 0.5 : (f(v) - a) / (b - a)), ticks: [lo, hi].map(fmtNum), log };
    }
    const cats = [...new Set(vals.map((v) => JSON.stringify(v)))].sort();
    return { key: k, pos: (v) => (cats.length < 2 ? 0.5 : cats.indexOf(JSON.stringify(v)) / (cats.length - 1)), ticks: cats, cats: true };
  });
}
function parallelCoords(title, trials, keys, metric, smallerIsBetter) {
  const NS = "http://www.w3.org/2000/svg";
  const scored = trials.filter((t) => typeof t.best_validation === "number");
  const W = Math.max(460, 130 * (keys.length + 1)), H = 280, T = 24, B = 30, L = 40, R = 40;
  const svg = document.createElementNS(NS, "svg");
  svg.setAttribute("viewBox", `0 0 ${W} ${H}`);
  svg.setAttribute("class", "pcoords");
  const mk = (tag, attrs, text) => {
    const e = document.createElementNS(NS, tag);
    for (const [k, v] of Object.entries(attrs)) e.setAttribute(k, v);
    if (text !== undefined) e.textContent = text;
    svg.appendChild(e);
    return e;
  };
  if (!scored.length || !keys.length) {
    mk("text", { x: W / 2, y: H / 2, "text-anchor": "middle", fill: "#6b7685", "font-size": 12 }, "no scored trials");
    return h("div", { class: "card chart wide" }, h("div", { class: "title" }, title), svg);
  }
  const axes = hpAxes(scored, keys);
  const ms = scored.map((t) => t.best_validation);
  const m0 = Math.min(...ms), m1 = Math.max(...ms);
  axes.push({ key: metric, pos: (v) => (m1 === m0 ? 0.5 : (v - m0) / (m1 - m0)), ticks: [m0, m1].map(fmtNum), metric: true });
  const xs = axes.map((_, i) => L + (i * (W - L - R)) / Math.max(1, axes.length - 1));
  const y = (p) => H - B - p * (H - T - B);
  // colour: 0 = best, 1 = worst
  const rank = (v) => (m1 === m0 ? 0 : smallerIsBetter === false ? (m1 - v) / (m1 - m0) : (v - m0) / (m1 - m0));
  const colour = (q) => `rgb(${Math.round(200 - 170 * q)},${Math.round(40 + 60 * q)},${Math.round(46 + 150 * q)})`;
  // worst first so the best trials are drawn on top
  for (const t of scored.slice().sort((a, b) => rank(b.best_validation) - rank(a.best_validation))) {
    const pts = axes.map((a, i) => xs[i] + "," + y(a.pos(a.metric ? t.best_validation : t.hparams[a.key])));
    const line = mk("polyline", { points: pts.join(" "), fill: "none", stroke: colour(rank(t.best_validation)),
      "stroke-width": 1.4, "stroke-opacity": 0.8, "data-trial": t.id });
    const tip = document.createElementNS(NS, "title");
    tip.textContent = `trial ${t.id}: ${metric}=${fmtNum(t.best_validation)}`;
    line.appendChild(tip);
  }
  axes.forEach((a, i) => {
    mk("line", { x1: xs[i], x2: xs[i], y1: T, y2: H - B, stroke: "#6b7685" });
    mk("text", { x: xs[i], y: 14, "text-anchor": "middle", "font-size": 11, "font-weight": a.metric ? "bold" : "normal" },
      a.key + (a.log ? " (log)" : ""));
    const ticks = a.cats ? a.ticks : [a.ticks[0], a.ticks[1]];
    ticks.forEach((tk, j) => {
      const p = a.cats ? (ticks.length < 2 ? 0.5 : j / (ticks.length - 1)) : j;
      mk("text", { x: xs[i] + 4, y: y(p) + (j === 0 && !a.cats ? -2 : 10), "font-size": 9, fill: "#6b7685" }, String(tk).replace(/^"|"$/g, ""));
    });
  });
  return h("div", { class: "card chart wide" }, h("div", { class: "title" }, title), svg,
    h("div", { class: "legend" }, h("span", {}, h("i", { style: `background:${colour(0)}` }), "best"),
      h("span", {}, h("i", { style: `background:${colour(1)}` }), "worst")));
}

// ------------------------------------------------------------------------------------ pages
async function pageLogin(params) {
  const user = h("input", { placeholder: "username", value: "determined", autocomplete: "username" });
  const pass = h("input", { placeholder: "password", type: "password", autocomplete: "current-password" });
  const msg = h("div");
  const go = async () => {
    try {
      const r = await api.post("/api/v1/auth/login", { username: user.value, password: pass.value });
      localStorage.setItem("det_token", r.token);
      localStorage.setItem("det_user", r.user.username);
      location.hash = params.get("next") || "#/";
    } catch (e) { msg.replaceChildren(errBox(e)); }
  };
  pass.addEventListener("keydown", (e) => { if (e.key === "Enter") go(); });
  return h("div", { class: "card login" }, h("h1", {}, "Sign in"), user, pass,
    h("button", { class: "primary", onclick: go }, "Sign in"), msg);
}

async function pageDashboard() {
  const [exps, agents, queue, info] = await Promise.all([
    api.get("/api/v1/experiments?limit=10"), api.get("/api/v1/agents"), api.get("/api/v1/job-queues"), api.get("/api/v1/master"),
  ]);
  let slots = 0, used = 0;
  for (const a of agents.agents) for (const s of Object.values(a.slots)) { slots += 1; if (s.container) used += 1; }
  const running = exps.experiments.filter((e) => e.state === "ACTIVE").length;
  return h("div", {}, h("h1", {}, "Home"),
    h("div", { class: "row" },
      stat("cluster", info.cluster_name), stat("agents", agents.agents.length), stat("slots in use", `${used} / ${slots}`),
      stat("active experiments", running), stat("queued jobs", queue.jobs.filter((j) => j.state === "QUEUED").length)),
    h("h2", {}, "Recent experiments"), experimentTable(exps.experiments));
}
const stat = (k, v) => h("div", { class: "card stat" }, h("div", { class: "k" }, k), h("div", { class: "v" }, v));

function experimentTable(rows) {
  return table([
    { key: "id", label: "ID", render: (e) => link("#/experiments/" + e.id, e.id) },
    { key: "name", label: "Name", render: (e) => link("#/experiments/" + e.id, e.name || "-") },
    { key: "state", label: "State", render: (e) => badge(e.state) },
    { key: "searcher_type", label: "Searcher", render: (e) => e.searcher_type || "-" },
    { key: "progress", label: "Progress", render: (e) => progressBar(e.progress) },
    { key: "start_time", label: "Started", render: (e) => fmtTime(e.start_time) },
    { key: "duration", label: "Duration", sort: (e) => (e.end_time || Date.now() / 1000) - e.start_time, render: (e) => fmtDur(e.start_time, e.end_time) },
    { key: "labels", label: "Labels", render: (e) => (e.labels || []).join(", ") },
    { key: "actions", label: "", render: experimentActions },
  ], rows, { sortKey: "id" });
}
function experimentActions(e) {
  const b = (label, verb) => h("button", { onclick: () => act(() => api.post(`/api/v1/experiments/${e.id}/${verb}`)) }, label);
  const out = [];
  if (e.state === "ACTIVE") out.push(b("Pause", "pause"));
  if (e.state === "PAUSED") out.push(b("Activate", "activate"));
  if (["ACTIVE", "PAUSED"].includes(e.state)) out.push(b("Cancel", "cancel"), b("Kill", "kill"));
  else out.push(e.archived ? b("Unarchive", "unarchive") : b("Archive", "archive"));
  return out;
}

// Experiment-list filter box -> the reference's filter-group JSON (master/experiment_filter.py):
// clauses separated by ";", each "<column> <op> <value>" with op one of = != < <= > >= contains
// notContains isEmpty notEmpty; columns: experiment fields (name, state, tags, numTrials, ...),
// hp.<name>, or <group>.<metric>.<min|max|mean|last> (e.g. validation.val_loss.min < 0.1).
function parseExperimentFilter(text, showArchived) {
  const children = [];
  for (const raw of text.split(";")) {
    const m = raw.trim().match(/^(\S+)\s+(=|!=|<=|>=|<|>|contains|notContains|isEmpty|notEmpty)\s*(.*)$/);
    if (!m) continue;
    const [, col, op, rest] = m;
    let value = rest.trim().replace(/^["']|["']$/g, "");
    const num = value !== "" && !isNaN(Number(value));
    const node = { kind: "field", columnName: col, operator: op, value: op.endsWith("Empty") ? null : (num ? Number(value) : value) };
    if (col.startsWith("hp.")) Object.assign(node, { location: "LOCATION_TYPE_HYPERPARAMETERS", type: num ? "COLUMN_TYPE_NUMBER" : "COLUMN_TYPE_TEXT" });
    else if (/\.(min|max|mean|last)$/.test(col)) Object.assign(node, { location: col.startsWith("training.") ? "LOCATION_TYPE_TRAINING" : "LOCATION_TYPE_VALIDATIONS", type: num ? "COLUMN_TYPE_NUMBER" : "COLUMN_TYPE_TEXT" });
    children.push(node);
  }
  return { filterGroup: { kind: "group", conjunction: "and", children }, showArchived };
}

async function pageExperiments(params) {
  const q = new URLSearchParams();
  if (params.get("archived") !== "all") q.set("archived", "false");
  if (params.get("state")) q.append("states", params.get("state"));
  if (params.get("project")) q.set("project_id", params.get("project"));
  let r;
  const ftext = params.get("filter") || "";
  if (ftext) {  // the filter DSL runs on the search route (SearchExperiments)
    const fq = new URLSearchParams({ filter: JSON.stringify(parseExperimentFilter(ftext, params.get("archived") === "all")) });
    if (params.get("project")) fq.set("project_id", params.get("project"));
    const sr = await api.get("/api/v1/experiments-search?" + fq);
    const rows = sr.experiments.map((x) => x.experiment).filter((e) => !params.get("state") || e.state === params.get("state"));
    r = { experiments: rows, pagination: { total: rows.length } };
  } else {
    r = await api.get("/api/v1/experiments?" + q);
  }
  const fbox = h("input", { type: "text", size: 48, value: ftext, placeholder: "filter: name contains resnet; validation.val_loss.min < 0.5; hp.lr > 0.01",
    onchange: (ev) => nav("#/experiments", { state: params.get("state"), archived: params.get("archived"), filter: ev.target.value }) });
  const state = h("select", { onchange: (ev) => nav("#/experiments", { state: ev.target.value, archived: params.get("archived") }) },
    ["", "ACTIVE", "PAUSED", "COMPLETED", "CANCELED", "ERROR"].map((s) => h("option", { value: s, selected: s === (params.get("state") || "") }, s || "all states")));
  const arch = h("label", {}, h("input", { type: "checkbox", checked: params.get("archived") === "all",
    onchange: (ev) => nav("#/experiments", { state: params.get("state"), archived: ev.target.checked ? "all" : "", filter: ftext }) }), " show archived");
  return h("div", {}, h("h1", {}, "Experiments"), h("div", { class: "toolbar" }, fbox, state, arch,
    h("span", { class: "muted" }, `${r.pagination.total} experiments`)), experimentTable(r.experiments));
}

function tabs(base, current, names) {
  return h("div", { class: "tabs" }, names.map((n) => h("a", { href: `${base}?tab=${n}`, class: n === current ? "on" : "" }, n)));
}

async function pageExperiment(params, id) {
  const tab = params.get("tab") || "overview";
  const { experiment: e } = await api.get(`/api/v1/experiments/${id}`);
  const head = h("div", {}, h("h1", {}, `Experiment ${e.id}: ${e.name || ""} `, badge(e.state)),
    h("div", { class: "toolbar" }, experimentActions(e), progressBar(e.progress),
      h("span", { class: "muted" }, `${e.searcher_type} searcher · pool ${e.resource_pool} · started ${fmtTime(e.start_time)}`)),
    tabs(`#/experiments/${id}`, tab, ["overview", "trials", "visualization", "checkpoints", "hyperparameters", "configuration", "notes"]));
  let body;
  if (tab === "overview" || tab === "trials") {
    const { trials } = await api.get(`/api/v1/experiments/${id}/trials`);
    const metric = (e.config.searcher || {}).metric;
    const hp = [...new Set(trials.flatMap((t) => Object.keys(t.hparams || {})))].filter((k) => typeof trials[0].hparams[k] !== "object");
    const cols = [
      { key: "id", label: "Trial", render: (t) => link("#/trials/" + t.id, t.id) },
      { key: "state", label: "State", render: (t) => badge(t.state) },
      { key: "best_validation", label: `Best ${metric || "validation"}`, sort: (t) => t.best_validation },
      { key: "steps_completed", label: "Batches" },
      { key: "restarts", label: "Restarts" },
      ...hp.slice(0, 6).map((k) => ({ key: "hp_" + k, label: k, sort: (t) => t.hparams[k], render: (t) => fmtNum(t.hparams[k]) })),
      { key: "start_time", label: "Started", render: (t) => fmtTime(t.start_time) },
    ];
    const parts = [];
    if (tab === "overview") {
      const vh = await api.get(`/api/v1/experiments/${id}/validation-history`);
      parts.push(h("div", { class: "charts" }, lineChart(`Best ${metric || "validation metric"} over time`,
        [{ name: metric, points: vh.validation_history.map((v) => [v.end_time - e.start_time, v.searcher_metric]) }], "seconds since start"),
      lineChart("Trials by best validation", [{ name: metric, points: trials.filter((t) => typeof t.best_validation === "number").map((t) => [t.id, t.best_validation]) }], "trial id")));
    }
    const picked = new Set();
    cols.unshift({ key: "pick", label: "", render: (t) => h("input", { type: "checkbox", class: "pick",
      onchange: (ev) => { if (ev.target.checked) picked.add(t.id); else picked.delete(t.id); } }) });
    const compare = h("button", { onclick: () => {
      if (picked.size < 1) { alert("select trials to compare"); return; }
      nav("#/compare", { trials: [...picked].sort((a, b) => a - b).join(",") });
    } }, "Compare selected");
    parts.push(h("h2", {}, "Trials"), h("div", { class: "toolbar" }, compare), table(cols, trials, { sortKey: "id", desc: false }));
    body = parts;
  } else if (tab === "visualization") {
    // hyperparameter search view: learning curves of up to 20 trials + metric vs each numeric hparam
    const { trials } = await api.get(`/api/v1/experiments/${id}/trials`);
    const metric = (e.config.searcher || {}).metric;
    const shown = trials.slice(0, 20);
    const curves = await Promise.all(shown.map((t) => api.get(`/api/v1/trials/${t.id}/metrics?group=validation`)
      .then((r) => ({ name: "trial " + t.id, points: r.metrics.filter((m) => typeof (m.metrics || {})[metric] === "number")
        .map((m) => [m.steps_completed, m.metrics[metric]]) })).catch(() => ({ name: "trial " + t.id, points: [] }))));
    const numeric = [...new Set(trials.flatMap((t) => Object.keys(t.hparams || {})))]
      .filter((k) => trials.some((t) => typeof (t.hparams || {})[k] === "number"));
    const scored = trials.filter((t) => typeof t.best_validation === "number");
    const hpKeys = [...new Set(trials.flatMap((t) => Object.keys(t.hparams || {})))]
      .filter((k) => trials.every((t) => (t.hparams || {})[k] !== undefined && typeof t.hparams[k] !== "object"))
      .filter((k) => new Set(trials.map((t) => JSON.stringify(t.hparams[k]))).size > 1);
    body = [h("div", { class: "charts" }, parallelCoords(`Hyperparameters → best ${metric}`, trials, hpKeys, metric,
      (e.config.searcher || {}).smaller_is_better)),
      h("div", { class: "charts" }, lineChart(`Validation ${metric} by trial`, curves, "batches")),
      h("h2", {}, `Best ${metric} vs hyperparameters`),
      numeric.length ? h("div", { class: "charts" }, numeric.map((k) => lineChart(k,
        [{ name: k, points: scored.filter((t) => typeof t.hparams[k] === "number").map((t) => [t.hparams[k], t.best_validation]) }],
        k, { scatter: true })))
        : h("div", { class: "muted" }, "no numeric hyperparameters")];
  } else if (tab === "checkpoints") {
    const { checkpoints } = await api.get(`/api/v1/experiments/${id}/checkpoints?sort_by=searcher_metric`);
    body = checkpointTable(checkpoints);
  } else if (tab === "hyperparameters") {
    body = h("pre", {}, JSON.stringify(e.config.hyperparameters, null, 2));
  } else if (tab === "configuration") {
    body = h("pre", {}, JSON.stringify(e.config, null, 2));
  } else {
    const ta = h("textarea", { rows: 14, style: "width:100%" }); ta.value = e.notes || "";
    body = h("div", { class: "card" }, ta, h("div", {}, h("button", { class: "primary",
      onclick: () => act(() => api.patch(`/api/v1/experiments/${id}`, { notes: ta.value })) }, "Save notes")));
  }
  return h("div", {}, head, body);
}

function checkpointTable(rows) {
  return table([
    { key: "uuid", label: "UUID", render: (c) => h("span", { class: "mono" }, c.uuid) },
    { key: "trial_id", label: "Trial", sort: (c) => c.training.trial_id, render: (c) => c.training.trial_id ? link("#/trials/" + c.training.trial_id, c.training.trial_id) : "-" },
    { key: "steps", label: "Batches", sort: (c) => c.training.steps_completed, render: (c) => fmtNum(c.training.steps_completed) },
    { key: "state", label: "State", render: (c) => badge(c.state) },
    { key: "val", label: "Validation", render: (c) => {
      const m = ((c.training || {}).validation_metrics || {}).avg_metrics || {};
      return Object.entries(m).slice(0, 3).map(([k, v]) => `${k}=${fmtNum(v)}`).join(" ");
    } },
    { key: "report_time", label: "Reported", render: (c) => fmtTime(c.report_time) },
    { key: "register", label: "", render: (c) => h("button", { onclick: () => registerCheckpoint(c.uuid) }, "Register") },
  ], rows, { sortKey: "report_time" });
}
async function registerCheckpoint(uuid) {
  const name = prompt("Register checkpoint in model (name):");
  if (!name) return;
  await act(async () => {
    try { await api.get(`/api/v1/models/${encodeURIComponent(name)}`); } catch (e) { await api.post("/api/v1/models", { name }); }
    await api.post(`/api/v1/models/${encodeURIComponent(name)}/versions`, { checkpoint_uuid: uuid });
  }, () => { location.hash = "#/models/" + encodeURIComponent(name); });
}

async function pageTrial(params, id) {
  const tab = params.get("tab") || "metrics";
  const { trial: t } = await api.get(`/api/v1/trials/${id}`);
  const head = h("div", {}, h("h1", {}, `Trial ${t.id} `, badge(t.state)),
    h("div", { class: "toolbar" }, link("#/experiments/" + t.experiment_id, `experiment ${t.experiment_id}`),
      h("span", { class: "muted" }, `batches ${t.steps_completed || 0} · restarts ${t.restarts || 0} · started ${fmtTime(t.start_time)}`),
      !["COMPLETED", "CANCELED", "ERROR"].includes(t.state) ? h("button", { onclick: () => act(() => api.post(`/api/v1/trials/${id}/kill`)) }, "Kill") : null),
    tabs(`#/trials/${id}`, tab, ["metrics", "workloads", "hyperparameters", "checkpoints", "logs", "profiler"]));
  let body;
  if (tab === "metrics") {
    const { metrics } = await api.get(`/api/v1/trials/${id}/metrics`);
    const groups = [...new Set(metrics.map((m) => m.group))];
    body = metricCharts(groups.map((g) => ({ name: g, rows: metrics.filter((m) => m.group === g) })));
  } else if (tab === "hyperparameters") {
    body = table([{ key: "k", label: "Hyperparameter" }, { key: "v", label: "Value", render: (r) => typeof r.v === "object" ? JSON.stringify(r.v) : fmtNum(r.v) }],
      Object.entries(t.hparams || {}).map(([k, v]) => ({ k, v })), { sortKey: "k", desc: false });
  } else if (tab === "checkpoints") {
    body = checkpointTable((await api.get(`/api/v1/trials/${id}/checkpoints`)).checkpoints);
  } else if (tab === "workloads") {
    body = await workloadsView(id, params.get("filter") || "");
  } else if (tab === "profiler") {
    body = await profilerView(id);
  } else {
    body = logView(`/api/v1/trials/${id}/logs`);
  }
  return h("div", {}, head, body);
}

// Workloads tab (reference TrialDetailsWorkloads): training / validation / checkpoint rows in
// batch order with their metrics; filter to validations or checkpoints.
async function workloadsView(id, filter) {
  const q = filter ? "?filter=FILTER_OPTION_" + filter : "";
  const { workloads } = await api.get(`/api/v1/trials/${id}/workloads` + q);
  const rows = workloads.map((w, i) => {
    const kind = Object.keys(w)[0], x = w[kind];
    const m = ((x.metrics || {}).avg_metrics) || {};
    return { i, kind, batches: x.total_batches, end_time: x.end_time,
      detail: kind === "checkpoint" ? `${x.uuid} (${(x.state || "").replace(/^STATE_/, "")})`
        : Object.entries(m).filter(([, v]) => typeof v === "number").map(([k, v]) => `${k}=${fmtNum(v)}`).join("  ") };
  });
  const sel = h("select", { onchange: (ev) => nav(`#/trials/${id}`, { tab: "workloads", filter: ev.target.value }) },
    [["", "all workloads"], ["VALIDATION", "validations"], ["CHECKPOINT", "checkpoints"]].map(([v, l]) =>
      h("option", { value: v, selected: v === filter }, l)));
  return h("div", {}, h("div", { class: "toolbar" }, sel, h("span", { class: "muted" }, `${rows.length} workloads`)),
    table([
      { key: "kind", label: "Type", render: (r) => badge(r.kind.toUpperCase()) },
      { key: "batches", label: "Batches" },
      { key: "detail", label: "Metrics / checkpoint", render: (r) => h("span", { class: "mono" }, r.detail) },
      { key: "end_time", label: "Finished", render: (r) => fmtTime(r.end_time) },
    ], rows, { sortKey: "i", desc: false }));
}

// Trial comparison (reference TrialsComparisonModal): hyperparameters side by side, the latest
// summary of each metric, and every metric's curves overlaid, one series per trial.
async function pageCompare(params) {
  const ids = (params.get("trials") || "").split(",").filter((x) => /^\d+$/.test(x));
  if (!ids.length) return h("div", { class: "muted" }, "no trials selected");
  const q = ids.map((i) => "trial_ids=" + i).join("&");
  const { trials } = await api.get(`/api/v1/trials/time-series?${q}`);
  const hpKeys = [...new Set(trials.flatMap((x) => Object.keys(x.trial.hparams || {})))].sort();
  const hpRows = hpKeys.map((k) => {
    const vals = trials.map((x) => (x.trial.hparams || {})[k]);
    const differs = new Set(vals.map((v) => JSON.stringify(v))).size > 1;
    return h("tr", { class: differs ? "differs" : "" }, h("td", {}, k),
      vals.map((v) => h("td", {}, typeof v === "object" ? JSON.stringify(v) : fmtNum(v))));
  });
  const series = [...new Set(trials.flatMap((x) => Object.keys(x.metrics)))].sort();
  const last = (pts) => (pts && pts.length ? pts[pts.length - 1].value : undefined);
  const sumRows = [
    h("tr", {}, h("td", {}, "state"), trials.map((x) => h("td", {}, badge(x.trial.state)))),
    h("tr", {}, h("td", {}, "batches"), trials.map((x) => h("td", {}, fmtNum(x.trial.steps_completed)))),
    h("tr", {}, h("td", {}, "best validation"), trials.map((x) => h("td", {}, fmtNum(x.trial.best_validation)))),
    ...series.map((sname) => h("tr", {}, h("td", {}, sname), trials.map((x) => h("td", {}, fmtNum(last(x.metrics[sname])))))),
  ];
  const headRow = h("tr", {}, h("th", {}, ""), trials.map((x) => h("th", {}, link("#/trials/" + x.trial.id, "trial " + x.trial.id))));
  const charts = series.map((sname) => lineChart(sname, trials.map((x) => ({
    name: "trial " + x.trial.id,
    points: (x.metrics[sname] || []).filter((p) => typeof p.value === "number").map((p) => [p.steps_completed, p.value]),
  })), "batches"));
  return h("div", {}, h("h1", {}, `Compare trials ${ids.join(", ")}`),
    h("h2", {}, "Hyperparameters"), h("table", { class: "compare" }, h("thead", {}, headRow.cloneNode(true)), h("tbody", {}, hpRows)),
    h("h2", {}, "Latest metrics"), h("table", { class: "compare" }, h("thead", {}, headRow), h("tbody", {}, sumRows)),
    h("h2", {}, "Curves"), h("div", { class: "charts" }, charts));
}

// Profiler tab (reference TrialDetailsProfiles): system metrics vs seconds since the first
// sample, one line per GPU / agent; loop timings and samples/s vs batch, one line per timing.
async function profilerView(id) {
  const [{ labels }, { batches }] = await Promise.all([
    api.get(`/api/v1/trials/${id}/profiler/available_series`), api.get(`/api/v1/trials/${id}/profiler/metrics`)]);
  if (!batches.length) return h("div", { class: "muted" }, "no profiler data (set profiling.enabled in the experiment config)");
  const t0 = Math.min(...batches.flatMap((b) => b.timestamps.map((t) => Date.parse(t))));
  const byType = (ty) => batches.filter((b) => b.labels.metricType === ty);
  const sys = byType("PROFILER_METRIC_TYPE_SYSTEM");
  const names = [...new Set(sys.map((b) => b.labels.name))].sort();
  const sysCharts = names.map((n) => lineChart(n, sys.filter((b) => b.labels.name === n).map((b) => ({
    name: b.labels.gpuUuid ? `gpu ${b.labels.gpuUuid}` : (b.labels.agentId || "agent"),
    points: b.values.map((v, i) => [(Date.parse(b.timestamps[i]) - t0) / 1000, v]),
  })), "seconds"));
  const timing = byType("PROFILER_METRIC_TYPE_TIMING");
  const timingChart = lineChart("timings (s)", timing.map((b) => ({
    name: b.labels.name, points: b.values.map((v, i) => [b.batches[i], v]) })), "batch");
  const misc = byType("PROFILER_METRIC_TYPE_MISC").map((b) => lineChart(b.labels.name, [{
    name: b.labels.name, points: b.values.map((v, i) => [b.batches[i], v]) }], "batch"));
  const summary = table([{ key: "metricType", label: "Type" }, { key: "name", label: "Series" },
    { key: "gpuUuid", label: "GPU" }, { key: "agentId", label: "Agent" }], labels, { sortKey: "metricType", desc: false });
  return h("div", {}, h("h2", {}, "Timings"), h("div", { class: "charts" }, timingChart, ...misc),
    h("h2", {}, "System metrics"), h("div", { class: "charts" }, ...sysCharts), h("h2", {}, "Series"), summary);
}

// incremental log tail with follow; stops when the page changes
function logView(path) {
  const pre = h("pre", {}, "");
  let after = 0, alive = true, page = location.hash;
  const tick = async () => {
    if (!alive || location.hash !== page) return;
    try {
      const r = await api.get(`${path}?after_id=${after}`);
      const atBottom = pre.scrollTop + pre.clientHeight >= pre.scrollHeight - 20;
      for (const l of r.logs) {
        after = Math.max(after, l.id);
        pre.appendChild(document.createTextNode((l.rank_id !== null && l.rank_id !== undefined ? `[rank=${l.rank_id}] ` : "") + l.log.replace(/\n?$/, "\n")));
      }
      if (atBottom) pre.scrollTop = pre.scrollHeight;
      if (r.done && !r.logs.length) alive = false;
    } catch (e) { alive = false; pre.appendChild(document.createTextNode("\n[" + e.message + "]\n")); }
    if (alive) setTimeout(tick, 2000);
  };
  tick();
  return pre;
}

async function pageCluster() {
  const [{ agents }, { resource_pools }] = await Promise.all([api.get("/api/v1/agents"), api.get("/api/v1/resource-pools")]);
  const pools = table([
    { key: "name", label: "Pool" }, { key: "slot_type", label: "Type" }, { key: "num_agents", label: "Agents" },
    { key: "slots_used", label: "Slots used", render: (p) => `${p.slots_used} / ${p.slots_available}` },
    { key: "scheduler_type", label: "Scheduler", render: (p) => `${p.scheduler_type} (${p.scheduler_fitting_policy})` },
  ], resource_pools, { sortKey: "name", desc: false });
  const ag = table([
    { key: "id", label: "Agent" }, { key: "resource_pool", label: "Pool" },
    { key: "slots", label: "Slots", sort: (a) => Object.keys(a.slots).length, render: (a) => h("div", { class: "slots" },
      Object.values(a.slots).map((s) => h("div", { class: "slot" + (s.container ? " used" : "") + (s.enabled ? "" : " off"),
        title: `${s.device.brand || s.device.type || ""} ${s.device.uuid || ""}${s.container ? " · " + s.container.id : ""}` }))) },
    { key: "enabled", label: "State", render: (a) => a.draining ? badge("DRAINING") : a.enabled ? badge("ENABLED") : badge("DISABLED") },
    { key: "last_seen", label: "Last seen", render: (a) => fmtTime(a.last_seen) },
    { key: "act", label: "", render: (a) => a.enabled
      ? h("button", { onclick: () => act(() => api.post(`/api/v1/agents/${a.id}/disable`, { drain: true })) }, "Drain")
      : h("button", { onclick: () => act(() => api.post(`/api/v1/agents/${a.id}/enable`)) }, "Enable") },
  ], agents, { sortKey: "id", desc: false });
  return h("div", {}, h("h1", {}, "Cluster"), h("h2", {}, "Resource pools"), pools, h("h2", {}, "Agents"), ag);
}

async function pageJobs() {
  const { jobs } = await api.get("/api/v1/job-queues");
  const prio = (j) => h("button", { onclick: () => {
    const p = prompt(`New priority for ${j.name || j.job_id}:`, j.priority);
    if (p !== null) act(() => api.post("/api/v1/job-queues", { updates: [{ job_id: j.job_id, priority: parseInt(p, 10) }] }));
  } }, "Priority");
  return h("div", {}, h("h1", {}, "Job Queue"), table([
    { key: "position", label: "#" }, { key: "job_id", label: "Job", render: (j) => taskLink(j.job_id, j.name) },
    { key: "state", label: "State", render: (j) => badge(j.state) }, { key: "slots", label: "Slots" },
    { key: "priority", label: "Priority" }, { key: "weight", label: "Weight" }, { key: "resource_pool", label: "Pool" },
    { key: "submission_time", label: "Submitted", render: (j) => fmtTime(j.submission_time) }, { key: "act", label: "", render: prio },
  ], jobs, { sortKey: "position", desc: false }));
}
function taskLink(id, name) {
  const m = /^exp-(\d+)$/.exec(id) || /^(\d+)\./.exec(id);
  return m ? link("#/experiments/" + m[1], name || id) : link(`#/tasks/${encodeURIComponent(id)}/logs`, name || id);
}

const NTSC = [["commands", "COMMAND"], ["notebooks", "NOTEBOOK"], ["shells", "SHELL"], ["tensorboards", "TENSORBOARD"]];
async function pageTasks() {
  const lists = await Promise.all(NTSC.map(([p]) => api.get("/api/v1/" + p)));
  const rows = lists.flatMap((l, i) => l[NTSC[i][0]].map((t) => Object.assign({ kind: NTSC[i][0] }, t)));
  const open = (t) => h("button", { onclick: () => window.open(`/proxy/${t.task_id}/?token=${encodeURIComponent(api.token)}`, "_blank") }, "Open");
  const launch = (p, body) => act(() => api.post("/api/v1/" + p, body));
  return h("div", {}, h("h1", {}, "Tasks"),
    h("div", { class: "toolbar" },
      h("button", { class: "primary", onclick: () => launch("notebooks", { config: { resources: { slots: 1 } } }) }, "Launch JupyterLab-style notebook"),
      h("button", { onclick: () => launch("notebooks", { config: { resources: { slots: 0 } } }) }, "Launch CPU notebook"),
      h("button", { onclick: () => {
        const ids = prompt("TensorBoard for experiment ids (comma separated):");
        if (ids) launch("tensorboards", { experiment_ids: ids.split(",").map((s) => parseInt(s, 10)).filter((x) => !isNaN(x)) });
      } }, "Launch TensorBoard")),
    table([
      { key: "task_id", label: "Task", render: (t) => h("span", { class: "mono" }, t.task_id) },
      { key: "type", label: "Type" }, { key: "name", label: "Name", render: (t) => t.name || "-" },
      { key: "state", label: "State", render: (t) => badge(t.state) }, { key: "slots", label: "Slots" },
      { key: "act", label: "", render: (t) => [
        ["notebooks", "shells", "tensorboards"].includes(t.kind) && !["TERMINATED", "COMPLETED"].includes(t.state) ? open(t) : null,
        link(`#/tasks/${encodeURIComponent(t.task_id)}/logs`, "Logs"), " ",
        h("button", { onclick: () => act(() => api.post(`/api/v1/${t.kind}/${t.task_id}/kill`)) }, "Kill")] },
    ], rows, { sortKey: "task_id" }));
}
async function pageTaskLogs(params, id) {
  const tid = decodeURIComponent(id);
  return h("div", {}, h("h1", {}, "Task logs: ", h("span", { class: "mono" }, tid)), logView(`/api/v1/tasks/${encodeURIComponent(tid)}/logs`));
}

async function pageModels(params) {
  const { models } = await api.get("/api/v1/models" + (params.get("archived") === "all" ? "" : "?archived=false"));
  const name = h("input", { placeholder: "new model name" });
  return h("div", {}, h("h1", {}, "Model Registry"),
    h("div", { class: "toolbar" }, name, h("button", { class: "primary", onclick: () => name.value && act(() => api.post("/api/v1/models", { name: name.value })) }, "Create model")),
    table([
      { key: "name", label: "Name", render: (m) => link("#/models/" + encodeURIComponent(m.name), m.name) },
      { key: "description", label: "Description", render: (m) => m.description || "" },
      { key: "num_versions", label: "Versions" }, { key: "labels", label: "Labels", render: (m) => (m.labels || []).join(", ") },
      { key: "last_updated_time", label: "Updated", render: (m) => fmtTime(m.last_updated_time) },
      { key: "act", label: "", render: (m) => h("button", { onclick: () => act(() => api.post(`/api/v1/models/${encodeURIComponent(m.name)}/${m.archived ? "unarchive" : "archive"}`)) }, m.archived ? "Unarchive" : "Archive") },
    ], models, { sortKey: "last_updated_time" }));
}
async function pageModel(params, name) {
  const n = decodeURIComponent(name);
  const r = await api.get(`/api/v1/models/${encodeURIComponent(n)}/versions`);
  const desc = h("input", { value: r.model.description || "", style: "width:420px" });
  return h("div", {}, h("h1", {}, "Model: " + n),
    h("div", { class: "toolbar" }, desc, h("button", { onclick: () => act(() => api.patch(`/api/v1/models/${encodeURIComponent(n)}`, { description: desc.value })) }, "Save description")),
    h("h2", {}, "Versions"),
    table([
      { key: "version", label: "Version" }, { key: "name", label: "Name", render: (v) => v.name || "-" },
      { key: "ck", label: "Checkpoint", render: (v) => h("span", { class: "mono" }, v.checkpoint.uuid) },
      { key: "trial", label: "Trial", render: (v) => { const t = (v.checkpoint.training || {}).trial_id; return t ? link("#/trials/" + t, t) : "-"; } },
      { key: "comment", label: "Comment", render: (v) => v.comment || "" },
      { key: "creation_time", label: "Created", render: (v) => fmtTime(v.creation_time) },
      { key: "act", label: "", render: (v) => h("button", { onclick: () => confirm(`Delete version ${v.version}?`) && act(() => api.del(`/api/v1/models/${encodeURIComponent(n)}/versions/${v.version}`)) }, "Delete") },
    ], r.model_versions, { sortKey: "version" }));
}

async function pageWorkspaces() {
  const { workspaces } = await api.get("/api/v1/workspaces");
  const name = h("input", { placeholder: "new workspace name" });
  return h("div", {}, h("h1", {}, "Workspaces"),
    h("div", { class: "toolbar" }, name, h("button", { class: "primary", onclick: () => name.value && act(() => api.post("/api/v1/workspaces", { name: name.value })) }, "Create workspace")),
    table([
      { key: "name", label: "Name", render: (w) => link("#/workspaces/" + w.id, w.name) },
      { key: "num_projects", label: "Projects" }, { key: "pinned", label: "Pinned", render: (w) => w.pinned ? "yes" : "" },
      { key: "archived", label: "Archived", render: (w) => w.archived ? "yes" : "" },
      { key: "default_compute_pool", label: "Default pool", render: (w) => w.default_compute_pool || "-" },
    ], workspaces, { sortKey: "name", desc: false }));
}
async function pageWorkspace(params, id) {
  const [{ workspace: w }, { projects }] = await Promise.all([api.get(`/api/v1/workspaces/${id}`), api.get(`/api/v1/workspaces/${id}/projects`)]);
  const name = h("input", { placeholder: "new project name" });
  return h("div", {}, h("h1", {}, "Workspace: " + w.name),
    h("div", { class: "toolbar" }, name, h("button", { class: "primary", onclick: () => name.value && act(() => api.post(`/api/v1/workspaces/${id}/projects`, { name: name.value })) }, "Create project"),
      h("button", { onclick: () => act(() => api.post(`/api/v1/workspaces/${id}/${w.pinned ? "unpin" : "pin"}`)) }, w.pinned ? "Unpin" : "Pin")),
    table([
      { key: "name", label: "Project", render: (p) => link("#/projects/" + p.id, p.name) },
      { key: "description", label: "Description", render: (p) => p.description || "" },
      { key: "num_experiments", label: "Experiments" }, { key: "archived", label: "Archived", render: (p) => p.archived ? "yes" : "" },
    ], projects, { sortKey: "name", desc: false }));
}
async function pageProject(params, id) {
  const [{ project: p }, exps] = await Promise.all([api.get(`/api/v1/projects/${id}`), api.get(`/api/v1/experiments?project_id=${id}`)]);
  const notes = (p.notes || []).map((n) => h("div", { class: "card" }, h("b", {}, n.name), h("pre", {}, n.contents)));
  return h("div", {}, h("h1", {}, "Project: " + p.name), h("div", { class: "muted" }, p.description || ""),
    link("#/workspaces/" + p.workspace_id, "back to workspace"), h("h2", {}, "Experiments"), experimentTable(exps.experiments),
    notes.length ? [h("h2", {}, "Notes"), notes] : null);
}

async function pageWebhooks() {
  const { webhooks } = await api.get("/api/v1/webhooks");
  const url = h("input", { placeholder: "https://…", style: "width:320px" });
  const type = h("select", {}, h("option", {}, "DEFAULT"), h("option", {}, "SLACK"));
  const states = h("input", { placeholder: "trigger states, e.g. COMPLETED,ERROR", style: "width:260px" });
  const regex = h("input", { placeholder: "task log regex (optional)", style: "width:200px" });
  const create = () => act(() => api.post("/api/v1/webhooks", { url: url.value, webhook_type: type.value,
    triggers: states.value.split(",").map((s) => s.trim()).filter(Boolean).map((s) => ({ trigger_type: "TRIGGER_TYPE_EXPERIMENT_STATE_CHANGE", condition: { state: s } }))
      .concat(regex.value ? [{ trigger_type: "TRIGGER_TYPE_TASK_LOG", condition: { regex: regex.value } }] : []) }));
  return h("div", {}, h("h1", {}, "Webhooks"), h("div", { class: "toolbar" }, url, type, states, regex, h("button", { class: "primary", onclick: create }, "Create")),
    table([
      { key: "id", label: "ID" }, { key: "url", label: "URL" }, { key: "webhook_type", label: "Type" },
      { key: "triggers", label: "Triggers", render: (w) => (w.triggers || []).map((t) => (t.condition || {}).state || ((t.condition || {}).regex ? "log /" + t.condition.regex + "/" : t.trigger_type)).join(", ") },
      { key: "act", label: "", render: (w) => [h("button", { onclick: () => act(() => api.post(`/api/v1/webhooks/${w.id}/test`)) }, "Test"),
        h("button", { onclick: () => act(() => api.del(`/api/v1/webhooks/${w.id}`)) }, "Delete")] },
    ], webhooks, { sortKey: "id", desc: false }));
}

async function pageClusterLogs() {
  const pre = h("pre", {}, "");
  let after = 0, page = location.hash;
  const tick = async () => {
    if (location.hash !== page) return;
    try {
      const r = await api.get(`/api/v1/master/logs?after_id=${after}` + (after ? "" : "&tail=500"));
      for (const l of r.logs) { after = Math.max(after, l.id); pre.appendChild(document.createTextNode(`${fmtTime(l.timestamp)} ${l.level} ${l.message}\n`)); }
      if (r.logs.length) pre.scrollTop = pre.scrollHeight;
      setTimeout(tick, 3000);
    } catch (e) { pre.appendChild(document.createTextNode("[" + e.message + "]\n")); }
  };
  tick();
  return h("div", {}, h("h1", {}, "Cluster Logs"), pre);
}

async function pageUsers() {
  const { users } = await api.get("/api/v1/users");
  const name = h("input", { placeholder: "username" });
  const admin = h("input", { type: "checkbox" });
  return h("div", {}, h("h1", {}, "Users"),
    h("div", { class: "toolbar" }, name, h("label", {}, admin, " admin"),
      h("button", { class: "primary", onclick: () => name.value && act(() => api.post("/api/v1/users", { user: { username: name.value, admin: admin.checked, active: true } })) }, "Add user")),
    table([
      { key: "id", label: "ID" }, { key: "username", label: "Username" }, { key: "display_name", label: "Display name", render: (u) => u.display_name || "" },
      { key: "admin", label: "Admin", render: (u) => u.admin ? "yes" : "" }, { key: "active", label: "Active", render: (u) => u.active ? "yes" : "no" },
      { key: "act", label: "", render: (u) => h("button", { onclick: () => act(() => api.patch(`/api/v1/users/${u.id}`, { active: !u.active })) }, u.active ? "Deactivate" : "Activate") },
    ], users, { sortKey: "id", desc: false }));
}

// ------------------------------------------------------------------------------------ router
const ROUTES = [
  [/^\/login$/, pageLogin, false],
  [/^\/?$/, pageDashboard, true],
  [/^\/experiments$/, pageExperiments, true],
  [/^\/experiments\/(\d+)$/, pageExperiment, true],
  [/^\/trials\/(\d+)$/, pageTrial, false],
  [/^\/compare$/, pageCompare, false],
  [/^\/cluster$/, pageCluster, true],
  [/^\/jobs$/, pageJobs, true],
  [/^\/tasks$/, pageTasks, true],
  [/^\/tasks\/([^/]+)\/logs$/, pageTaskLogs, false],
  [/^\/models$/, pageModels, false],
  [/^\/models\/([^/]+)$/, pageModel, false],
  [/^\/workspaces$/, pageWorkspaces, false],
  [/^\/workspaces\/(\d+)$/, pageWorkspace, false],
  [/^\/projects\/(\d+)$/, pageProject, false],
  [/^\/webhooks$/, pageWebhooks, false],
  [/^\/logs$/, pageClusterLogs, false],
  [/^\/admin\/users$/, pageUsers, false],
];
function nav(path, params) {
  const q = new URLSearchParams();
  for (const [k, v] of Object.entries(params || {})) if (v) q.set(k, v);
  location.hash = path + (q.toString() ? "?" + q : "");
}
let refreshTimer = null, generation = 0;
async function render() {
  clearTimeout(refreshTimer);
  const raw = location.hash.replace(/^#/, "") || "/";
  const [path, qs] = raw.split("?");
  const params = new URLSearchParams(qs || "");
  if (!api.token && path !== "/login") { location.hash = "#/login?next=" + encodeURIComponent(location.hash || "#/"); return; }
  document.querySelectorAll("#nav a").forEach((a) => {
    const target = a.getAttribute("href").slice(1);
    a.classList.toggle("active", target === "/" ? path === "/" : path.startsWith(target));
  });
  const user = localStorage.getItem("det_user");
  document.getElementById("who").replaceChildren(api.token ? h("span", {}, user || "", " · ",
    h("a", { href: "#/login", onclick: () => { api.post("/api/v1/auth/logout").catch(() => {}); localStorage.removeItem("det_token"); } }, "sign out")) : "");
  const main = document.getElementById("main");
  const gen = ++generation;
  for (const [rx, page, live] of ROUTES) {
    const m = rx.exec(path);
    if (!m) continue;
    try {
      const el = await page(params, ...m.slice(1));
      if (gen !== generation) return;  // a newer navigation won
      main.replaceChildren(el);
    } catch (e) {
      if (gen === generation) main.replaceChildren(errBox(e));
    }
    // live pages refresh in place while nothing is being edited
    if (live) refreshTimer = setTimeout(() => {
      const a = document.activeElement;
      if (gen === generation && !(a && ["INPUT", "TEXTAREA", "SELECT"].includes(a.tagName))) render();
      else if (gen === generation) refreshTimer = setTimeout(render, 5000);
    }, 5000);
    return;
  }
  main.replaceChildren(h("h1", {}, "Not found"));
}
window.addEventListener("hashchange", render);
render();
