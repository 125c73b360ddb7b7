// Renders pages of the web UI (determined_clone_amd/webui/static/app.js) in node without a
// browser: a minimal DOM (elements, text nodes, SVG namespace, events ignored), localStorage,
// location and a fetch over node's http module against a live master. Prints one JSON object per
// route: the page's text, the number of elements per tag and any render error.
// Usage: node webui_render.js APP_JS MASTER_URL TOKEN ROUTE [ROUTE ...]   (ROUTE like "/compare?trials=1,2")
"use strict";
const fs = require("fs");
const http = require("http");
const vm = require("vm");

class Node_ {
  constructor() { this.childNodes = []; this.parentNode = null; }
  appendChild(c) { c.parentNode = this; this.childNodes.push(c); return c; }
  replaceChildren(...kids) { this.childNodes = []; for (const k of kids) this.appendChild(k); }
  get textContent() { return this.childNodes.map((c) => c.textContent).join(" "); }
  set textContent(v) { this.childNodes = [new Text_(String(v))]; }
  set innerHTML(v) { this.childNodes = []; }
}
class Text_ extends Node_ {
  constructor(t) { super(); this.text = t; }
  get textContent() { return this.text; }
  cloneNode() { return new Text_(this.text); }
}
class Element_ extends Node_ {
  constructor(tag) { super(); this.tagName = tag.toUpperCase(); this.attrs = {}; this.className = ""; this.style = {}; this.value = ""; }
  setAttribute(k, v) { this.attrs[k] = String(v); if (k === "value") this.value = String(v); }
  getAttribute(k) { return this.attrs[k]; }
  addEventListener() {}
  get classList() { return { toggle() {}, add() {}, remove() {} }; }
  querySelectorAll() { return []; }
  cloneNode(deep) {
    const e = new Element_(this.tagName);
    e.attrs = Object.assign({}, this.attrs); e.className = this.className;
    if (deep) for (const c of this.childNodes) e.appendChild(c.cloneNode(true));
    return e;
  }
}
const byId = {};
global.Node = Node_;
global.document = {
  createElement: (t) => new Element_(t),
  createElementNS: (ns, t) => new Element_(t),
  createTextNode: (t) => new Text_(t),
  getElementById: (id) => byId[id] || (byId[id] = new Element_("div")),
  querySelectorAll: () => [],
  activeElement: null,
};
const store = {};
global.localStorage = { getItem: (k) => (k in store ? store[k] : null), setItem: (k, v) => { store[k] = String(v); }, removeItem: (k) => { delete store[k]; } };
global.location = { hash: "#/__none__" };
global.window = { addEventListener() {} };
global.alert = (m) => { throw new Error("alert: " + m); };
global.prompt = () => null;

const [appJs, master, token, ...routes] = process.argv.slice(2);
store.det_token = token;
global.fetch = (path, opts) => new Promise((resolve, reject) => {
  const u = new URL(path, master);
  const req = http.request(u, { method: opts.method, headers: opts.headers }, (res) => {
    let body = "";
    res.on("data", (d) => { body += d; });
    res.on("end", () => resolve({ status: res.statusCode, ok: res.statusCode < 400, statusText: res.statusMessage,
      json: async () => JSON.parse(body) }));
  });
  req.on("error", reject);
  if (opts.body) req.write(opts.body);
  req.end();
});

// load the app; its top-level render() runs against "#/__none__" (Not found) harmlessly
vm.runInThisContext(fs.readFileSync(appJs, "utf8") + "\n;global.__app = { ROUTES, render };", { filename: "app.js" });

function census(el, out) {
  if (el instanceof Element_) out[el.tagName.toLowerCase()] = (out[el.tagName.toLowerCase()] || 0) + 1;
  for (const c of el.childNodes) census(c, out);
  return out;
}

(async () => {
  const results = [];
  for (const route of routes) {
    const [path, qs] = route.split("?");
    const params = new URLSearchParams(qs || "");
    const hit = global.__app.ROUTES.find(([rx]) => rx.test(path));
    const res = { route };
    try {
      if (!hit) throw new Error("no route");
      const el = await hit[1](params, ...hit[0].exec(path).slice(1));
      res.text = el.textContent.replace(/\s+/g, " ").slice(0, 4000);
      res.tags = census(el, {});
      res.trial_lines = [];
      (function walk(e) {
        if (e instanceof Element_ && e.tagName === "POLYLINE" && e.attrs["data-trial"]) res.trial_lines.push(+e.attrs["data-trial"]);
        for (const c of e.childNodes) walk(c);
      })(el);
    } catch (e) {
      res.error = String(e && e.stack || e);
    }
    results.push(res);
  }
  process.stdout.write(JSON.stringify(results) + "\n");
})();
