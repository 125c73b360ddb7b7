"""Master REST API load test (reference: ``performance/src/api_performance_tests.ts``, a k6
script run nightly against a seeded cluster).

Same shape, no k6/node dependency: every virtual user (a thread with its own session) walks the
read-mostly endpoint groups the web UI and CLI hit -- master/agents/workspaces/pools, users and
login, models, NTSC lists, job queues, projects, experiments search / metric streams / file tree,
trials, tasks and their logs, master logs, resource allocation -- then sleeps 1 s; the number of
users follows ramping stages (k6 ``ramping-vus``). Thresholds as in the reference: p95 latency
< 1000 ms overall and per group, failure rate < 5 % (aborts the run when crossed).

Seeding: ``--seed`` creates an experiment with a finished trial (training + validation metrics),
a registered model version and a task log, the data the reference passes in by environment
(``experiment_id``, ``trial_id``, ``model_name`` ...). Writes a text summary to stdout, and
``--junit``/``--json`` reports.

    python tools/api_load_test.py -m http://127.0.0.1:8080 --seed \
        --stages 60s:25,120s:25,60s:0 --junit results.xml
"""
import argparse
import json
import os
import sys
import threading
import time
import uuid
from typing import Any, Callable, Dict, List, Optional, Tuple
from xml.sax.saxutils import escape

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from determined_clone_amd.common.api import Session  # noqa: E402


def parse_stages(spec: str) -> List[Tuple[float, int]]:
    """``"5m:25,10m:25,5m:0"`` -> [(300.0, 25), (600.0, 25), (300.0, 0)]."""
    out = []
    for part in spec.split(","):
        dur, target = part.split(":")
        mult = {"s": 1.0, "m": 60.0, "h": 3600.0}.get(dur[-1], None)
        secs = float(dur[:-1]) * mult if mult else float(dur)
        out.append((secs, int(target)))
    return out


def target_at(stages: List[Tuple[float, int]], t: float) -> int:
    """Linear ramp between stage targets, like k6's ramping-vus executor (starts from 0)."""
    prev = 0
    for dur, tgt in stages:
        if t < dur:
            return int(round(prev + (tgt - prev) * (t / dur if dur > 0 else 1.0)))
        t -= dur
        prev = tgt
    return -1  # finished


def seed(s: Session) -> Dict[str, Any]:
    """An experiment with one finished trial + metrics, a model version, task logs."""
    cfg = {"name": "load-test-seed", "entrypoint": "model_def:T", "searcher": {
        "name": "single", "metric": "val_loss", "max_length": {"batches": 100}},
        "hyperparameters": {"lr": 0.1}}
    eid = s.post("/api/v1/experiments", {"config": cfg, "unmanaged": True})["experiment"]["id"]
    trial = s.post("/api/v1/trials", {"experiment_id": eid, "hparams": {"lr": 0.1},
                                      "unmanaged": True})["trial"]
    tid, task_id = trial["id"], trial["taskId"]
    for b in (25, 50, 75, 100):
        s.post(f"/api/v1/trials/{tid}/metrics", {"metrics": {
            "trial_id": tid, "steps_completed": b, "avg_metrics": {"loss": 1.0 / b}}, "group": "training"})
    s.post(f"/api/v1/trials/{tid}/metrics", {"metrics": {
        "trial_id": tid, "steps_completed": 100, "avg_metrics": {"val_loss": 0.5}}, "group": "validation"})
    name = f"load-model-{uuid.uuid4().hex[:6]}"
    s.post("/api/v1/models", {"name": name, "labels": ["load"]})
    ck = str(uuid.uuid4())
    s.post("/api/v1/checkpoints", {
        "uuid": ck, "task_id": task_id, "allocation_id": f"{task_id}.1", "report_time": time.time(),
        "resources": {"state_dict.pth": 1}, "metadata": {"steps_completed": 100}, "state": "COMPLETED"})
    ver = s.post(f"/api/v1/models/{name}/versions", {"checkpoint_uuid": ck})["model_version"]["version"]
    s.post("/api/v1/task/logs", {"logs": [{"task_id": task_id, "log": f"line {i}\n", "level": "INFO"}
                                          for i in range(20)]})
    return {"experiment_id": eid, "trial_id": tid, "model_name": name, "model_version": ver,
            "task_id": task_id, "metric_name": "val_loss", "metric_type": "METRIC_TYPE_VALIDATION",
            "workspace_id": 1, "project_id": 1, "resource_pool": "default"}


def groups(sd: Dict[str, Any]) -> List[Tuple[str, str]]:
    """(group name, path) pairs; entries needing seeded ids are skipped when absent."""
    g = [("get master configuration", "/api/v1/master"), ("get agents", "/api/v1/agents"),
         ("get workspaces", "/api/v1/workspaces"), ("get user settings", "/api/v1/users/setting"),
         ("get resource pools", "/api/v1/resource-pools"), ("get users", "/api/v1/users"),
         ("get models", "/api/v1/models"), ("get tensorboards", "/api/v1/tensorboards"),
         ("get shells", "/api/v1/shells"), ("get notebooks", "/api/v1/notebooks"),
         ("get commands", "/api/v1/commands"), ("get job queue stats", "/api/v1/job-queues/stats"),
         ("get user activity", "/api/v1/user/projects/activity"), ("get webhooks", "/api/v1/webhooks"),
         ("get model labels", "/api/v1/model/labels"),
         ("get experiments", "/api/v1/experiments?showTrialData=true"),
         ("get master logs", "/api/v1/master/logs?offset=-1&limit=0"),
         ("get resource allocations", "/api/v1/resources/allocation/aggregated?startDate=2000-01-01"
          f"&endDate={time.strftime('%Y-%m-%d')}&period=RESOURCE_ALLOCATION_AGGREGATION_PERIOD_DAILY"),
         ("get tasks", "/api/v1/tasks"), ("get task count", "/api/v1/tasks/count")]
    ws, pj = sd.get("workspace_id", 1), sd.get("project_id", 1)
    g += [("get available resource pools", f"/api/v1/workspaces/{ws}/available-resource-pools"),
          ("get workspace projects", f"/api/v1/workspaces/{ws}/projects"),
          ("get project", f"/api/v1/projects/{pj}"),
          ("get project metric ranges", f"/api/v1/projects/{pj}/experiments/metric-ranges"),
          ("get project columns", f"/api/v1/projects/{pj}/columns"),
          ("search experiments", f"/api/v1/experiments-search?projectId={pj}"),
          ("get job queue", f"/api/v1/job-queues-v2?resourcePool={sd.get('resource_pool', 'default')}"),
          ("get workspace model labels", f"/api/v1/model/labels?workspaceId={ws}")]
    if sd.get("resource_pool"):
        g.append(("get pool bindings", f"/api/v1/resource-pools/{sd['resource_pool']}/workspace-bindings"))
    if sd.get("model_name"):
        g.append(("get model versions", f"/api/v1/models/{sd['model_name']}/versions"))
        if sd.get("model_version"):
            g.append(("get model version", f"/api/v1/models/{sd['model_name']}/versions/{sd['model_version']}"))
    if sd.get("trial_id"):
        t = sd["trial_id"]
        g += [("get trial", f"/api/v1/trials/{t}"), ("get trial workloads", f"/api/v1/trials/{t}/workloads"),
              ("get trial log fields", f"/api/v1/trials/{t}/logs/fields"),
              ("get trials time series", f"/api/v1/trials/time-series?trialIds={t}&startBatches=0"
               "&metricType=METRIC_TYPE_UNSPECIFIED")]
    if sd.get("experiment_id"):
        e = sd["experiment_id"]
        g += [("get experiment", f"/api/v1/experiments/{e}"),
              ("get experiment trials", f"/api/v1/experiments/{e}/trials"),
              ("get experiment file tree", f"/api/v1/experiments/{e}/file_tree"),
              ("get metric names", f"/api/v1/experiments/metrics-stream/metric-names?ids={e}")]
        if sd.get("metric_name") and sd.get("metric_type"):
            q = f"metricName={sd['metric_name']}&metricType={sd['metric_type']}"
            g += [("get experiment batches", f"/api/v1/experiments/{e}/metrics-stream/batches?{q}"),
                  ("get experiment trials sample", f"/api/v1/experiments/{e}/metrics-stream/trials-sample?{q}"),
                  ("get experiment trials snapshot", f"/api/v1/experiments/{e}/metrics-stream/trials-snapshot"
                   f"?{q}&batchesProcessed=100&batchesMargin=10")]
    if sd.get("task_id"):
        k = sd["task_id"]
        g += [("get task", f"/api/v1/tasks/{k}"), ("get task log fields", f"/api/v1/tasks/{k}/logs/fields"),
              ("get task logs", f"/api/v1/tasks/{k}/logs")]
    return g


class Stats:
    def __init__(self) -> None:
        self.lock = threading.Lock()
        self.lat: Dict[str, List[float]] = {}
        self.fail: Dict[str, int] = {}
        self.total = 0
        self.failed = 0
        self.errors: Dict[str, str] = {}

    def add(self, group: str, ms: float, ok: bool, err: str = "") -> None:
        with self.lock:
            self.lat.setdefault(group, []).append(ms)
            self.total += 1
            if not ok:
                self.failed += 1
                self.fail[group] = self.fail.get(group, 0) + 1
                self.errors.setdefault(group, err[:200])

    @staticmethod
    def pct(xs: List[float], p: float) -> float:
        if not xs:
            return 0.0
        ys = sorted(xs)
        return ys[min(len(ys) - 1, int(round(p / 100.0 * (len(ys) - 1))))]


def run(master: str, stages: List[Tuple[float, int]], sd: Dict[str, Any], login: Callable[[], Session],
        p95_ms: float = 1000.0, max_fail_rate: float = 0.05, think_s: float = 1.0) -> Dict[str, Any]:
    st = Stats()
    gs = groups(sd)
    stop = threading.Event()
    aborted = threading.Event()
    users: List[Tuple[threading.Thread, threading.Event]] = []

    def vu(quit_ev: threading.Event) -> None:
        s = login()
        while not (quit_ev.is_set() or stop.is_set()):
            for name, path in gs:
                if quit_ev.is_set() or stop.is_set():
                    return
                t0 = time.perf_counter()
                try:
                    s.get(path)
                    st.add(name, (time.perf_counter() - t0) * 1e3, True)
                except Exception as e:  # noqa: BLE001 - any failure counts against the threshold
                    st.add(name, (time.perf_counter() - t0) * 1e3, False, repr(e))
            t0 = time.perf_counter()
            try:
                Session(master).post("/api/v1/auth/login", {"username": "admin", "password": ""})
                st.add("login", (time.perf_counter() - t0) * 1e3, True)
            except Exception as e:  # noqa: BLE001
                st.add("login", (time.perf_counter() - t0) * 1e3, False, repr(e))
            quit_ev.wait(think_s)

    t_start = time.time()
    peak = 0
    while True:
        tgt = target_at(stages, time.time() - t_start)
        if tgt < 0:
            break
        alive = [u for u in users if not u[1].is_set()]
        while len(alive) < tgt:
            ev = threading.Event()
            th = threading.Thread(target=vu, args=(ev,), daemon=True)
            th.start()
            users.append((th, ev))
            alive.append((th, ev))
        while len(alive) > tgt:
            alive.pop()[1].set()
        peak = max(peak, tgt)
        with st.lock:
            if st.total >= 50 and st.failed / st.total > max_fail_rate:
                aborted.set()
        if aborted.is_set():
            break
        time.sleep(0.1)
    stop.set()
    for th, _ in users:
        th.join(timeout=30)
    all_lat = [x for xs in st.lat.values() for x in xs]
    per = {g: {"count": len(xs), "p50_ms": round(Stats.pct(xs, 50), 2), "p95_ms": round(Stats.pct(xs, 95), 2),
               "failed": st.fail.get(g, 0), "ok": Stats.pct(xs, 95) < p95_ms and not st.fail.get(g, 0),
               **({"error": st.errors[g]} if g in st.errors else {})}
           for g, xs in sorted(st.lat.items())}
    dur = time.time() - t_start
    fail_rate = st.failed / st.total if st.total else 0.0
    p95 = Stats.pct(all_lat, 95)
    return {"requests": st.total, "failed": st.failed, "fail_rate": round(fail_rate, 4),
            "duration_s": round(dur, 2), "rps": round(st.total / dur, 1) if dur else 0.0,
            "peak_vus": peak, "p50_ms": round(Stats.pct(all_lat, 50), 2), "p95_ms": round(p95, 2),
            "thresholds": {"http_req_duration p(95)<%g" % p95_ms: p95 < p95_ms,
                           "http_req_failed rate<%g" % max_fail_rate: fail_rate < max_fail_rate},
            "aborted": aborted.is_set(), "groups": per}


def text_summary(r: Dict[str, Any]) -> str:
    lines = [f"requests={r['requests']} failed={r['failed']} ({100 * r['fail_rate']:.2f}%) "
             f"rps={r['rps']} peak_vus={r['peak_vus']} p50={r['p50_ms']}ms p95={r['p95_ms']}ms "
             f"duration={r['duration_s']}s" + (" ABORTED" if r["aborted"] else "")]
    for k, ok in r["thresholds"].items():
        lines.append(f"  {'PASS' if ok else 'FAIL'} {k}")
    for g, d in r["groups"].items():
        lines.append(f"  {'ok  ' if d['ok'] else 'FAIL'} {g:<36} n={d['count']:<6} p50={d['p50_ms']:>8}ms "
                     f"p95={d['p95_ms']:>8}ms failed={d['failed']}")
    return "\n".join(lines)


def junit(r: Dict[str, Any]) -> str:
    cases = []
    for g, d in r["groups"].items():
        body = "" if d["ok"] else (f'<failure message="p95={d["p95_ms"]}ms failed={d["failed"]}">'
                                   f"{escape(d.get('error', ''))}</failure>")
        cases.append(f'<testcase name="{escape(g)}" time="{d["p50_ms"] / 1e3:.4f}">{body}</testcase>')
    nfail = sum(1 for d in r["groups"].values() if not d["ok"])
    return (f'<?xml version="1.0"?>\n<testsuites><testsuite name="API Load Tests" tests="{len(cases)}" '
            f'failures="{nfail}">' + "".join(cases) + "</testsuite></testsuites>\n")


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("-m", "--master", default=os.environ.get("DET_MASTER", "http://127.0.0.1:8080"))
    ap.add_argument("-u", "--user", default="admin")
    ap.add_argument("--password", default=os.environ.get("DET_PASS", ""))
    ap.add_argument("--stages", default="5m:25,10m:25,5m:0")
    ap.add_argument("--seed", action="store_true", help="create the experiment/trial/model/task data")
    ap.add_argument("--seeded", default=None, help="JSON of seeded ids (experiment_id, trial_id, ...)")
    ap.add_argument("--p95-ms", type=float, default=1000.0)
    ap.add_argument("--max-fail-rate", type=float, default=0.05)
    ap.add_argument("--think-s", type=float, default=1.0)
    ap.add_argument("--junit", default=None)
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)

    def login() -> Session:
        s = Session(a.master)
        s.token = s.post("/api/v1/auth/login", {"username": a.user, "password": a.password})["token"]
        return s

    sd: Dict[str, Any] = json.loads(a.seeded) if a.seeded else {}
    if a.seed:
        sd.update(seed(login()))
    r = run(a.master, parse_stages(a.stages), sd, login, a.p95_ms, a.max_fail_rate, a.think_s)
    r["seeded"] = sd
    print(text_summary(r))
    if a.junit:
        with open(a.junit, "w") as f:
            f.write(junit(r))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(r, f, indent=1)
    return 0 if all(r["thresholds"].values()) and not r["aborted"] else 1


if __name__ == "__main__":
    sys.exit(main())
