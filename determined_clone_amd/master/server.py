"""Master REST API (reference: `proto/src/determined/api/v1/api.proto` served by grpc-gateway,
handlers in `master/internal/api_*.go`). JSON over HTTP, ``/api/v1/...`` paths, bearer tokens.
Served by a threading HTTP server so long-polls (preemption signals, agent actions, log follow)
each hold their own thread."""
import base64
import json
import logging
import re
import ssl
import sys
import threading
import time
import http.cookies
import traceback
import urllib.error
import urllib.parse
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Callable, Dict, List, Optional, Tuple

from determined_clone_amd import __version__
from determined_clone_amd.errors import InvalidConfigurationException
from determined_clone_amd.master.core import Master, hash_password
from determined_clone_amd.master.db import dec, now
from determined_clone_amd.master.experiment import TERMINAL, experiment_row_to_api, trial_row_to_api
from determined_clone_amd.util import PROXY_SECRET_HEADER

logger = logging.getLogger("determined_clone_amd.master.api")
audit_logger = logging.getLogger("determined_clone_amd.master.audit")

Handler = Callable[..., Any]
ROUTES: List[Tuple[str, "re.Pattern[str]", Handler, bool]] = []


class HTTPError(Exception):
    def __init__(self, status: int, msg: str) -> None:
        self.status = status
        super().__init__(msg)


def route(method: str, pattern: str, auth: bool = True, first: bool = False) -> Callable[[Handler], Handler]:
    """Register a handler; ``first`` puts it ahead of earlier routes (a literal path such as
    ``/api/v1/tasks/count`` must win over ``/api/v1/tasks/{task_id}``)."""
    rx = re.compile("^" + re.sub(r"\{(\w+)\}", r"(?P<\1>[^/]+)", pattern) + "$")

    def deco(fn: Handler) -> Handler:
        if first:
            ROUTES.insert(0, (method, rx, fn, auth))
        else:
            ROUTES.append((method, rx, fn, auth))
        return fn

    return deco


class Req:
    def __init__(self, m: Master, params: Dict[str, str], query: Dict[str, List[str]], body: Any,
                 user: Optional[Dict[str, Any]]) -> None:
        self.m = m
        self.p = params
        self.q = query
        self.body = body if body is not None else {}
        self.user = user

    def qget(self, k: str, default: Any = None) -> Any:
        v = self.q.get(k)
        return v[0] if v else default

    def qlist(self, k: str) -> List[str]:
        return self.q.get(k, [])

    def require_admin(self) -> None:
        if not self.user or not self.user.get("admin"):
            raise HTTPError(403, "admin privileges required")


def require(r: Req, perm: str, workspace_id: Optional[int] = None) -> None:
    """403 unless the caller holds ``perm`` (cluster-wide or in ``workspace_id``); see
    ``master/rbac.py`` for the basic / rbac modes."""
    if not r.m.authz.permitted(r.user, perm, workspace_id):
        raise HTTPError(403, f"permission denied: {perm}" + (f" in workspace {workspace_id}" if workspace_id else ""))


def _project_workspace(m: Master, project_id: Optional[int]) -> int:
    row = m.db.one("SELECT workspace_id FROM projects WHERE id=?", [project_id or 1])
    return int(row["workspace_id"]) if row else 1


def _int(v: Any) -> int:
    try:
        return int(v)
    except (TypeError, ValueError):
        raise HTTPError(400, f"expected an integer, got {v!r}")


def _paginate(rows: List[Any], r: Req) -> Dict[str, Any]:
    off = _int(r.qget("offset", 0))
    lim = _int(r.qget("limit", 0))
    total = len(rows)
    sl = rows[off:off + lim] if lim > 0 else rows[off:]
    return {"items": sl, "pagination": {"offset": off, "limit": lim, "start_index": off,
                                        "end_index": off + len(sl), "total": total}}


# =========================================================================== auth / users / master
@route("POST", "/api/v1/auth/login", auth=False)
def login(r: Req) -> Any:
    try:
        token, user = r.m.login(r.body.get("username", ""), r.body.get("password", ""))
    except PermissionError as e:
        raise HTTPError(401, str(e))
    return {"token": token, "user": user}


@route("POST", "/api/v1/auth/logout")
def logout(r: Req) -> Any:
    return {}


@route("GET", "/api/v1/me")
def me(r: Req) -> Any:
    return {"user": Master.user_api(r.user)}


@route("GET", "/api/v1/users")
def users(r: Req) -> Any:
    return {"users": [Master.user_api(u) for u in r.m.db.all("SELECT * FROM users ORDER BY id")]}


@route("GET", "/api/v1/users/{uid}")
def get_user(r: Req) -> Any:
    u = r.m.db.one("SELECT * FROM users WHERE id=?", [_int(r.p["uid"])])
    if not u:
        raise HTTPError(404, "user not found")
    return {"user": Master.user_api(u)}


@route("POST", "/api/v1/users")
def post_user(r: Req) -> Any:
    require(r, "ADMINISTRATE_USER")
    u = r.body.get("user", r.body)
    if r.m.db.one("SELECT id FROM users WHERE username=?", [u["username"]]):
        raise HTTPError(409, "user already exists")
    uid = r.m.db.insert("users", {"username": u["username"], "admin": int(bool(u.get("admin"))),
                                  "active": int(u.get("active", True)), "display_name": u.get("display_name"),
                                  "password_hash": hash_password(r.body.get("password", "")), "created": now()})
    return {"user": Master.user_api(r.m.db.one("SELECT * FROM users WHERE id=?", [uid]))}


@route("PATCH", "/api/v1/users/{uid}")
def patch_user(r: Req) -> Any:
    uid = _int(r.p["uid"])
    if r.user["id"] != uid:
        r.require_admin()
    fields = {}
    for k in ("display_name", "username"):
        if k in r.body:
            fields[k] = r.body[k]
    for k in ("admin", "active"):
        if k in r.body:
            r.require_admin()
            fields[k] = int(bool(r.body[k]))
    if "password" in r.body:
        fields["password_hash"] = hash_password(r.body["password"])
    if "agent_user_group" in r.body:
        aug = r.body["agent_user_group"] or {}
        fields["agent_uid"] = aug.get("agent_uid")
        fields["agent_user"] = aug.get("agent_user")
    r.m.db.update("users", "id", uid, fields)
    return {"user": Master.user_api(r.m.db.one("SELECT * FROM users WHERE id=?", [uid]))}


@route("POST", "/api/v1/users/{uid}/password")
def set_password(r: Req) -> Any:
    uid = _int(r.p["uid"])
    if r.user["id"] != uid:
        r.require_admin()
    r.m.db.update("users", "id", uid, {"password_hash": hash_password(r.body.get("password", ""))})
    return {}


@route("GET", "/api/v1/master", auth=False)
def master_info(r: Req) -> Any:
    return {"version": __version__, "master_id": r.m.cluster_id, "cluster_id": r.m.cluster_id,
            "cluster_name": r.m.cluster_name, "telemetry_enabled": False,
            "sso_providers": list(getattr(r.m, "sso_providers", [])),
            "product": "determined_clone_amd", "uptime_s": time.time() - r.m.start_time}


@route("GET", "/api/v1/master/logs")
def master_logs(r: Req) -> Any:
    """MasterLogs: the master's own log records (ring buffer), after ``after_id`` or the last
    ``tail`` entries."""
    require(r, "VIEW_MASTER_LOGS")
    return {"logs": r.m.log_buffer.entries(_int(r.qget("after_id", 0)), _int(r.qget("tail", 0)))}


@route("GET", "/api/v1/master/config")
def master_config(r: Req) -> Any:
    require(r, "VIEW_MASTER_CONFIG")
    return {"config": {"scheduler": {"type": r.m.rm.policy, "fitting_policy": r.m.rm.fit,
                                     "preemption": r.m.rm.preemption},
                       "checkpoint_storage": r.m.checkpoint_storage}}


# =========================================================================== OAuth clients
# The reference's OAuth2 client registry (``/oauth2/clients``, used by SCIM provisioning) is an
# enterprise add-on: its OSS master answers 404 and the SDK raises EnterpriseOnlyError
# (harness/determined/common/experimental/determined.py:478-520). Here it is a small admin-only
# registry in the master's kv store: id + generated secret + redirect domain.
def _oauth_clients(m: Master) -> List[Dict[str, Any]]:
    return list(m.db.kv_get("oauth2_clients", []))


@route("GET", "/oauth2/clients")
def oauth_clients(r: Req) -> Any:
    r.require_admin()
    return [{"id": c["id"], "name": c["name"], "domain": c["domain"]} for c in _oauth_clients(r.m)]


@route("POST", "/oauth2/clients")
def oauth_client_add(r: Req) -> Any:
    r.require_admin()
    name, domain = r.body.get("name"), r.body.get("domain")
    if not name or not domain:
        raise HTTPError(400, "name and domain are required")
    import secrets as _secrets

    c = {"id": _secrets.token_hex(8), "secret": _secrets.token_hex(24), "name": str(name),
         "domain": str(domain)}
    r.m.db.kv_set("oauth2_clients", _oauth_clients(r.m) + [c])
    return {"id": c["id"], "secret": c["secret"]}


@route("DELETE", "/oauth2/clients/{cid}")
def oauth_client_remove(r: Req) -> Any:
    r.require_admin()
    cs = _oauth_clients(r.m)
    keep = [c for c in cs if c["id"] != r.p["cid"]]
    if len(keep) == len(cs):
        raise HTTPError(404, "oauth client not found")
    r.m.db.kv_set("oauth2_clients", keep)
    return {}


# =========================================================================== agents
@route("POST", "/api/v1/agents/register")
def agent_register(r: Req) -> Any:
    r.m.register_agent(r.body)
    return {}


@route("GET", "/api/v1/agents")
def agents(r: Req) -> Any:
    return {"agents": [a.to_dict() for a in r.m.rm.agents.values()]}


@route("GET", "/api/v1/agents/{aid}")
def agent(r: Req) -> Any:
    a = r.m.rm.agents.get(r.p["aid"])
    if a is None:
        raise HTTPError(404, "agent not found")
    return {"agent": a.to_dict()}


@route("POST", "/api/v1/agents/{aid}/enable")
def agent_enable(r: Req) -> Any:
    require(r, "UPDATE_AGENTS")
    r.m.rm.set_agent_enabled(r.p["aid"], True)
    return {}


@route("POST", "/api/v1/agents/{aid}/disable")
def agent_disable(r: Req) -> Any:
    require(r, "UPDATE_AGENTS")
    r.m.rm.set_agent_enabled(r.p["aid"], False, drain=bool(r.body.get("drain")))
    return {}


@route("POST", "/api/v1/agents/{aid}/slots/{sid}/enable")
def slot_enable(r: Req) -> Any:
    require(r, "UPDATE_AGENTS")
    r.m.rm.set_slot_enabled(r.p["aid"], _int(r.p["sid"]), True)
    return {}


@route("POST", "/api/v1/agents/{aid}/slots/{sid}/disable")
def slot_disable(r: Req) -> Any:
    require(r, "UPDATE_AGENTS")
    r.m.rm.set_slot_enabled(r.p["aid"], _int(r.p["sid"]), False)
    return {}


@route("GET", "/api/v1/agents/{aid}/actions")
def agent_actions(r: Req) -> Any:
    a = r.m.rm.agents.get(r.p["aid"])
    if a is None:
        raise HTTPError(404, "agent not registered")
    a.last_seen = time.time()
    return {"actions": a.pop_all(float(r.qget("timeout_seconds", 20)))}


@route("POST", "/api/v1/agents/{aid}/events")
def agent_events(r: Req) -> Any:
    for ev in r.body.get("events", [r.body]):
        r.m.container_event(r.p["aid"], ev["allocation_id"], ev["state"], ev.get("exit_code"))
    return {}


@route("GET", "/api/v1/resource-pools")
def resource_pools(r: Req) -> Any:
    return {"resource_pools": r.m.rm.pools()}


@route("GET", "/api/v1/job-queues")
def job_queue(r: Req) -> Any:
    return {"jobs": r.m.rm.queue()}


@route("POST", "/api/v1/job-queues")
def update_job_queue(r: Req) -> Any:
    for u in r.body.get("updates", []):
        r.m.rm.set_job_priority(u["job_id"], u.get("priority"), u.get("weight"), u.get("queue_position"))
    return {}


# =========================================================================== experiments
@route("POST", "/api/v1/experiments")
def create_experiment(r: Req) -> Any:
    require(r, "CREATE_EXPERIMENT", _project_workspace(r.m, r.body.get("project_id")))
    md = r.body.get("model_definition")
    blob = base64.b64decode(md) if md else None
    try:
        e = r.m.create_experiment(r.body["config"], blob, r.body.get("parent_id"),
                                  activate=r.body.get("activate", True),
                                  project_id=r.body.get("project_id"), owner_id=r.user["id"],
                                  template=r.body.get("template"), unmanaged=bool(r.body.get("unmanaged")),
                                  validate_only=bool(r.body.get("validate_only")))
    except InvalidConfigurationException as ex:
        raise HTTPError(400, str(ex))
    except KeyError as ex:
        raise HTTPError(404, str(ex))
    if e is None:
        return {"experiment": None, "config": None}
    return {"experiment": r.m.experiment_api(e.id), "config": e.config}


@route("GET", "/api/v1/experiments")
def list_experiments(r: Req) -> Any:
    rows = r.m.db.all("SELECT * FROM experiments ORDER BY id DESC")
    arch = r.qget("archived")
    states = set(r.qlist("states"))
    out = []
    for row in rows:
        d = experiment_row_to_api(row, r.m.experiments.get(row["id"]))
        if arch is not None and d["archived"] != (arch in ("true", "1")):
            continue
        if states and d["state"] not in states:
            continue
        if r.qget("project_id") and str(d["project_id"]) != r.qget("project_id"):
            continue
        out.append(d)
    p = _paginate(out, r)
    return {"experiments": p["items"], "pagination": p["pagination"]}


@route("GET", "/api/v1/experiments/labels")
def experiment_labels(r: Req) -> Any:
    labels: Dict[str, int] = {}
    for row in r.m.db.all("SELECT config FROM experiments"):
        for l in (dec(row["config"], {}) or {}).get("labels", []) or []:
            labels[l] = labels.get(l, 0) + 1
    return {"labels": sorted(labels, key=lambda k: -labels[k])}


@route("GET", "/api/v1/experiments/{eid}")
def get_experiment(r: Req) -> Any:
    try:
        d = r.m.experiment_api(_int(r.p["eid"]))
    except KeyError as e:
        raise HTTPError(404, str(e))
    return {"experiment": d, "config": d["config"]}


def _exp(r: Req, perm: Optional[str] = None):
    try:
        e = r.m.get_experiment(_int(r.p["eid"]))
    except KeyError as ex:
        raise HTTPError(404, str(ex))
    if perm is not None:
        row = r.m.db.one("SELECT project_id FROM experiments WHERE id=?", [e.id])
        require(r, perm, _project_workspace(r.m, row["project_id"] if row else None))
    return e


@route("POST", "/api/v1/experiments/continue")
def continue_experiment(r: Req) -> Any:
    """ContinueExperiment: merge ``override_config`` (YAML text or a mapping) into a terminal
    single-trial experiment's config and resume its trial."""
    import yaml

    from determined_clone_amd.config import expconf
    from determined_clone_amd.util import merge_dicts

    r.p["eid"] = str(r.body.get("id"))
    e = _exp(r, "UPDATE_EXPERIMENT")
    ov = r.body.get("override_config") or {}
    if isinstance(ov, str):
        ov = yaml.safe_load(ov) or {}
    try:
        cfg = expconf.complete(merge_dicts(e.config, expconf.parse(ov) if ov else {}))
        e.continue_with(cfg)
    except (InvalidConfigurationException, ValueError) as ex:
        raise HTTPError(400, str(ex))
    return {"experiment": r.m.experiment_api(e.id), "config": e.config}


@route("POST", "/api/v1/experiments/{eid}/activate")
def exp_activate(r: Req) -> Any:
    _exp(r, "UPDATE_EXPERIMENT").activate()
    return {}


@route("POST", "/api/v1/experiments/{eid}/pause")
def exp_pause(r: Req) -> Any:
    _exp(r, "UPDATE_EXPERIMENT").pause()
    return {}


@route("POST", "/api/v1/experiments/{eid}/cancel")
def exp_cancel(r: Req) -> Any:
    _exp(r, "UPDATE_EXPERIMENT").cancel()
    return {}


@route("POST", "/api/v1/experiments/{eid}/kill")
def exp_kill(r: Req) -> Any:
    _exp(r, "UPDATE_EXPERIMENT").cancel(kill=True)
    return {}


@route("POST", "/api/v1/experiments/{eid}/archive")
def exp_archive(r: Req) -> Any:
    e = _exp(r, "UPDATE_EXPERIMENT_METADATA")
    if e.state not in TERMINAL:
        raise HTTPError(400, "only terminal experiments can be archived")
    r.m.db.update("experiments", "id", e.id, {"archived": 1})
    return {}


@route("POST", "/api/v1/experiments/{eid}/unarchive")
def exp_unarchive(r: Req) -> Any:
    r.m.db.update("experiments", "id", _exp(r, "UPDATE_EXPERIMENT_METADATA").id, {"archived": 0})
    return {}


@route("PATCH", "/api/v1/experiments/{eid}")
def exp_patch(r: Req) -> Any:
    e = _exp(r, "UPDATE_EXPERIMENT_METADATA")
    cfg = dict(e.config)
    for k in ("name", "description", "labels"):
        if k in r.body:
            cfg[k] = r.body[k]
    e.config = cfg
    fields: Dict[str, Any] = {"config": cfg}
    if "notes" in r.body:
        fields["notes"] = r.body["notes"]
    if "checkpoint_storage" in r.body:  # GC policy (save_*) only; the storage backend is fixed
        gc = {k: int(v) for k, v in (r.body["checkpoint_storage"] or {}).items()
              if k in ("save_experiment_best", "save_trial_best", "save_trial_latest")}
        cfg["checkpoint_storage"] = dict(cfg.get("checkpoint_storage") or {}, **gc)
        e.config = cfg
        fields["config"] = cfg
    if "resources" in r.body:
        res = r.body["resources"] or {}
        if "priority" in res or "weight" in res:
            e.priority = int(res.get("priority", e.priority))
            e.weight = float(res.get("weight", e.weight))
            r.m.rm.set_job_priority(e.job_id, e.priority, e.weight)
        if "max_slots" in res:
            e.max_slots = res["max_slots"]
    r.m.db.update("experiments", "id", e.id, fields)
    return {"experiment": r.m.experiment_api(e.id)}


@route("DELETE", "/api/v1/experiments/{eid}")
def exp_delete(r: Req) -> Any:
    e = _exp(r, "DELETE_EXPERIMENT")
    if e.state not in TERMINAL:
        raise HTTPError(400, "cannot delete an experiment that is still running")
    uuids = [c["uuid"] for c in r.m.db.all("SELECT uuid FROM checkpoints WHERE experiment_id=?", [e.id])]
    r.m.delete_checkpoints(uuids, e)
    tids = [t["id"] for t in r.m.db.all("SELECT id FROM trials WHERE experiment_id=?", [e.id])]
    for tid in tids:
        r.m.db.execute("DELETE FROM metrics WHERE trial_id=?", [tid])
    r.m.db.execute("DELETE FROM trials WHERE experiment_id=?", [e.id])
    r.m.db.execute("DELETE FROM experiments WHERE id=?", [e.id])
    r.m.experiments.pop(e.id, None)
    return {}


@route("GET", "/api/v1/experiments/{eid}/trials")
def exp_trials(r: Req) -> Any:
    e = _exp(r)
    rows = r.m.db.all("SELECT * FROM trials WHERE experiment_id=? ORDER BY id", [e.id])
    out = [trial_row_to_api(row, e.trials.get(row["request_id"])) for row in rows]
    sb = r.qget("sort_by")
    if sb == "best_validation":
        out.sort(key=lambda t: (t["best_validation"] is None, t["best_validation"] or 0))
    p = _paginate(out, r)
    return {"trials": p["items"], "pagination": p["pagination"]}


@route("GET", "/api/v1/experiments/{eid}/checkpoints")
def exp_checkpoints(r: Req) -> Any:
    e = _exp(r)
    rows = r.m.db.all("SELECT * FROM checkpoints WHERE experiment_id=? ORDER BY report_time", [e.id])
    states = set(r.qlist("states"))
    out = [r.m.checkpoint_api(row) for row in rows if not states or row["state"] in states]
    metric = e.config["searcher"].get("metric")
    if r.qget("sort_by") == "searcher_metric" and metric:
        def key(c: Dict[str, Any]) -> Any:
            v = ((c["training"].get("validation_metrics") or {}).get("avg_metrics") or {}).get(metric)
            return (v is None, v if e.smaller_is_better or v is None else -v)

        out.sort(key=key)
    return {"checkpoints": out}


@route("GET", "/api/v1/experiments/{eid}/validation-history")
def exp_val_history(r: Req) -> Any:
    e = _exp(r)
    metric = e.config["searcher"].get("metric")
    hist = []
    best = None
    for row in r.m.db.all("SELECT m.*, t.id as tid FROM metrics m JOIN trials t ON m.trial_id=t.id "
                          "WHERE t.experiment_id=? AND m.grp='validation' ORDER BY m.end_time", [e.id]):
        v = (dec(row["metrics"], {}) or {}).get(metric)
        if not isinstance(v, (int, float)):
            continue
        if best is None or (v < best if e.smaller_is_better else v > best):
            best = v
            hist.append({"trial_id": row["tid"], "end_time": row["end_time"], "searcher_metric": v})
    return {"validation_history": hist}


@route("GET", "/api/v1/experiments/{eid}/searcher/best_searcher_validation_metric")
def exp_best_metric(r: Req) -> Any:
    return {"metric": _exp(r).best_metric}


@route("GET", "/api/v1/experiments/{eid}/model_def")
def exp_model_def(r: Req) -> Any:
    row = r.m.db.one("SELECT model_definition FROM experiments WHERE id=?", [_int(r.p["eid"])])
    if row is None:
        raise HTTPError(404, "experiment not found")
    b = row["model_definition"]
    return {"b64_tgz": base64.b64encode(b).decode() if b else ""}


@route("GET", "/api/v1/experiments/{eid}/searcher_events")
def searcher_events(r: Req) -> Any:
    e = _exp(r)
    m = e.searcher.method
    if not hasattr(m, "events_after"):
        raise HTTPError(400, "experiment does not use a custom searcher")
    return {"searcher_events": m.state["events"]}


@route("POST", "/api/v1/experiments/{eid}/searcher_operations")
def post_searcher_ops(r: Req) -> Any:
    from determined_clone_amd.searcher import op_from_dict

    e = _exp(r)
    m = e.searcher.method
    if not hasattr(m, "ack_events"):
        raise HTTPError(400, "experiment does not use a custom searcher")
    with e.lock:
        if r.body.get("triggered_by_event_id") is not None:
            m.ack_events(int(r.body["triggered_by_event_id"]))
        if "progress" in r.body:
            m.state["progress"] = float(r.body["progress"])
        ops = [op_from_dict(o) for o in r.body.get("searcher_operations", [])]
        e.searcher.record(ops)
        e._process(ops)
        e._persist()
    return {}


@route("POST", "/api/v1/preview-hp-search")
def preview_hp_search(r: Req) -> Any:
    from determined_clone_amd.config import expconf
    from determined_clone_amd.searcher import make_search_method, simulate

    try:
        cfg = expconf.complete(r.body["config"])
    except InvalidConfigurationException as e:
        raise HTTPError(400, str(e))
    res = simulate(make_search_method(cfg["searcher"]), cfg["hyperparameters"],
                   seed=int(r.body.get("seed", 0)))
    return {"simulation": {"trials": res["trials"], "results": res["results"]}}


# =========================================================================== trials
def _trial(r: Req):
    try:
        return r.m.trial_by_id(_int(r.p["tid"]))
    except KeyError as e:
        raise HTTPError(404, str(e))


@route("GET", "/api/v1/trials/{tid}")
def get_trial(r: Req) -> Any:
    try:
        return {"trial": r.m.trial_api(_int(r.p["tid"]))}
    except KeyError as e:
        raise HTTPError(404, str(e))


@route("POST", "/api/v1/trials/{tid}/kill")
def kill_trial(r: Req) -> Any:
    t = _trial(r)
    t.exp.kill_trial(t)
    return {}


@route("GET", "/api/v1/trials/{tid}/searcher/operation")
def trial_searcher_op(r: Req) -> Any:
    t = _trial(r)
    with t.exp.lock:
        return t.searcher_operation()


@route("POST", "/api/v1/trials/{tid}/searcher/completed_operation")
def trial_completed_op(r: Req) -> Any:
    t = _trial(r)
    try:
        t.exp.validation_completed(t, int(r.body["op"]["length"]), r.body.get("searcher_metric"))
    except ValueError as e:
        raise HTTPError(400, str(e))
    return {}


@route("POST", "/api/v1/trials/{tid}/progress")
def trial_progress(r: Req) -> Any:
    t = _trial(r)
    t.exp.progress(t, float(r.body.get("progress", 0)))
    return {}


@route("POST", "/api/v1/trials/{tid}/early_exit")
def trial_early_exit(r: Req) -> Any:
    t = _trial(r)
    t.exp.early_exit(t, r.body.get("reason", "EXITED_REASON_UNSPECIFIED"))
    return {}


@route("POST", "/api/v1/trials/{tid}/metrics")
def post_metrics(r: Req) -> Any:
    r.m.report_metrics(_int(r.p["tid"]), r.body)
    return {}


@route("GET", "/api/v1/trials/{tid}/metrics")
def get_metrics(r: Req) -> Any:
    grp = r.qget("group")
    sql = "SELECT * FROM metrics WHERE trial_id=?"
    args: List[Any] = [_int(r.p["tid"])]
    if grp:
        sql += " AND grp=?"
        args.append(grp)
    rows = r.m.db.all(sql + " ORDER BY steps_completed, id", args)
    return {"metrics": [{"group": x["grp"], "steps_completed": x["steps_completed"],
                         "metrics": dec(x["metrics"], {}), "trial_run_id": x["trial_run_id"],
                         "end_time": x["end_time"]} for x in rows]}


@route("POST", "/api/v1/trials/{tid}/runner/metadata")
def runner_metadata(r: Req) -> Any:
    r.m.db.update("trials", "id", _int(r.p["tid"]), {"runner_state": (r.body.get("metadata") or {}).get("state", "")})
    return {}


@route("POST", "/api/v1/trials/{tid}/heartbeat")
def trial_heartbeat(r: Req) -> Any:
    t = _trial(r)
    t.exp.unmanaged_heartbeat(t, str(r.body.get("state", "RUNNING")))
    return {}


@route("GET", "/api/v1/trials/{tid}/checkpoints")
def trial_checkpoints(r: Req) -> Any:
    rows = r.m.db.all("SELECT * FROM checkpoints WHERE trial_id=? ORDER BY steps_completed", [_int(r.p["tid"])])
    return {"checkpoints": [r.m.checkpoint_api(x) for x in rows]}


@route("GET", "/api/v1/trials/{tid}/logs")
def trial_logs(r: Req) -> Any:
    row = r.m.db.one("SELECT task_id FROM trials WHERE id=?", [_int(r.p["tid"])])
    if row is None:
        raise HTTPError(404, "trial not found")
    return _logs(r, row["task_id"])


@route("GET", "/api/v1/trials/{tid}/profiler/metrics")
def get_profiler(r: Req) -> Any:
    """GetTrialProfilerMetrics: the trial's profiler series as TrialProfilerMetricsBatch objects
    (one per series), filtered by ``labels.name`` / ``labels.agent_id`` / ``labels.gpu_uuid`` /
    ``labels.metric_type``; ``follow`` is accepted and answered with what exists now."""
    where, args = ["trial_id=?"], [_int(r.p["tid"])]
    for q, col in (("labels.name", "name"), ("labels.agent_id", "agent_id"),
                   ("labels.gpu_uuid", "gpu_uuid"), ("labels.metric_type", "metric_type")):
        v = r.qget(q)
        if v not in (None, ""):
            where.append(f"COALESCE({col}, '')=?")
            args.append(v)
    rows = r.m.db.all(f"SELECT * FROM profiler_metrics WHERE {' AND '.join(where)} ORDER BY ts, id", args)
    series: Dict[Any, Dict[str, Any]] = {}
    for x in rows:
        key = (x["name"], x["agent_id"] or "", x["gpu_uuid"] or "", x["metric_type"] or "")
        b = series.get(key)
        if b is None:
            b = series[key] = {"values": [], "batches": [], "timestamps": [], "labels": {
                "trialId": _int(r.p["tid"]), "name": key[0], "agentId": key[1], "gpuUuid": key[2],
                "metricType": key[3] or "PROFILER_METRIC_TYPE_UNSPECIFIED"}}
        v = dec(x["value"], None)
        b["values"].append(v["value"] if isinstance(v, dict) else v)
        b["batches"].append(x["batch"] if x["batch"] is not None else 0)
        b["timestamps"].append(v.get("time") if isinstance(v, dict) else x["ts"])
    return {"batches": list(series.values())}


# =========================================================================== allocations
def _alloc(r: Req):
    a = r.m.allocations.get(r.p["aid"])
    if a is None:
        raise HTTPError(404, "allocation not found")
    return a


@route("GET", "/api/v1/allocations/{aid}/signals/preemption")
def preemption_signal(r: Req) -> Any:
    a = _alloc(r)
    to = min(float(r.qget("timeout_seconds", 60)), 3600)
    return {"preempt": bool(a.preempt.wait(to))}


@route("POST", "/api/v1/allocations/{aid}/signals/ack_preemption")
def ack_preemption(r: Req) -> Any:
    _alloc(r).preempt_acked = True
    return {}


@route("POST", "/api/v1/allocations/{aid}/ready")
def alloc_ready(r: Req) -> Any:
    _alloc(r).ready = True
    return {}


@route("POST", "/api/v1/allocations/{aid}/proxy_address")
def alloc_proxy(r: Req) -> Any:
    _alloc(r).proxy_address = r.body.get("proxy_address")
    return {}


@route("POST", "/api/v1/allocations/{aid}/all_gather")
def alloc_allgather(r: Req) -> Any:
    a = _alloc(r)
    key = r.body["request_uuid"]
    n = int(r.body["num_peers"])
    with a.allgather_cv:
        lst = a.allgather.setdefault(key, [])
        lst.append(r.body.get("data"))
        a.allgather_cv.notify_all()
        a.allgather_cv.wait_for(lambda: len(a.allgather[key]) >= n, timeout=600)
        return {"data": list(a.allgather[key])}


# =========================================================================== tasks / logs
@route("POST", "/api/v1/task/logs")
def post_task_logs(r: Req) -> Any:
    r.m.post_logs(r.body.get("logs", []))
    return {}


def _logs(r: Req, task_id: str) -> Any:
    after = _int(r.qget("after_id", 0))
    follow = r.qget("follow") in ("true", "1")
    rows = r.m.task_logs(task_id, after)
    if follow and not rows:
        with r.m.log_cv:
            r.m.log_cv.wait(float(r.qget("timeout_seconds", 10)))
        rows = r.m.task_logs(task_id, after)
    done = all(a.exited for a in r.m.allocations.values() if a.task_id == task_id)
    return {"logs": [{"id": x["id"], "log": x["log"], "rank_id": x["rank_id"], "timestamp": x["timestamp"],
                      "level": x["level"], "agent_id": x["agent_id"], "stdtype": x["stdtype"]} for x in rows],
            "done": done}


@route("GET", "/api/v1/tasks/{task_id}/logs")
def task_logs(r: Req) -> Any:
    return _logs(r, r.p["task_id"])


@route("GET", "/api/v1/tasks")
def list_tasks(r: Req) -> Any:
    return {"tasks": list(r.m.tasks.values())}


@route("GET", "/api/v1/tasks/{task_id}")
def get_task(r: Req) -> Any:
    t = r.m.db.one("SELECT * FROM tasks WHERE task_id=?", [r.p["task_id"]])
    allocs = r.m.db.all("SELECT * FROM allocations WHERE task_id=?", [r.p["task_id"]])
    # a trial's task exists from trial creation on (unmanaged trials never get an allocation)
    if t is None and not allocs and not r.m.db.one("SELECT id FROM trials WHERE task_id=?", [r.p["task_id"]]):
        raise HTTPError(404, "task not found")
    return {"task": {"task_id": r.p["task_id"], "type": (t or {}).get("task_type", "TRIAL"),
                     "allocations": allocs}}


@route("GET", "/api/v1/tasks/{task_id}/context")
def task_context(r: Req) -> Any:
    tid = r.p["task_id"]
    blob = r.m.db.kv_get(f"context:{tid}")
    if blob is not None:
        return {"b64_tgz": base64.b64encode(bytes.fromhex(blob)).decode()}
    exp_id = tid.split(".")[0]
    if exp_id.isdigit():
        row = r.m.db.one("SELECT model_definition FROM experiments WHERE id=?", [int(exp_id)])
        if row and row["model_definition"]:
            return {"b64_tgz": base64.b64encode(row["model_definition"]).decode()}
    return {"b64_tgz": ""}


# NTSC: commands / shells / notebooks / tensorboards
for _kind, _path in (("COMMAND", "commands"), ("SHELL", "shells"), ("NOTEBOOK", "notebooks"),
                     ("TENSORBOARD", "tensorboards")):
    def _mk(kind: str, path: str) -> None:
        @route("POST", f"/api/v1/{path}")
        def launch(r: Req, kind: str = kind) -> Any:
            require(r, "CREATE_NSC", r.body.get("workspace_id"))
            cfg = r.body.get("config") or {}
            res = cfg.get("resources") or {}
            ep = r.body.get("entrypoint") or cfg.get("entrypoint") or []
            if isinstance(ep, str):
                ep = ["bash", "-c", ep]
            if kind == "TENSORBOARD" and not ep:
                eids = [int(x) for x in r.body.get("experiment_ids") or []]
                if r.body.get("filters") is not None:  # reference api_tensorboard.go:484-487
                    from determined_clone_amd.master.experiment_filter import bulk_filter_sql

                    where, params = bulk_filter_sql(r.body["filters"])
                    eids = [row["id"] for row in r.m.db.all(
                        f"SELECT e.id FROM experiments e WHERE {where} ORDER BY e.id", params)]
                ep = ["python3", "-m", "determined_clone_amd.exec.tensorboard"] + [str(x) for x in eids]
            if kind == "NOTEBOOK" and not ep:
                ep = ["python3", "-m", "determined_clone_amd.exec.notebook"]
            if kind == "SHELL" and not ep:
                ep = ["python3", "-m", "determined_clone_amd.exec.shell"]
            ctx = base64.b64decode(r.body["files"]) if r.body.get("files") else None
            env = dict((cfg.get("environment") or {}).get("environment_variables") or {})
            idle = cfg.get("idle_timeout")
            if idle and kind in ("NOTEBOOK", "SHELL"):  # expconf duration ("30m") or seconds
                from determined_clone_amd.master.provisioner import _seconds

                env[f"DET_{kind}_IDLE_TIMEOUT"] = str(_seconds(idle))
            t = r.m.launch_command(kind, ep, int(res.get("slots", 0)), int(res.get("priority") or 42),
                                   res.get("resource_pool") or "default", env,
                                   r.user["id"], ctx, cfg.get("description"), config=cfg)
            return {path[:-1]: t}

        @route("GET", f"/api/v1/{path}")
        def list_(r: Req, kind: str = kind) -> Any:
            return {path: [dict(t, id=t["task_id"]) for t in r.m.tasks.values() if t.get("type") == kind]}

        @route("GET", f"/api/v1/{path}/{{task_id}}")
        def get_(r: Req, kind: str = kind) -> Any:
            t = r.m.tasks.get(r.p["task_id"])
            if t is None or t.get("type") != kind:
                raise HTTPError(404, f"{kind.lower()} not found")
            ready = any(a.task_id == t["task_id"] and a.proxy_address and not a.exited
                        for a in list(r.m.allocations.values()))
            return {path[:-1]: dict(t, id=t["task_id"], service_ready=ready,
                                    proxy_path=f"/proxy/{t['task_id']}/")}

        @route("POST", f"/api/v1/{path}/{{task_id}}/kill")
        def kill_(r: Req, kind: str = kind) -> Any:
            for a in list(r.m.allocations.values()):
                if a.task_id == r.p["task_id"]:
                    r.m.kill_allocation(a.id)
            return {}

    _mk(_kind, _path)


# =========================================================================== checkpoints
@route("POST", "/api/v1/checkpoints")
def report_checkpoint(r: Req) -> Any:
    r.m.report_checkpoint(r.body)
    return {}


@route("GET", "/api/v1/checkpoints/{uuid}")
def get_checkpoint(r: Req) -> Any:
    row = r.m.db.one("SELECT * FROM checkpoints WHERE uuid=?", [r.p["uuid"]])
    if row is None:
        raise HTTPError(404, "checkpoint not found")
    c = r.m.checkpoint_api(row)
    if row.get("experiment_id"):
        e = r.m.experiments.get(row["experiment_id"])
        if e is not None:
            c["storage"] = e.config.get("checkpoint_storage")
    return {"checkpoint": c}


def _checkpoint_edit_check(r: Req, uuids: List[str]) -> None:
    """The caller must be allowed to edit every owning experiment (the reference's
    checkpointsRBACEditCheck, `master/internal/api_checkpoint.go`)."""
    for u in uuids:
        row = r.m.db.one("SELECT experiment_id FROM checkpoints WHERE uuid=?", [u])
        if row is None:
            raise HTTPError(404, f"checkpoint {u} not found")
        eid = row.get("experiment_id")
        if eid is None:
            require(r, "UPDATE_EXPERIMENT")
            continue
        erow = r.m.db.one("SELECT project_id FROM experiments WHERE id=?", [eid])
        require(r, "UPDATE_EXPERIMENT", _project_workspace(r.m, erow["project_id"] if erow else None))


def _remove_checkpoint_files(r: Req, uuids: List[str], globs: List[str]) -> None:
    for g in globs:
        if not isinstance(g, str) or not g:
            raise HTTPError(400, "cannot have empty string glob")
        if ".." in g:
            raise HTTPError(400, f"glob '{g}' cannot contain '..'")
    _checkpoint_edit_check(r, uuids)
    registered = r.m.registered_checkpoints(uuids)
    if registered:
        raise HTTPError(400, "this subset of checkpoints provided are in the model registry and "
                             f"cannot be deleted: {registered}")
    r.m.delete_checkpoints(uuids, globs=globs)


@route("POST", "/api/v1/checkpoints/rm")
def rm_checkpoint_files(r: Req) -> Any:
    _remove_checkpoint_files(r, list(r.body.get("checkpoint_uuids", [])),
                             list(r.body.get("checkpoint_globs") or r.body.get("globs") or ["**/*"]))
    return {}


@route("DELETE", "/api/v1/checkpoints")
def delete_checkpoints(r: Req) -> Any:
    _remove_checkpoint_files(r, list(r.body.get("checkpoint_uuids", [])), ["**/*"])
    return {}


@route("PATCH", "/api/v1/checkpoints/{uuid}/metadata")
def patch_checkpoint_md(r: Req) -> Any:
    row = r.m.db.one("SELECT metadata FROM checkpoints WHERE uuid=?", [r.p["uuid"]])
    if row is None:
        raise HTTPError(404, "checkpoint not found")
    _checkpoint_edit_check(r, [r.p["uuid"]])
    md = dec(row["metadata"], {})
    md.update(r.body.get("metadata", {}))
    r.m.db.update("checkpoints", "uuid", r.p["uuid"], {"metadata": md})
    return {"checkpoint": r.m.checkpoint_api(r.m.db.one("SELECT * FROM checkpoints WHERE uuid=?", [r.p["uuid"]]))}


# =========================================================================== model registry
def _model_api(row: Dict[str, Any], db: Any) -> Dict[str, Any]:
    n = db.one("SELECT COUNT(*) AS n FROM model_versions WHERE model_id=?", [row["id"]])["n"]
    return {"id": row["id"], "name": row["name"], "description": row["description"],
            "metadata": dec(row["metadata"], {}), "labels": dec(row["labels"], []),
            "notes": row["notes"], "archived": bool(row["archived"]), "user_id": row["user_id"],
            "workspace_id": row["workspace_id"], "creation_time": row["creation_time"],
            "last_updated_time": row["last_updated_time"], "num_versions": n}


def _model(r: Req) -> Dict[str, Any]:
    key = r.p["name"]
    row = r.m.db.one("SELECT * FROM models WHERE name=?", [key])
    if row is None and key.isdigit():
        row = r.m.db.one("SELECT * FROM models WHERE id=?", [int(key)])
    if row is None:
        raise HTTPError(404, f"model {key} not found")
    return row


@route("POST", "/api/v1/models")
def post_model(r: Req) -> Any:
    require(r, "CREATE_MODEL_REGISTRY", r.body.get("workspace_id") or 1)
    if r.m.db.one("SELECT id FROM models WHERE name=?", [r.body["name"]]):
        raise HTTPError(409, "model already exists")
    mid = r.m.db.insert("models", {"name": r.body["name"], "description": r.body.get("description", ""),
                                   "metadata": r.body.get("metadata", {}), "labels": r.body.get("labels", []),
                                   "notes": r.body.get("notes", ""), "user_id": r.user["id"],
                                   "workspace_id": r.body.get("workspace_id", 1),
                                   "creation_time": now(), "last_updated_time": now()})
    return {"model": _model_api(r.m.db.one("SELECT * FROM models WHERE id=?", [mid]), r.m.db)}


@route("GET", "/api/v1/models")
def list_models(r: Req) -> Any:
    rows = [_model_api(x, r.m.db) for x in r.m.db.all("SELECT * FROM models ORDER BY id")]
    name = r.qget("name")
    if name:
        rows = [x for x in rows if name.lower() in x["name"].lower()]
    if r.qget("archived") is not None:
        rows = [x for x in rows if x["archived"] == (r.qget("archived") in ("true", "1"))]
    p = _paginate(rows, r)
    return {"models": p["items"], "pagination": p["pagination"]}


@route("GET", "/api/v1/models/{name}")
def get_model(r: Req) -> Any:
    return {"model": _model_api(_model(r), r.m.db)}


@route("PATCH", "/api/v1/models/{name}")
def patch_model(r: Req) -> Any:
    m = _model(r)
    body = r.body.get("model", r.body)
    fields = {k: body[k] for k in ("name", "description", "metadata", "labels", "notes") if k in body}
    fields["last_updated_time"] = now()
    r.m.db.update("models", "id", m["id"], fields)
    return {"model": _model_api(r.m.db.one("SELECT * FROM models WHERE id=?", [m["id"]]), r.m.db)}


@route("POST", "/api/v1/models/{name}/archive")
def archive_model(r: Req) -> Any:
    r.m.db.update("models", "id", _model(r)["id"], {"archived": 1})
    return {}


@route("POST", "/api/v1/models/{name}/unarchive")
def unarchive_model(r: Req) -> Any:
    r.m.db.update("models", "id", _model(r)["id"], {"archived": 0})
    return {}


@route("DELETE", "/api/v1/models/{name}")
def delete_model(r: Req) -> Any:
    m = _model(r)
    require(r, "DELETE_MODEL_REGISTRY" if m.get("user_id") in (None, r.user["id"])
            else "DELETE_OTHER_USER_MODEL_REGISTRY", m.get("workspace_id") or 1)
    r.m.db.execute("DELETE FROM model_versions WHERE model_id=?", [m["id"]])
    r.m.db.execute("DELETE FROM models WHERE id=?", [m["id"]])
    return {}


def _mv_api(row: Dict[str, Any], m: Any) -> Dict[str, Any]:
    ck = m.db.one("SELECT * FROM checkpoints WHERE uuid=?", [row["checkpoint_uuid"]])
    return {"id": row["id"], "model_id": row["model_id"], "version": row["version"],
            "name": row["name"], "comment": row["comment"], "notes": row["notes"],
            "metadata": dec(row["metadata"], {}), "labels": dec(row["labels"], []),
            "creation_time": row["creation_time"], "last_updated_time": row["last_updated_time"],
            "checkpoint": m.checkpoint_api(ck) if ck else {"uuid": row["checkpoint_uuid"]}}


@route("POST", "/api/v1/models/{name}/versions")
def post_model_version(r: Req) -> Any:
    m = _model(r)
    require(r, "EDIT_MODEL_REGISTRY", m.get("workspace_id") or 1)
    ck = r.body.get("checkpoint_uuid")
    if not r.m.db.one("SELECT uuid FROM checkpoints WHERE uuid=?", [ck]):
        raise HTTPError(404, f"checkpoint {ck} not found")
    v = (r.m.db.one("SELECT MAX(version) AS v FROM model_versions WHERE model_id=?", [m["id"]])["v"] or 0) + 1
    vid = r.m.db.insert("model_versions", {"model_id": m["id"], "version": v, "checkpoint_uuid": ck,
                                           "name": r.body.get("name"), "comment": r.body.get("comment", ""),
                                           "metadata": r.body.get("metadata", {}), "labels": r.body.get("labels", []),
                                           "notes": r.body.get("notes", ""), "user_id": r.user["id"],
                                           "creation_time": now(), "last_updated_time": now()})
    return {"model_version": _mv_api(r.m.db.one("SELECT * FROM model_versions WHERE id=?", [vid]), r.m)}


@route("GET", "/api/v1/models/{name}/versions")
def list_model_versions(r: Req) -> Any:
    m = _model(r)
    rows = r.m.db.all("SELECT * FROM model_versions WHERE model_id=? ORDER BY version", [m["id"]])
    return {"model": _model_api(m, r.m.db), "model_versions": [_mv_api(x, r.m) for x in rows]}


@route("GET", "/api/v1/models/{name}/versions/{ver}")
def get_model_version(r: Req) -> Any:
    m = _model(r)
    row = r.m.db.one("SELECT * FROM model_versions WHERE model_id=? AND version=?", [m["id"], _int(r.p["ver"])])
    if row is None:
        raise HTTPError(404, "model version not found")
    return {"model_version": _mv_api(row, r.m)}


@route("PATCH", "/api/v1/models/{name}/versions/{ver}")
def patch_model_version(r: Req) -> Any:
    m = _model(r)
    body = r.body.get("model_version", r.body)
    fields = {k: body[k] for k in ("name", "comment", "notes", "metadata", "labels") if k in body}
    fields["last_updated_time"] = now()
    r.m.db.execute("UPDATE model_versions SET " + ",".join(f"{k}=?" for k in fields) +
                   " WHERE model_id=? AND version=?",
                   [json.dumps(v) if isinstance(v, (dict, list)) else v for v in fields.values()] + [m["id"], _int(r.p["ver"])])
    return get_model_version(r)


@route("DELETE", "/api/v1/models/{name}/versions/{ver}")
def delete_model_version(r: Req) -> Any:
    m = _model(r)
    require(r, "DELETE_MODEL_VERSION", m.get("workspace_id") or 1)
    r.m.db.execute("DELETE FROM model_versions WHERE model_id=? AND version=?", [m["id"], _int(r.p["ver"])])
    return {}


# =========================================================================== templates
@route("GET", "/api/v1/templates")
def list_templates(r: Req) -> Any:
    return {"templates": [{"name": x["name"], "config": dec(x["config"], {}), "workspace_id": x["workspace_id"]}
                          for x in r.m.db.all("SELECT * FROM templates ORDER BY name")]}


@route("GET", "/api/v1/templates/{name}")
def get_template(r: Req) -> Any:
    x = r.m.db.one("SELECT * FROM templates WHERE name=?", [r.p["name"]])
    if x is None:
        raise HTTPError(404, "template not found")
    return {"template": {"name": x["name"], "config": dec(x["config"], {}), "workspace_id": x["workspace_id"]}}


@route("PUT", "/api/v1/templates/{name}")
def put_template(r: Req) -> Any:
    from determined_clone_amd.config import expconf

    require(r, "UPDATE_TEMPLATES")
    cfg = expconf.parse(r.body.get("config", {}))
    r.m.db.upsert("templates", {"name": r.p["name"], "config": cfg, "workspace_id": r.body.get("workspace_id", 1)})
    return get_template(r)


@route("POST", "/api/v1/templates")
def post_template(r: Req) -> Any:
    r.p["name"] = r.body["name"]
    return put_template(r)


@route("DELETE", "/api/v1/templates/{name}")
def delete_template(r: Req) -> Any:
    require(r, "DELETE_TEMPLATES")
    r.m.db.execute("DELETE FROM templates WHERE name=?", [r.p["name"]])
    return {}


# =========================================================================== workspaces / projects
def _ws_api(row: Dict[str, Any], db: Any) -> Dict[str, Any]:
    return {"id": row["id"], "name": row["name"], "archived": bool(row["archived"]),
            "pinned": bool(row["pinned"]), "user_id": row["user_id"],
            "num_projects": db.one("SELECT COUNT(*) AS n FROM projects WHERE workspace_id=?", [row["id"]])["n"],
            "checkpoint_storage_config": dec(row.get("checkpoint_storage")),
            "default_compute_pool": row.get("default_pool")}


def _proj_api(row: Dict[str, Any], db: Any) -> Dict[str, Any]:
    return {"id": row["id"], "name": row["name"], "workspace_id": row["workspace_id"],
            "description": row["description"], "notes": dec(row["notes"], []),
            "archived": bool(row["archived"]), "user_id": row["user_id"],
            "num_experiments": db.one("SELECT COUNT(*) AS n FROM experiments WHERE project_id=?", [row["id"]])["n"]}


@route("GET", "/api/v1/workspaces")
def list_workspaces(r: Req) -> Any:
    return {"workspaces": [_ws_api(x, r.m.db) for x in r.m.db.all("SELECT * FROM workspaces ORDER BY id")]}


@route("POST", "/api/v1/workspaces")
def post_workspace(r: Req) -> Any:
    require(r, "CREATE_WORKSPACE")
    if r.m.db.one("SELECT id FROM workspaces WHERE name=?", [r.body["name"]]):
        raise HTTPError(409, "workspace already exists")
    wid = r.m.db.insert("workspaces", {"name": r.body["name"], "user_id": r.user["id"], "created": now(),
                                       "checkpoint_storage": r.body.get("checkpoint_storage_config"),
                                       "default_pool": r.body.get("default_compute_pool")})
    return {"workspace": _ws_api(r.m.db.one("SELECT * FROM workspaces WHERE id=?", [wid]), r.m.db)}


def _ws(r: Req) -> Dict[str, Any]:
    row = r.m.db.one("SELECT * FROM workspaces WHERE id=?", [_int(r.p["wid"])])
    if row is None:
        raise HTTPError(404, "workspace not found")
    return row


@route("GET", "/api/v1/workspaces/{wid}")
def get_workspace(r: Req) -> Any:
    return {"workspace": _ws_api(_ws(r), r.m.db)}


@route("PATCH", "/api/v1/workspaces/{wid}")
def patch_workspace(r: Req) -> Any:
    w = _ws(r)
    require(r, "UPDATE_WORKSPACE", w["id"])
    if "checkpoint_storage_config" in r.body:
        require(r, "SET_WORKSPACE_CHECKPOINT_STORAGE_CONFIG", w["id"])
    fields = {}
    if "name" in r.body:
        fields["name"] = r.body["name"]
    if "checkpoint_storage_config" in r.body:
        fields["checkpoint_storage"] = r.body["checkpoint_storage_config"]
    r.m.db.update("workspaces", "id", w["id"], fields)
    return get_workspace(r)


@route("DELETE", "/api/v1/workspaces/{wid}")
def delete_workspace(r: Req) -> Any:
    w = _ws(r)
    require(r, "DELETE_WORKSPACE", w["id"])
    if w["id"] == 1:
        raise HTTPError(400, "cannot delete the default workspace")
    r.m.db.execute("DELETE FROM projects WHERE workspace_id=?", [w["id"]])
    r.m.db.execute("DELETE FROM workspaces WHERE id=?", [w["id"]])
    return {"completed": True}


for _act, _val in (("archive", 1), ("unarchive", 0)):
    def _mkws(act: str, val: int) -> None:
        @route("POST", f"/api/v1/workspaces/{{wid}}/{act}")
        def f(r: Req, val: int = val) -> Any:
            r.m.db.update("workspaces", "id", _ws(r)["id"], {"archived": val})
            return {}

        @route("POST", f"/api/v1/projects/{{pid}}/{act}")
        def g(r: Req, val: int = val) -> Any:
            r.m.db.update("projects", "id", _int(r.p["pid"]), {"archived": val})
            return {}

    _mkws(_act, _val)


@route("POST", "/api/v1/workspaces/{wid}/pin")
def pin_workspace(r: Req) -> Any:
    r.m.db.update("workspaces", "id", _ws(r)["id"], {"pinned": 1})
    return {}


@route("POST", "/api/v1/workspaces/{wid}/unpin")
def unpin_workspace(r: Req) -> Any:
    r.m.db.update("workspaces", "id", _ws(r)["id"], {"pinned": 0})
    return {}


@route("GET", "/api/v1/workspaces/{wid}/projects")
def ws_projects(r: Req) -> Any:
    w = _ws(r)
    return {"projects": [_proj_api(x, r.m.db) for x in r.m.db.all("SELECT * FROM projects WHERE workspace_id=? ORDER BY id", [w["id"]])]}


@route("POST", "/api/v1/workspaces/{wid}/projects")
def post_project(r: Req) -> Any:
    w = _ws(r)
    require(r, "CREATE_PROJECT", w["id"])
    if r.m.db.one("SELECT id FROM projects WHERE workspace_id=? AND name=?", [w["id"], r.body["name"]]):
        raise HTTPError(409, "project already exists")
    pid = r.m.db.insert("projects", {"name": r.body["name"], "workspace_id": w["id"], "user_id": r.user["id"],
                                     "description": r.body.get("description", ""), "created": now()})
    return {"project": _proj_api(r.m.db.one("SELECT * FROM projects WHERE id=?", [pid]), r.m.db)}


@route("GET", "/api/v1/projects/{pid}")
def get_project(r: Req) -> Any:
    row = r.m.db.one("SELECT * FROM projects WHERE id=?", [_int(r.p["pid"])])
    if row is None:
        raise HTTPError(404, "project not found")
    return {"project": _proj_api(row, r.m.db)}


@route("PATCH", "/api/v1/projects/{pid}")
def patch_project(r: Req) -> Any:
    fields = {k: r.body[k] for k in ("name", "description") if k in r.body}
    r.m.db.update("projects", "id", _int(r.p["pid"]), fields)
    return get_project(r)


@route("POST", "/api/v1/projects/{pid}/notes")
def add_project_note(r: Req) -> Any:
    row = r.m.db.one("SELECT notes FROM projects WHERE id=?", [_int(r.p["pid"])])
    notes = dec(row["notes"], []) + [{"name": r.body.get("name", ""), "contents": r.body.get("contents", "")}]
    r.m.db.update("projects", "id", _int(r.p["pid"]), {"notes": notes})
    return {"notes": notes}


@route("DELETE", "/api/v1/projects/{pid}")
def delete_project(r: Req) -> Any:
    pid = _int(r.p["pid"])
    require(r, "DELETE_PROJECT", _project_workspace(r.m, pid))
    if pid == 1:
        raise HTTPError(400, "cannot delete the default project")
    r.m.db.execute("DELETE FROM projects WHERE id=?", [pid])
    return {"completed": True}


@route("POST", "/api/v1/experiments/{eid}/move")
def move_experiment(r: Req) -> Any:
    e = _exp(r, "DELETE_EXPERIMENT")
    dest = _int(r.body["destination_project_id"])
    require(r, "CREATE_EXPERIMENT", _project_workspace(r.m, dest))
    r.m.db.update("experiments", "id", e.id, {"project_id": dest})
    return {}


# =========================================================================== webhooks
@route("GET", "/api/v1/webhooks")
def list_webhooks(r: Req) -> Any:
    return {"webhooks": [_webhook_out(x) for x in r.m.webhooks.hooks()]}


def _webhook_out(row: Dict[str, Any]) -> Dict[str, Any]:
    """webhookv1.Webhook: proto enum names for the webhook and trigger types."""
    from determined_clone_amd.master import webhooks as wh

    out = dict(row)
    out["webhook_type"] = "WEBHOOK_TYPE_" + wh.norm_webhook_type(row.get("webhook_type"))
    out["triggers"] = [dict(t, trigger_type="TRIGGER_TYPE_" + wh.norm_trigger_type(t.get("trigger_type")),
                            webhook_id=row.get("id"))
                       for t in row.get("triggers") or []]
    return out


@route("POST", "/api/v1/webhooks")
def post_webhook(r: Req) -> Any:
    from determined_clone_amd.master import webhooks as wh

    require(r, "EDIT_WEBHOOKS")
    try:
        triggers = wh.validate_triggers(r.body.get("triggers", []))
    except ValueError as e:
        raise HTTPError(400, str(e))
    wtype = wh.norm_webhook_type(r.body.get("webhook_type"))
    if wtype not in (wh.DEFAULT, wh.SLACK):
        raise HTTPError(400, f"unknown webhook type {r.body.get('webhook_type')!r}")
    wid = r.m.db.insert("webhooks", {"url": r.body["url"], "webhook_type": wtype, "triggers": triggers,
                                     "mode": r.body.get("mode", "WORKSPACE"), "name": r.body.get("name"),
                                     "workspace_id": r.body.get("workspace_id")})
    r.m.webhooks.reload_triggers()
    row = r.m.db.one("SELECT * FROM webhooks WHERE id=?", [wid])
    return {"webhook": _webhook_out(dict(row, triggers=triggers))}


@route("DELETE", "/api/v1/webhooks/{wid}")
def delete_webhook(r: Req) -> Any:
    require(r, "EDIT_WEBHOOKS")
    r.m.db.execute("DELETE FROM webhooks WHERE id=?", [_int(r.p["wid"])])
    r.m.webhooks.reload_triggers()
    return {}


# =========================================================================== server plumbing
class _Handler(BaseHTTPRequestHandler):
    master: Master = None  # type: ignore[assignment]
    protocol_version = "HTTP/1.1"
    # headers and body leave in separate writes on a kept-alive connection: with Nagle on, the
    # body waits for the client's delayed ACK of the headers (~40 ms per request on Linux)
    disable_nagle_algorithm = True

    def log_message(self, fmt: str, *args: Any) -> None:  # quiet
        logger.debug(fmt % args)

    def _send(self, status: int, payload: Any) -> None:
        data = json.dumps(payload, default=str).encode()
        try:
            self.send_response(status)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)
        except (BrokenPipeError, ConnectionResetError):  # client went away (long-poll cancelled)
            self.close_connection = True

    def _dispatch(self, method: str) -> None:
        parsed = urllib.parse.urlparse(self.path)
        query = urllib.parse.parse_qs(parsed.query)
        length = int(self.headers.get("Content-Length") or 0)
        raw = self.rfile.read(length) if length else b""
        if parsed.path.startswith("/proxy/"):
            return self._proxy(method, parsed, query, raw)
        if parsed.path.startswith("/tunnel/") and method == "GET":
            return self._tunnel(parsed, query)
        if method == "GET" and parsed.path in ("/prom/det-state-metrics", "/debug/prom/metrics"):
            from determined_clone_amd.master import prom

            ctype, data = (prom.state_metrics(self.master) if parsed.path.startswith("/prom/")
                           else prom.process_metrics())
            return self._send_raw(200, ctype, data)
        if method == "GET" and not parsed.path.startswith(("/api/", "/oauth2/")):
            return self._static(parsed.path)
        try:
            body = json.loads(raw) if raw else None
        except ValueError:
            return self._send(400, {"error": "invalid JSON body"})
        for m, rx, fn, auth in ROUTES:
            if m != method:
                continue
            match = rx.match(parsed.path)
            if not match:
                continue
            user = None
            hdr = self.headers.get("Authorization", "")
            if hdr.startswith("Bearer "):
                user = self.master.user_for_token(hdr[7:])
            if auth and user is None:
                return self._send(401, {"error": "unauthenticated"})
            started = time.time()
            code, payload = 200, None
            try:
                out = fn(Req(self.master, match.groupdict(), query, body, user))
                payload = out if out is not None else {}
            except HTTPError as e:
                code, payload = e.status, {"error": str(e)}
            except KeyError as e:
                code, payload = 404, {"error": f"not found: {e}"}
            except Exception as e:  # pragma: no cover - surfaced to the client
                logger.error(traceback.format_exc())
                code, payload = 500, {"error": f"{type(e).__name__}: {e}"}
            self._send(code, payload)
            self._account(fn.__name__, method, parsed.path, code, started, user)
            return
        self._send(404, {"error": f"no route for {method} {parsed.path}"})

    def _send_raw(self, status: int, ctype: str, data: bytes) -> None:
        self.send_response(status)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    # task-plumbing endpoints polled/posted by every running task or agent: not audited
    _UNAUDITED = ("agent_events", "post_task_logs", "post_metrics", "trial_progress", "trial_heartbeat",
                  "profiler_metrics_batch", "runner_metadata", "agent_register", "alloc_allgather", "ack_preemption",
                  "alloc_ready", "alloc_proxy", "report_checkpoint", "trial_completed_op")

    def _account(self, handler: str, method: str, path: str, code: int, started: float,
                 user: Optional[Dict[str, Any]]) -> None:
        """Request metrics (/debug/prom/metrics) and the audit log: one structured line per
        user-initiated mutating call (reference: `master/internal/audit.go`)."""
        from determined_clone_amd.master import prom

        prom.observe(handler, method, code, started)
        if method != "GET" and handler not in self._UNAUDITED:
            audit_logger.info(json.dumps({
                "user": (user or {}).get("username"), "user_id": (user or {}).get("id"),
                "method": method, "path": path, "handler": handler, "status": code,
                "remote": self.client_address[0] if self.client_address else None,
                "ms": round((time.time() - started) * 1e3, 1)}))

    def _static(self, path: str) -> None:
        """The web UI (``determined_clone_amd/webui``): ``/`` redirects to ``/det/``."""
        from determined_clone_amd import webui

        if path == "/":
            self.send_response(302)
            self.send_header("Location", "/det/")
            self.send_header("Content-Length", "0")
            self.end_headers()
            return
        found = webui.resolve(path)
        if found is None:
            return self._send(404, {"error": f"no route for GET {path}"})
        ctype, body = found
        self.send_response(200)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self.send_header("Cache-Control", "no-cache")
        self.end_headers()
        self.wfile.write(body)

    # ------------------------------------------------------------------ task access
    def _task_access(self, user: Dict[str, Any], task_id: str) -> Optional[str]:
        """None when ``user`` may reach ``task_id``'s services through /proxy/ or /tunnel/, else
        why not. NTSC tasks: their owner (or an admin). Trials: the experiment's owner, an admin,
        or (``security.authz.type: rbac``) a holder of UPDATE_EXPERIMENT in its workspace -- a
        tunnel is a raw socket into the trial's container, so viewing rights are not enough
        (reference: `master/internal/proxy` + `ExperimentAuthZ.CanEditExperiment` under RBAC)."""
        if user.get("admin"):
            return None
        owner = self.master.task_owner(task_id)
        if owner is not None:
            return None if owner == user["id"] else "not the task owner"
        exp = self.master.task_experiment(task_id)
        if exp is None:
            return "not the task owner"
        if exp["owner_id"] == user["id"]:
            return None
        ws = _project_workspace(self.master, exp["project_id"])
        if self.master.authz.mode != "basic" and self.master.authz.permitted(user, "UPDATE_EXPERIMENT", ws):
            return None
        return f"not permitted on experiment {exp['id']}"

    def _task_ports(self, task_id: str, svc_port: Optional[int]) -> set:
        """Ports a tunnel may reach on a task's host: the service port it registered plus the
        ``environment.proxy_ports`` its config declares (reference: allocation.go registerProxies
        over ``req.ProxyPorts``)."""
        allowed = {svc_port} if svc_port else set()
        exp = self.master.task_experiment(task_id)
        cfg = exp["config"] if exp is not None else (self.master.tasks.get(task_id) or {}).get("config") or {}
        for pp in ((cfg.get("environment") or {}).get("proxy_ports") or []):
            try:
                allowed.add(int(pp["proxy_port"] if isinstance(pp, dict) else pp))
            except (KeyError, TypeError, ValueError):
                continue
        return allowed

    # ------------------------------------------------------------------ TCP tunnel
    def _task_host(self, task_id: str) -> Optional[Tuple[str, Optional[int]]]:
        """(host, service port) of a live task: its registered proxy address, else the first
        address of the agent running its first container; None when neither is known."""
        allocs = [a for a in list(self.master.allocations.values()) if a.task_id == task_id and not a.exited]
        if not allocs:
            return None
        a = allocs[0]
        if a.proxy_address:
            u = urllib.parse.urlsplit(a.proxy_address)
            return u.hostname or "127.0.0.1", u.port
        for p in a.placements:
            agent = self.master.rm.agents.get(p.get("agent_id"))
            if agent is not None and agent.addresses:
                return agent.addresses[0], None
        return None

    def _tunnel(self, parsed: Any, query: Dict[str, List[str]]) -> None:
        """``GET /tunnel/{task_id}?port=N`` with ``Upgrade: det-tcp``: after ``101 Switching
        Protocols`` the connection is a raw byte pipe to port N (default: the task's service port)
        on the task's host -- ssh into a shell, or ``det task tunnel -p`` to any port a trial
        opens (reference: the master's TCP-over-WebSocket proxy, `harness/determined/cli/
        tunnel.py` / `proxy.py`). Authenticated like ``/proxy/`` (``_task_access``); only the
        task's service port and its declared ``proxy_ports`` are reachable."""
        import socket
        import ssl

        task_id = parsed.path.split("/", 3)[2] if parsed.path.count("/") >= 2 else ""
        if self.headers.get("Upgrade", "").lower() != "det-tcp":
            return self._send(400, {"error": "tunnel requests must send 'Upgrade: det-tcp'"})
        user = self._proxy_user(query)
        if user is None:
            return self._send(401, {"error": "unauthenticated"})
        target = self._task_host(task_id)
        if target is None:
            return self._send(404, {"error": f"no running task {task_id}"})
        denied = self._task_access(user, task_id)
        if denied:
            return self._send(403, {"error": denied})
        host, svc_port = target
        try:
            port = int(query["port"][0]) if query.get("port") else svc_port
        except ValueError:
            return self._send(400, {"error": "port must be an integer"})
        if not port:
            return self._send(400, {"error": "task has no service port; pass ?port="})
        if port not in self._task_ports(task_id, svc_port):
            return self._send(403, {"error": f"port {port} is neither the task's service port nor "
                                             "one of its environment.proxy_ports"})
        try:
            upstream = socket.create_connection((host, port), timeout=10)
        except OSError as e:
            return self._send(502, {"error": f"cannot reach {host}:{port}: {e}"})
        upstream.settimeout(None)
        self.send_response(101, "Switching Protocols")
        self.send_header("Upgrade", "det-tcp")
        self.send_header("Connection", "Upgrade")
        self.end_headers()
        self.wfile.flush()
        self.close_connection = True
        client = self.connection
        client.settimeout(None)

        def pump(src: Any, dst: Any) -> None:
            try:
                while True:
                    data = src.recv(65536)
                    if not data:
                        break
                    dst.sendall(data)
            except OSError:
                pass
            finally:
                try:
                    # TLS has no half-close: end an HTTPS client's connection outright
                    if isinstance(dst, ssl.SSLSocket):
                        dst.close()
                    else:
                        dst.shutdown(socket.SHUT_WR)
                except OSError:
                    pass

        t = threading.Thread(target=pump, args=(upstream, client), daemon=True)
        t.start()
        pump(client, upstream)
        t.join()
        upstream.close()

    # ------------------------------------------------------------------ task proxy
    def _proxy_user(self, query: Dict[str, List[str]]) -> Optional[Dict[str, Any]]:
        hdr = self.headers.get("Authorization", "")
        token = hdr[7:] if hdr.startswith("Bearer ") else None
        if token is None:
            cookies = http.cookies.SimpleCookie(self.headers.get("Cookie", ""))
            token = cookies["auth"].value if "auth" in cookies else None
        if token is None and query.get("token"):
            token = query["token"][0]
        return self.master.user_for_token(token) if token else None

    def _proxy(self, method: str, parsed: Any, query: Dict[str, List[str]], raw: bytes) -> None:
        """Reverse proxy ``/proxy/{task_id}/<path>`` to the service a task registered with
        ``POST /api/v1/allocations/{id}/proxy_address`` (notebooks, shells, TensorBoards;
        reference: `master/internal/proxy`). Authenticated by bearer token, the ``auth`` cookie
        or ``?token=`` (browsers); a token in the query is moved into the cookie."""
        parts = parsed.path.split("/", 3)
        task_id = parts[2] if len(parts) > 2 else ""
        rest = "/" + (parts[3] if len(parts) > 3 else "")
        user = self._proxy_user(query)
        if user is None:
            return self._send(401, {"error": "unauthenticated"})
        alloc = next((a for a in list(self.master.allocations.values())
                      if a.task_id == task_id and not a.exited and a.proxy_address), None)
        if alloc is None:
            return self._send(404, {"error": f"no running service for task {task_id}"})
        denied = self._task_access(user, task_id)
        if denied:
            return self._send(403, {"error": denied})
        q = [(k, v) for k, vs in query.items() if k != "token" for v in vs]
        url = alloc.proxy_address.rstrip("/") + rest + ("?" + urllib.parse.urlencode(q) if q else "")
        fwd = {k: v for k, v in self.headers.items()
               if k.lower() not in ("host", "authorization", "cookie", "content-length", "connection",
                                    PROXY_SECRET_HEADER.lower())}
        fwd["X-Forwarded-Prefix"] = f"/proxy/{task_id}"
        secret = self.master.task_proxy_secret(task_id)
        if secret:
            fwd[PROXY_SECRET_HEADER] = secret
        try:
            req = urllib.request.Request(url, data=raw or None, method=method, headers=fwd)
            try:
                resp = urllib.request.urlopen(req, timeout=300)
            except urllib.error.HTTPError as e:
                resp = e
            body = resp.read()
            status = resp.status if hasattr(resp, "status") else resp.code
            self.send_response(status)
            for k, v in resp.headers.items():
                if k.lower() not in ("transfer-encoding", "connection", "content-length", "server", "date"):
                    self.send_header(k, v)
            if query.get("token"):
                self.send_header("Set-Cookie", f"auth={query['token'][0]}; Path=/proxy/{task_id}; HttpOnly")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)
        except (urllib.error.URLError, OSError) as e:
            self._send(502, {"error": f"task service unreachable: {e}"})

    def do_GET(self) -> None:
        self._dispatch("GET")

    def do_POST(self) -> None:
        self._dispatch("POST")

    def do_PATCH(self) -> None:
        self._dispatch("PATCH")

    def do_PUT(self) -> None:
        self._dispatch("PUT")

    def do_DELETE(self) -> None:
        self._dispatch("DELETE")


class MasterServer:
    """The master's HTTP(S) front end. ``tls``: master.yaml ``security.tls`` (``cert``, ``key``
    PEM files; reference `master/internal/config/config.go` TLSConfig) -- when given, every route,
    the proxy and the tunnels are served over TLS and ``master_url`` is ``https://``."""

    def __init__(self, master: Master, host: str = "127.0.0.1", port: int = 8080,
                 tls: Optional[Dict[str, str]] = None) -> None:
        handler = type("H", (_Handler,), {"master": master})
        self.httpd = ThreadingHTTPServer((host, port), handler)
        self.httpd.daemon_threads = True
        scheme = "http"
        if tls and (tls.get("cert") or tls.get("key")):
            if not (tls.get("cert") and tls.get("key")):
                raise ValueError("security.tls needs both cert and key")
            import ssl

            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.load_cert_chain(tls["cert"], tls["key"])
            # handshake lazily in the per-connection thread, not in the accept loop
            self.httpd.socket = ctx.wrap_socket(self.httpd.socket, server_side=True,
                                                do_handshake_on_connect=False)
            scheme = "https"
            base_handle_error = self.httpd.handle_error

            def handle_error(request: Any, client_address: Any) -> None:
                # a client that rejects our certificate (or speaks plain HTTP) ends its
                # handshake: one log line, not a traceback
                err = sys.exc_info()[1]
                if isinstance(err, (ssl.SSLError, ConnectionResetError)):
                    logger.info(f"TLS handshake with {client_address[0]} failed: {err}")
                    return
                base_handle_error(request, client_address)

            self.httpd.handle_error = handle_error
        self.master = master
        self.port = self.httpd.server_address[1]
        master.master_url = f"{scheme}://{host}:{self.port}"
        self._thread: Optional[threading.Thread] = None

    def start(self) -> "MasterServer":
        self._thread = threading.Thread(target=self.httpd.serve_forever, daemon=True, name="master-http")
        self._thread.start()
        self.master.rm.start_provisioners(self.master.master_url)
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
        self.master.rm.close()
        self.master.webhooks.close()  # undelivered events stay queued for the next master


# routes that live in their own modules register on import
from determined_clone_amd.master import api_extra, rbac_api, unmanaged_api  # noqa: E402,F401
