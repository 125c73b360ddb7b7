"""Remaining ``det`` commands (reference: `harness/determined/cli/{resources,dev,resource_pool,
workspace,project,master,job,experiment,trial,model,user,template,command,notebook,shell,
tensorboard}.py`): resource accounting CSVs, dev helpers (auth token, curl, raw API call),
resource-pool bindings, workspace/project listings and edits, master config show/set, batch job
updates, experiment TensorBoard-file deletion, trial support bundles, model move, user
rename/edit/agent-user link, template create/config/set-value, NTSC config/logs/priority."""
import argparse
import csv
import json
import os
import sys
import tarfile
import time
from typing import Any, Dict, List

import yaml

from determined_clone_amd.cli import cli as C


def _ws_id(s: Any, name: str) -> int:
    for w in s.get("/api/v1/workspaces")["workspaces"]:
        if w["name"] == name or str(w["id"]) == str(name):
            return int(w["id"])
    raise SystemExit(f"workspace {name!r} not found")


def _project_id(s: Any, ws: str, name: str) -> int:
    wid = _ws_id(s, ws)
    for p in s.get(f"/api/v1/workspaces/{wid}/projects")["projects"]:
        if p["name"] == name or str(p["id"]) == str(name):
            return int(p["id"])
    raise SystemExit(f"project {name!r} not found in workspace {ws!r}")


# ----------------------------------------------------------------------------- resources
def resources_raw(args):
    q = {"timestamp_after": _ts(args.start), "timestamp_before": _ts(args.end)}
    rows = C.session(args).get("/api/v1/resources/allocation/raw", params=q)["resource_entries"]
    _csv(rows, ["allocation_id", "task_id", "kind", "resource_pool", "start_time", "end_time", "slots", "seconds"])


def resources_aggregated(args):
    q = {"timestamp_after": _ts(args.start), "timestamp_before": _ts(args.end)}
    rows = C.session(args).get("/api/v1/resources/allocation/aggregated", params=q)["resource_entries"]
    out = []
    for r in rows:
        out.append({"period_start": r["period_start"], "seconds": r["seconds"],
                    **{f"pool:{k}": v for k, v in r["by_resource_pool"].items()},
                    **{f"kind:{k}": v for k, v in r["by_task_kind"].items()}})
    cols = sorted({k for r in out for k in r}, key=lambda k: (k != "period_start", k != "seconds", k))
    _csv(out, cols)


def _ts(v: str) -> float:
    if not v:
        return 0.0
    try:
        return float(v)
    except ValueError:
        return time.mktime(time.strptime(v, "%Y-%m-%d"))


def _csv(rows: List[Dict[str, Any]], cols: List[str]) -> None:
    w = csv.DictWriter(sys.stdout, fieldnames=cols, extrasaction="ignore")
    w.writeheader()
    for r in rows:
        w.writerow(r)


# ----------------------------------------------------------------------------- dev
def dev_auth_token(args):
    print(C.session(args).token)


def dev_curl(args):
    s = C.session(args)
    body = json.loads(args.data) if args.data else None
    print(json.dumps(s.request(args.method.upper(), args.path, body), indent=2, default=str))


def dev_call(args):
    """det dev call METHOD PATH [key=value ...]: JSON body from key=value pairs."""
    s = C.session(args)
    body: Dict[str, Any] = {}
    for kv in args.params:
        k, _, v = kv.partition("=")
        try:
            body[k] = json.loads(v)
        except ValueError:
            body[k] = v
    print(json.dumps(s.request(args.method.upper(), args.path, body or None), indent=2, default=str))


def dev_bindings_list(args):
    from determined_clone_amd.master.server import ROUTES

    for method, rx, fn, _ in ROUTES:
        print(f"{method:6s} {rx.pattern.strip('^$')}  ({fn.__name__})")


# ----------------------------------------------------------------------------- resource pools
def rp_bind(kind: str):
    def f(args):
        s = C.session(args)
        ids = [_ws_id(s, w) for w in args.workspace_names]
        path = f"/api/v1/resource-pools/{args.pool_name}/workspace-bindings"
        method = {"add": "POST", "remove": "DELETE", "replace": "PUT"}[kind]
        s.request(method, path, {"workspace_ids": ids})
    return f


def rp_list_workspaces(args):
    s = C.session(args)
    ids = s.get(f"/api/v1/resource-pools/{args.pool_name}/workspace-bindings")["workspace_ids"]
    names = {w["id"]: w["name"] for w in s.get("/api/v1/workspaces")["workspaces"]}
    C.render_table([{"id": i, "name": names.get(i)} for i in ids], ["id", "name"], args.json)


# ----------------------------------------------------------------------------- workspaces / projects
def workspace_list_projects(args):
    s = C.session(args)
    C.render_table(s.get(f"/api/v1/workspaces/{_ws_id(s, args.name)}/projects")["projects"],
                   ["id", "name", "num_experiments", "archived"], args.json)


def workspace_list_pools(args):
    s = C.session(args)
    print("\n".join(s.get(f"/api/v1/workspaces/{_ws_id(s, args.name)}/available-resource-pools")["resource_pool_names"]))


def workspace_edit(args):
    s = C.session(args)
    body: Dict[str, Any] = {}
    if args.name:
        body["name"] = args.name
    if args.checkpoint_storage_config_file:
        body["checkpoint_storage_config"] = C._read_config(args.checkpoint_storage_config_file)
    s.patch(f"/api/v1/workspaces/{_ws_id(s, args.workspace_name)}", body)


def project_list_experiments(args):
    s = C.session(args)
    pid = _project_id(s, args.workspace, args.name)
    C.render_table(s.get("/api/v1/experiments", params={"project_id": pid})["experiments"],
                   ["id", "name", "state", "progress", "archived"], args.json)


def project_edit(args):
    s = C.session(args)
    body = {k: v for k, v in (("name", args.new_name), ("description", args.description)) if v}
    s.patch(f"/api/v1/projects/{_project_id(s, args.workspace, args.name)}", body)


# ----------------------------------------------------------------------------- master / jobs
def master_config_show(args):
    cfg = C.session(args).get("/api/v1/master/config")["config"]
    print(json.dumps(cfg, indent=2) if args.json else yaml.safe_dump(cfg))


def master_config_set(args):
    body = {"config": {"log": {"level": args.log_level}}} if args.log_level else {"config": {}}
    C.session(args).patch("/api/v1/master/config", body)


def job_update_batch(args):
    """det job update-batch JOB_ID.priority=N JOB_ID.weight=W ..."""
    ups: Dict[str, Dict[str, Any]] = {}
    for item in args.updates:
        key, _, val = item.partition("=")
        jid, _, field = key.rpartition(".")
        if field not in ("priority", "weight") or not jid:
            raise SystemExit(f"bad update {item!r}: expected JOB_ID.priority=N or JOB_ID.weight=W")
        ups.setdefault(jid, {"job_id": jid})[field] = int(val) if field == "priority" else float(val)
    C.session(args).post("/api/v1/job-queues", {"updates": list(ups.values())})


# ----------------------------------------------------------------------------- experiments / trials / models
def experiment_delete_tb_files(args):
    C.session(args).delete(f"/api/v1/experiments/{args.experiment_id}/tensorboard-files")


def trial_support_bundle(args):
    """Tarball of a trial's description, metrics, checkpoints, logs and experiment config."""
    s = C.session(args)
    t = s.get(f"/api/v1/trials/{args.trial_id}")["trial"]
    parts = {
        "trial.json": t,
        "experiment.json": s.get(f"/api/v1/experiments/{t['experiment_id']}"),
        "metrics.json": s.get(f"/api/v1/trials/{args.trial_id}/metrics"),
        "checkpoints.json": s.get(f"/api/v1/trials/{args.trial_id}/checkpoints"),
        "logs.txt": "\n".join(x["log"] for x in s.get(f"/api/v1/trials/{args.trial_id}/logs")["logs"]),
    }
    out = os.path.join(args.output_dir or ".", f"det-bundle-trial-{args.trial_id}-{int(time.time())}.tar.gz")
    import io

    with tarfile.open(out, "w:gz") as tf:
        for name, obj in parts.items():
            data = (obj if isinstance(obj, str) else json.dumps(obj, indent=2, default=str)).encode()
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            tf.addfile(ti, io.BytesIO(data))
    print(out)


def model_move(args):
    s = C.session(args)
    s.post(f"/api/v1/models/{args.name}/move", {"destination_workspace_id": _ws_id(s, args.workspace_name)})


# ----------------------------------------------------------------------------- users
def _uid(s: Any, username: str) -> int:
    return int(s.get(f"/api/v1/users/{username}/by-username")["user"]["id"])


def user_rename(args):
    s = C.session(args)
    s.patch(f"/api/v1/users/{_uid(s, args.target_user)}", {"username": args.new_username})


def user_edit(args):
    s = C.session(args)
    body: Dict[str, Any] = {}
    if args.display_name is not None:
        body["display_name"] = args.display_name
    if args.username is not None:
        body["username"] = args.username
    if args.admin is not None:
        body["admin"] = args.admin
    if args.active is not None:
        body["active"] = args.active
    s.patch(f"/api/v1/users/{_uid(s, args.target_user)}", body)


def user_link_agent(args):
    s = C.session(args)
    s.patch(f"/api/v1/users/{_uid(s, args.det_username)}", {"agent_user_group": {
        "agent_uid": args.agent_uid, "agent_user": args.agent_user,
        "agent_gid": args.agent_gid, "agent_group": args.agent_group}})


# ----------------------------------------------------------------------------- templates
def template_create(args):
    C.session(args).post("/api/v1/templates", {"name": args.name, "config": C._read_config(args.template_file)})
    print(f"Created template {args.name}")


def template_config(args):
    t = C.session(args).get(f"/api/v1/templates/{args.name}")["template"]
    print(yaml.safe_dump(t["config"]))


def template_set_value(args):
    """det template set-value NAME key.path=value: patch one field of a template's config."""
    key, _, raw = args.assignment.partition("=")
    val: Any = yaml.safe_load(raw)
    patch: Dict[str, Any] = {}
    cur = patch
    parts = key.split(".")
    for p in parts[:-1]:
        cur = cur.setdefault(p, {})
    cur[parts[-1]] = val
    C.session(args).patch(f"/api/v1/templates/{args.name}", {"config": patch})


# ----------------------------------------------------------------------------- NTSC
def ntsc_config(path: str):
    def f(args):
        t = C.session(args).get(f"/api/v1/{path}/{args.task_id}")[path[:-1]]
        print(yaml.safe_dump({k: t.get(k) for k in ("entrypoint", "slots", "name", "priority") if k in t}))
    return f


def ntsc_logs(args):
    s = C.session(args)
    if args.follow:
        C._follow_logs(s, f"/api/v1/tasks/{args.task_id}/logs")
    else:
        for x in s.get(f"/api/v1/tasks/{args.task_id}/logs")["logs"]:
            print(x["log"])


def ntsc_priority(path: str):
    def f(args):
        C.session(args).post(f"/api/v1/{path}/{args.task_id}/set_priority", {"priority": args.priority})
    return f


def register(cmd, group, sub_lookup) -> None:
    """Attach to the parser built by ``cli.build_parser`` (``sub_lookup(name)`` returns an existing
    group's subparsers)."""
    r = group("resources res")
    for name, fn in (("raw", resources_raw), ("aggregated agg", resources_aggregated)):
        sp = cmd(r, name, fn)
        sp.add_argument("--start", default="")
        sp.add_argument("--end", default="")

    d = group("dev")
    cmd(d, "auth-token", dev_auth_token)
    sp = cmd(d, "curl c", dev_curl); sp.add_argument("path"); sp.add_argument("-X", "--method", default="GET")
    sp.add_argument("-d", "--data")
    sp = cmd(d, "call", dev_call); sp.add_argument("method"); sp.add_argument("path"); sp.add_argument("params", nargs="*")
    b = d.add_parser("bindings", aliases=["b"]).add_subparsers(dest="bcmd")
    cmd(b, "list ls", dev_bindings_list)

    rp = sub_lookup("resource-pool")
    bd = rp.add_parser("bindings").add_subparsers(dest="bindcmd")
    for name in ("add", "remove", "replace"):
        sp = cmd(bd, name, rp_bind(name)); sp.add_argument("pool_name"); sp.add_argument("workspace_names", nargs="*")
    sp = cmd(bd, "list-workspaces", rp_list_workspaces); sp.add_argument("pool_name")

    w = sub_lookup("workspace")
    sp = cmd(w, "list-projects", workspace_list_projects); sp.add_argument("name")
    sp = cmd(w, "list-pools", workspace_list_pools); sp.add_argument("name")
    sp = cmd(w, "edit", workspace_edit); sp.add_argument("workspace_name"); sp.add_argument("--name")
    sp.add_argument("--checkpoint-storage-config-file")
    p = sub_lookup("project")
    sp = cmd(p, "list-experiments", project_list_experiments); sp.add_argument("workspace"); sp.add_argument("name")
    sp = cmd(p, "edit", project_edit); sp.add_argument("workspace"); sp.add_argument("name")
    sp.add_argument("--new-name"); sp.add_argument("--description")

    m = sub_lookup("master")
    m_cfg = m.choices["config"]  # existing `det master config` stays the show command
    cs = m_cfg.add_subparsers(dest="cfgcmd")
    cmd(cs, "show", master_config_show)
    sp = cmd(cs, "set", master_config_set); sp.add_argument("--log-level")

    j = sub_lookup("job")
    sp = cmd(j, "update-batch", job_update_batch); sp.add_argument("updates", nargs="+")

    e = sub_lookup("experiment")
    sp = cmd(e, "delete-tb-files", experiment_delete_tb_files); sp.add_argument("experiment_id", type=int)
    t = sub_lookup("trial")
    sp = cmd(t, "support-bundle", trial_support_bundle); sp.add_argument("trial_id", type=int)
    sp.add_argument("-o", "--output-dir")
    mo = sub_lookup("model")
    sp = cmd(mo, "move", model_move); sp.add_argument("name"); sp.add_argument("workspace_name")

    u = sub_lookup("user")
    sp = cmd(u, "rename", user_rename); sp.add_argument("target_user"); sp.add_argument("new_username")
    sp = cmd(u, "edit", user_edit); sp.add_argument("target_user"); sp.add_argument("--display-name")
    sp.add_argument("--username")
    bool_ = lambda v: v.lower() in ("1", "true", "yes")  # noqa: E731
    sp.add_argument("--admin", type=bool_); sp.add_argument("--active", type=bool_)
    sp = cmd(u, "link-with-agent-user", user_link_agent); sp.add_argument("det_username")
    sp.add_argument("--agent-uid", type=int, required=True); sp.add_argument("--agent-gid", type=int, required=True)
    sp.add_argument("--agent-user", required=True); sp.add_argument("--agent-group", required=True)

    tp = sub_lookup("template")
    sp = cmd(tp, "create", template_create); sp.add_argument("name"); sp.add_argument("template_file")
    sp = cmd(tp, "config", template_config); sp.add_argument("name")
    sp = cmd(tp, "set-value", template_set_value); sp.add_argument("name"); sp.add_argument("assignment")

    for names, path in (("command", "commands"), ("notebook", "notebooks"), ("shell", "shells"),
                        ("tensorboard", "tensorboards")):
        g = sub_lookup(names)
        sp = cmd(g, "config", ntsc_config(path)); sp.add_argument("task_id")
        sp = cmd(g, "logs", ntsc_logs); sp.add_argument("task_id"); sp.add_argument("-f", "--follow", action="store_true")
        st = g.add_parser("set").add_subparsers(dest="setcmd")
        sp = cmd(st, "priority", ntsc_priority(path)); sp.add_argument("task_id"); sp.add_argument("priority", type=int)


_ = argparse
