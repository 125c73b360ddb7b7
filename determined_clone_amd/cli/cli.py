"""``det`` command-line interface (reference: `harness/determined/cli/*.py`).

Same command tree as the reference where it applies (experiment/e, trial/t, checkpoint, model,
template/tpl, agent/a, slot/s, task, command/cmd, shell, notebook, tensorboard, user/u, workspace,
project, job, resource-pool, master, deploy local, version), talking to the master's REST API.
"""
import argparse
import base64
import json
import os
import pathlib
import sys
import time
from typing import Any, Callable, Dict, List, Optional

import yaml

from determined_clone_amd import __version__
from determined_clone_amd.common.api import Session
from determined_clone_amd.errors import APIException, EnterpriseOnlyError

AUTH_FILE = pathlib.Path(os.environ.get("DET_CLONE_AUTH", pathlib.Path.home() / ".det-clone" / "auth.json"))


# ---------------------------------------------------------------------------- session helpers
def _load_tokens() -> Dict[str, Any]:
    try:
        return json.loads(AUTH_FILE.read_text())
    except (OSError, ValueError):
        return {}


def _save_tokens(d: Dict[str, Any]) -> None:
    AUTH_FILE.parent.mkdir(parents=True, exist_ok=True)
    AUTH_FILE.write_text(json.dumps(d))
    os.chmod(AUTH_FILE, 0o600)


def session(args: argparse.Namespace, login: bool = True) -> Session:
    s = Session(args.master)
    toks = _load_tokens().get(s.master, {})
    user = args.user or toks.get("active_user") or "admin"
    tok = (toks.get("tokens") or {}).get(user)
    if tok:
        s.token = tok
        try:
            s.get("/api/v1/me")
            return s
        except APIException:
            s.token = None
    if login:
        pw = os.environ.get("DET_PASS", "")
        r = s.post("/api/v1/auth/login", {"username": user, "password": pw})
        s.token = r["token"]
        d = _load_tokens()
        d.setdefault(s.master, {}).setdefault("tokens", {})[user] = s.token
        d[s.master]["active_user"] = user
        _save_tokens(d)
    return s


def render_table(rows: List[Dict[str, Any]], cols: List[str], as_json: bool = False) -> None:
    if as_json:
        print(json.dumps(rows, indent=2, default=str))
        return
    if not rows:
        print("(none)")
        return
    widths = {c: max(len(c), *(len(_fmt(r.get(c))) for r in rows)) for c in cols}
    print("  ".join(c.upper().ljust(widths[c]) for c in cols))
    print("  ".join("-" * widths[c] for c in cols))
    for r in rows:
        print("  ".join(_fmt(r.get(c)).ljust(widths[c]) for c in cols))


def _fmt(v: Any) -> str:
    if v is None:
        return ""
    if isinstance(v, float):
        if v > 1e9:
            return time.strftime("%Y-%m-%d %H:%M:%S", time.localtime(v))
        return f"{v:.6g}"
    if isinstance(v, (dict, list)):
        return json.dumps(v, default=str)
    return str(v)


# ---------------------------------------------------------------------------- user / master
def user_login(args):
    s = Session(args.master)
    import getpass

    pw = args.password if args.password is not None else (os.environ.get("DET_PASS") or getpass.getpass("Password: "))
    r = s.post("/api/v1/auth/login", {"username": args.username, "password": pw})
    d = _load_tokens()
    d.setdefault(s.master, {}).setdefault("tokens", {})[args.username] = r["token"]
    d[s.master]["active_user"] = args.username
    _save_tokens(d)
    print(f"logged in as {args.username}")


def user_logout(args):
    d = _load_tokens()
    m = Session(args.master).master
    d.pop(m, None)
    _save_tokens(d)


def user_whoami(args):
    print(f"You are logged in as user '{session(args).get('/api/v1/me')['user']['username']}'")


def user_list(args):
    render_table(session(args).get("/api/v1/users")["users"], ["id", "username", "admin", "active"], args.json)


def user_create(args):
    session(args).post("/api/v1/users", {"user": {"username": args.username, "admin": args.admin},
                                          "password": args.password or ""})


def user_set_active(active: bool):
    def f(args):
        s = session(args)
        u = [x for x in s.get("/api/v1/users")["users"] if x["username"] == args.username][0]
        s.patch(f"/api/v1/users/{u['id']}", {"active": active})
    return f


def user_change_password(args):
    s = session(args)
    name = args.target_user or s.get("/api/v1/me")["user"]["username"]
    u = [x for x in s.get("/api/v1/users")["users"] if x["username"] == name][0]
    s.post(f"/api/v1/users/{u['id']}/password", {"password": args.password})


def master_info(args):
    print(json.dumps(session(args, login=False).get("/api/v1/master"), indent=2))


def master_config(args):
    print(yaml.safe_dump(session(args).get("/api/v1/master/config")["config"]))


def version(args):
    print(f"client: {__version__}")
    try:
        print(f"master: {Session(args.master).get('/api/v1/master')['version']}")
    except Exception:
        print("master: unreachable")


# ---------------------------------------------------------------------------- experiments
def _read_config(path: str) -> Dict[str, Any]:
    with open(path) as f:
        return yaml.safe_load(f) or {}


def experiment_create(args):
    from determined_clone_amd.util import tar_directory

    cfg = _read_config(args.config_file)
    for kv in args.config or []:
        k, _, v = kv.partition("=")
        d = cfg
        parts = k.split(".")
        for p in parts[:-1]:
            d = d.setdefault(p, {})
        d[parts[-1]] = yaml.safe_load(v)
    if args.local:
        return _local_test(cfg, args.model_def) if args.test else _local_train(cfg, args.model_def)
    body: Dict[str, Any] = {"config": cfg, "activate": not args.paused}
    if args.model_def:
        body["model_definition"] = base64.b64encode(tar_directory(args.model_def)).decode()
    if args.template:
        body["template"] = args.template
    if args.project_id:
        body["project_id"] = args.project_id
    s = session(args)
    if args.test:
        return _cluster_test(s, body, cfg)
    exp = s.post("/api/v1/experiments", body)["experiment"]
    print(f"Created experiment {exp['id']}")
    if getattr(args, "publish", None):
        import threading

        threading.Thread(target=_publish_first_trial, args=(args, s, exp["id"]), daemon=True).start()
    if args.follow_first_trial:
        _follow_first_trial(s, exp["id"])
    elif getattr(args, "publish", None):
        _wait_terminal(s, exp["id"])


def _wait_terminal(s: Session, eid: int) -> str:
    while True:
        st = s.get(f"/api/v1/experiments/{eid}")["experiment"]["state"]
        if st in ("COMPLETED", "CANCELED", "ERROR", "DELETED"):
            return st
        time.sleep(2)


def _publish_first_trial(args, s: Session, eid: int) -> None:
    """``det e create -p LOCAL[:REMOTE]``: once the first trial has a task, serve the port map
    through the master's tunnel until the experiment ends (reference: `cli/proxy.py`
    tunnel_experiment)."""
    from determined_clone_amd.cli import tunnel

    task_id = None
    while task_id is None:
        ts = s.get(f"/api/v1/experiments/{eid}/trials")["trials"]
        task_id = next((t["task_id"] for t in ts if t.get("task_id")), None)
        if task_id is None:
            time.sleep(1)
    port_map = tunnel.parse_port_map(args.publish)
    with tunnel.listeners(s.master, s.token, task_id, port_map) as ports:
        for (local, remote), bound in zip(port_map.items(), ports):
            print(f"published 127.0.0.1:{bound} -> {task_id}:{remote}", flush=True)
        _wait_terminal(s, eid)


def _test_experiment_config(cfg: Dict[str, Any]) -> Dict[str, Any]:
    """The cluster test experiment (reference `_execution.py:77-120` _make_test_experiment_config):
    one batch, validation after it, no restarts, no kept checkpoints."""
    import uuid

    t = dict(cfg)
    t.update({
        "description": f"[test-mode] {t.get('description', str(uuid.uuid4()))}",
        "scheduling_unit": 1, "min_validation_period": {"batches": 1}, "max_restarts": 0,
        "checkpoint_storage": {**(t.get("checkpoint_storage") or {}), "save_experiment_best": 0,
                               "save_trial_best": 0, "save_trial_latest": 0},
        "searcher": {"name": "single", "metric": (t.get("searcher") or {}).get("metric", "validation_loss"),
                     "max_length": {"batches": 1}},
    })
    return t


def _cluster_test(s: Session, body: Dict[str, Any], cfg: Dict[str, Any]) -> None:
    """``det e create --test``: validate the config on the master, then run a one-batch test
    experiment on the cluster and follow it (reference `cli/experiment.py:269-281`)."""
    s.post("/api/v1/experiments", dict(body, validate_only=True))
    print("Experiment configuration validation succeeded")
    exp = s.post("/api/v1/experiments", dict(body, config=_test_experiment_config(cfg), activate=True))["experiment"]
    print(f"Created test experiment {exp['id']}")
    state = _wait_terminal(s, exp["id"])
    trials = s.get(f"/api/v1/experiments/{exp['id']}/trials")["trials"]
    if state != "COMPLETED":
        for t in trials[:1]:
            for line in s.get(f"/api/v1/trials/{t['id']}/logs")["logs"][-30:]:
                print(line["log"], end="" if line["log"].endswith("\n") else "\n")
        raise SystemExit(f"Test experiment {exp['id']} ended {state}")
    s.post(f"/api/v1/experiments/{exp['id']}/archive")
    print(f"Test experiment {exp['id']} completed successfully")


def _local_setup(cfg: Dict[str, Any], context: Optional[str]):
    from determined_clone_amd.config import expconf
    from determined_clone_amd.exec.harness import load_trial_class

    full = expconf.complete(cfg)
    if context:
        os.environ["DET_CONTEXT_DIR"] = os.path.abspath(context)
        if os.path.abspath(context) not in sys.path:
            sys.path.insert(0, os.path.abspath(context))
    hp = {k: (v.get("val") if isinstance(v, dict) and v.get("type") == "const" else
              v.get("minval") if isinstance(v, dict) and "minval" in v else
              (v.get("vals") or [None])[0] if isinstance(v, dict) and "vals" in v else v)
          for k, v in full["hyperparameters"].items()}
    return full, hp, load_trial_class(full["entrypoint"])


def _local_test(cfg: Dict[str, Any], context: Optional[str]) -> None:
    """``--local --test``: validate the config and run one batch of train + validate locally
    (reference `cli/experiment.py:327-354` local_experiment / test_one_batch)."""
    from determined_clone_amd import pytorch

    full, hp, cls = _local_setup(cfg, context)
    with pytorch.init(hparams=hp, exp_conf=full) as ctx:
        pytorch.Trainer(cls(ctx), ctx).fit(max_length=pytorch.Batch(1), test_mode=True,
                                           checkpoint_policy="none")
    print("Model definition test succeeded")


def _train_unit(spec: Any, gbs: Optional[int]):
    """An expconf length ({batches: N} / {epochs: N} / {records: N} / bare int = batches)."""
    from determined_clone_amd import pytorch

    if spec is None:
        return None
    if not isinstance(spec, dict):
        return pytorch.Batch(int(spec))
    unit, n = next(iter(spec.items()))
    if int(n) <= 0:  # expconf's "no period" default
        return None
    if unit == "epochs":
        return pytorch.Epoch(int(n))
    if unit == "records":
        return pytorch.Batch(max(1, -(-int(n) // int(gbs or 1))))
    return pytorch.Batch(int(n))


def _local_train(cfg: Dict[str, Any], context: Optional[str]) -> None:
    """``--local`` (without ``--test``): train one trial here, on this machine's GPUs, for the
    searcher's ``max_length`` with the config's validation / checkpoint periods -- no master.
    Hyperparameters take their const / first / lower-bound values. (The reference stops at
    ``--local --test``; full local training is this framework's addition.)"""
    from determined_clone_amd import pytorch

    full, hp, cls = _local_setup(cfg, context)
    gbs = hp.get("global_batch_size")
    max_length = _train_unit((full.get("searcher") or {}).get("max_length"), gbs)
    if max_length is None:
        raise SystemExit("--local training needs searcher.max_length")
    with pytorch.init(hparams=hp, exp_conf=full) as ctx:
        pytorch.Trainer(cls(ctx), ctx).fit(
            max_length=max_length,
            validation_period=_train_unit(full.get("min_validation_period"), gbs),
            checkpoint_period=_train_unit(full.get("min_checkpoint_period"), gbs),
            checkpoint_policy="all")
    unit = "epochs" if isinstance(max_length, pytorch.Epoch) else "batches"
    print(f"Local training finished ({max_length.value} {unit})")


def _follow_first_trial(s: Session, eid: int) -> None:
    tid = None
    while tid is None:
        ts = s.get(f"/api/v1/experiments/{eid}/trials")["trials"]
        if ts:
            tid = ts[0]["id"]
        else:
            time.sleep(1)
    _follow_logs(s, f"/api/v1/trials/{tid}/logs")


def _follow_logs(s: Session, path: str, follow: bool = True, tail: Optional[int] = None) -> None:
    after = 0
    first = True
    while True:
        r = s.get(path, params={"after_id": after, "follow": "true" if follow else "false",
                                "timeout_seconds": 5})
        logs = r["logs"]
        if first and tail is not None:
            logs = logs[-tail:]
        first = False
        for l in logs:
            print(l["log"])
            after = max(after, l["id"])
        if not follow or (r.get("done") and not r["logs"]):
            return


def experiment_list(args):
    params = {}
    if not args.all:
        params["archived"] = "false"
    exps = session(args).get("/api/v1/experiments", params=params)["experiments"]
    render_table(exps, ["id", "name", "state", "progress", "start_time", "end_time", "searcher_type",
                        "resource_pool"], args.json)


def experiment_describe(args):
    s = session(args)
    e = s.get(f"/api/v1/experiments/{args.experiment_id}")["experiment"]
    if args.json:
        trials = s.get(f"/api/v1/experiments/{args.experiment_id}/trials")["trials"]
        print(json.dumps({"experiment": e, "trials": trials}, indent=2, default=str))
        return
    render_table([e], ["id", "name", "state", "progress", "start_time", "end_time", "searcher_type", "labels"])
    print()
    trials = s.get(f"/api/v1/experiments/{args.experiment_id}/trials")["trials"]
    render_table(trials, ["id", "state", "hparams", "steps_completed", "best_validation", "restarts",
                          "latest_checkpoint"])


def experiment_config(args):
    print(yaml.safe_dump(session(args).get(f"/api/v1/experiments/{args.experiment_id}")["config"]))


def experiment_action(action: str):
    def f(args):
        session(args).post(f"/api/v1/experiments/{args.experiment_id}/{action}")
        print(f"{action}: experiment {args.experiment_id}")
    return f


def experiment_delete(args):
    session(args).delete(f"/api/v1/experiments/{args.experiment_id}")


def experiment_set(field: str):
    def f(args):
        session(args).patch(f"/api/v1/experiments/{args.experiment_id}", {field: args.value})
    return f


def experiment_label(add: bool):
    def f(args):
        s = session(args)
        labels = s.get(f"/api/v1/experiments/{args.experiment_id}")["experiment"]["labels"] or []
        labels = sorted(set(labels) | {args.label}) if add else [l for l in labels if l != args.label]
        s.patch(f"/api/v1/experiments/{args.experiment_id}", {"labels": labels})
    return f


def experiment_list_trials(args):
    render_table(session(args).get(f"/api/v1/experiments/{args.experiment_id}/trials")["trials"],
                 ["id", "state", "hparams", "steps_completed", "best_validation"], args.json)


def experiment_list_checkpoints(args):
    cks = session(args).get(f"/api/v1/experiments/{args.experiment_id}/checkpoints",
                            params={"sort_by": "searcher_metric"} if args.best else {})["checkpoints"]
    if args.best:
        cks = cks[:args.best]
    rows = [{"uuid": c["uuid"], "trial_id": c["training"]["trial_id"],
             "steps_completed": c["training"]["steps_completed"], "state": c["state"],
             "validation": ((c["training"].get("validation_metrics") or {}).get("avg_metrics"))} for c in cks]
    render_table(rows, ["uuid", "trial_id", "steps_completed", "state", "validation"], args.json)


def experiment_wait(args):
    s = session(args)
    while True:
        st = s.get(f"/api/v1/experiments/{args.experiment_id}")["experiment"]["state"]
        if st in ("COMPLETED", "CANCELED", "ERROR"):
            print(st)
            sys.exit(0 if st == "COMPLETED" else 1)
        time.sleep(args.polling_interval)


def experiment_download(args):
    s = session(args)
    cks = s.get(f"/api/v1/experiments/{args.experiment_id}/checkpoints", params={"sort_by": "searcher_metric"})["checkpoints"]
    for c in cks[:args.top_n]:
        _download_checkpoint(s, c["uuid"], os.path.join(args.output_dir, c["uuid"]))


def _overrides(cfg: Dict[str, Any], pairs: Optional[List[str]]) -> Dict[str, Any]:
    """Apply ``--config key.path=value`` overrides (values parsed as YAML)."""
    for kv in pairs or []:
        k, _, v = kv.partition("=")
        d = cfg
        parts = k.split(".")
        for p in parts[:-1]:
            d = d.setdefault(p, {})
        d[parts[-1]] = yaml.safe_load(v)
    return cfg


def experiment_continue(args):
    """``det e continue``: resume a terminal single-trial experiment with config overrides."""
    ov = _overrides(_read_config(args.config_file) if args.config_file else {}, args.config)
    s = session(args)
    e = s.post("/api/v1/experiments/continue", {"id": args.experiment_id, "override_config": ov})["experiment"]
    print(f"Continued experiment {e['id']}")
    if args.follow_first_trial:
        _follow_first_trial(s, e["id"])


def experiment_logs(args):
    s = session(args)
    trials = s.get(f"/api/v1/experiments/{args.experiment_id}/trials")["trials"]
    if not trials:
        raise SystemExit(f"experiment {args.experiment_id} has no trials yet")
    _follow_logs(s, f"/api/v1/trials/{trials[0]['id']}/logs", follow=args.follow, tail=args.tail)


def experiment_move(args):
    s = session(args)
    p = _project(s, args.workspace_name, args.project_name)
    s.post(f"/api/v1/experiments/{args.experiment_id}/move", {"destination_project_id": p["id"]})
    print(f"Moved experiment {args.experiment_id} to {args.workspace_name}/{args.project_name}")


def experiment_set_resource(field: str):
    def f(args):
        session(args).patch(f"/api/v1/experiments/{args.experiment_id}", {"resources": {field: args.value}})
        print(f"Set {field} of experiment {args.experiment_id} to {args.value}")
    return f


def experiment_set_gc_policy(args):
    policy = {k: getattr(args, k) for k in ("save_experiment_best", "save_trial_best", "save_trial_latest")}
    session(args).patch(f"/api/v1/experiments/{args.experiment_id}", {"checkpoint_storage": policy})
    print(f"Set GC policy of experiment {args.experiment_id}: {policy}")


def experiment_download_model_def(args):
    import io
    import tarfile

    b64 = session(args).get(f"/api/v1/experiments/{args.experiment_id}/model_def")["b64_tgz"]
    if not b64:
        raise SystemExit(f"experiment {args.experiment_id} has no model definition")
    out = args.output_dir or f"experiment_{args.experiment_id}_model_def"
    os.makedirs(out, exist_ok=True)
    with tarfile.open(fileobj=io.BytesIO(base64.b64decode(b64))) as tf:
        tf.extractall(out, filter="data")
    print(f"Downloaded model definition of experiment {args.experiment_id} to {out}")


def trial_download(args):
    s = session(args)
    cks = [c for c in s.get(f"/api/v1/trials/{args.trial_id}/checkpoints")["checkpoints"]
           if c["state"] == "COMPLETED"]
    if args.uuid:
        pick = args.uuid
    elif not cks:
        raise SystemExit(f"trial {args.trial_id} has no checkpoints")
    elif args.latest:
        pick = max(cks, key=lambda c: c["training"]["steps_completed"] or 0)["uuid"]
    else:
        metric = args.sort_by or s.get(f"/api/v1/experiments/{cks[0]['training']['experiment_id']}")[
            "config"]["searcher"].get("metric")

        def val(c):
            return ((c["training"].get("validation_metrics") or {}).get("avg_metrics") or {}).get(metric)

        scored = [c for c in cks if val(c) is not None]
        if not scored:
            raise SystemExit(f"no checkpoint of trial {args.trial_id} has a validation value of {metric}")
        pick = (min if args.smaller_is_better else max)(scored, key=val)["uuid"]
    out = args.output_dir or os.path.join("checkpoints", pick)
    _download_checkpoint(s, pick, out)
    if args.quiet:
        print(out)


def checkpoint_rm(args):
    session(args).post("/api/v1/checkpoints/rm", {"checkpoint_uuids": args.checkpoints_uuids.split(","),
                                                 "checkpoint_globs": args.glob})
    print(f"Removing files matching {args.glob} from checkpoints {args.checkpoints_uuids}")


def model_list_versions(args):
    r = session(args).get(f"/api/v1/models/{args.name}/versions")
    render_table([{"version": v["version"], "checkpoint": v["checkpoint"]["uuid"], "name": v.get("name"),
                   "comment": v.get("comment")} for v in r["model_versions"]],
                 ["version", "checkpoint", "name", "comment"], args.json)


def master_logs(args):
    s = session(args)
    after = 0
    first = True
    while True:
        params: Dict[str, Any] = {"after_id": after}
        if first and args.tail:
            params["tail"] = args.tail
        for e in s.get("/api/v1/master/logs", params=params)["logs"]:
            print(f"{_fmt(e['timestamp'])} [{e['level']}]: {e['message']}")
            after = max(after, e["id"])
        first = False
        if not args.follow:
            return
        time.sleep(1)


def _workspace(s: Session, name: str) -> Dict[str, Any]:
    for w in s.get("/api/v1/workspaces")["workspaces"]:
        if w["name"] == name:
            return w
    raise SystemExit(f"workspace {name} not found")


def _project(s: Session, ws: str, name: str) -> Dict[str, Any]:
    for p in s.get(f"/api/v1/workspaces/{_workspace(s, ws)['id']}/projects")["projects"]:
        if p["name"] == name:
            return p
    raise SystemExit(f"project {ws}/{name} not found")


def workspace_describe(args):
    s = session(args)
    w = _workspace(s, args.name)
    render_table([w], ["id", "name", "num_projects", "archived", "pinned"], args.json)
    if not args.json:
        render_table(s.get(f"/api/v1/workspaces/{w['id']}/projects")["projects"], ["id", "name", "num_experiments"])


def workspace_archive(archive: bool):
    def f(args):
        s = session(args)
        s.post(f"/api/v1/workspaces/{_workspace(s, args.name)['id']}/{'archive' if archive else 'unarchive'}")
    return f


def project_describe(args):
    s = session(args)
    p = _project(s, args.workspace, args.name)
    render_table([p], ["id", "name", "workspace_id", "num_experiments", "archived", "description"], args.json)
    if not args.json:
        exps = s.get("/api/v1/experiments", params={"project_id": p["id"]})["experiments"]
        render_table(exps, ["id", "name", "state", "progress"])


def project_delete(args):
    s = session(args)
    s.delete(f"/api/v1/projects/{_project(s, args.workspace, args.name)['id']}")


def project_archive(archive: bool):
    def f(args):
        s = session(args)
        s.post(f"/api/v1/projects/{_project(s, args.workspace, args.name)['id']}/{'archive' if archive else 'unarchive'}")
    return f


def preview_search(args):
    r = session(args).post("/api/v1/preview-hp-search", {"config": _read_config(args.config_file)})
    sim = r["simulation"]
    print(f"Using search method {_read_config(args.config_file)['searcher']['name']}: {sim['trials']} trials")
    rows = [{"trials": n, "training_lengths": k} for k, n in sim["results"].items()]
    render_table(rows, ["trials", "training_lengths"])


# ---------------------------------------------------------------------------- trials / checkpoints
def trial_describe(args):
    s = session(args)
    t = s.get(f"/api/v1/trials/{args.trial_id}")["trial"]
    if args.json:
        print(json.dumps(t, indent=2, default=str))
        return
    render_table([t], ["id", "experiment_id", "state", "steps_completed", "best_validation", "restarts", "hparams"])
    if args.metrics:
        ms = s.get(f"/api/v1/trials/{args.trial_id}/metrics")["metrics"]
        render_table([{"group": m["group"], "steps": m["steps_completed"], "metrics": m["metrics"]} for m in ms],
                     ["group", "steps", "metrics"])


def trial_logs(args):
    _follow_logs(session(args), f"/api/v1/trials/{args.trial_id}/logs", follow=args.follow, tail=args.tail)


def trial_kill(args):
    session(args).post(f"/api/v1/trials/{args.trial_id}/kill")


def _download_checkpoint(s: Session, uuid: str, out: str) -> None:
    from determined_clone_amd.common import storage

    c = s.get(f"/api/v1/checkpoints/{uuid}")["checkpoint"]
    sm = storage.build(c.get("storage") or {"type": "shared_fs", "host_path": "/tmp"})
    sm.download(uuid, out)
    print(f"downloaded checkpoint {uuid} to {out}")


def checkpoint_describe(args):
    print(json.dumps(session(args).get(f"/api/v1/checkpoints/{args.uuid}")["checkpoint"], indent=2, default=str))


def checkpoint_download(args):
    _download_checkpoint(session(args), args.uuid, args.output_dir or os.path.join("checkpoints", args.uuid))


def checkpoint_delete(args):
    session(args).request("DELETE", "/api/v1/checkpoints", body={"checkpoint_uuids": args.uuids})


# ---------------------------------------------------------------------------- model registry
def model_create(args):
    m = session(args).post("/api/v1/models", {"name": args.name, "description": args.description or ""})["model"]
    print(f"Created model {m['name']} (id {m['id']})")


def model_list(args):
    render_table(session(args).get("/api/v1/models")["models"], ["id", "name", "description", "num_versions", "archived"], args.json)


def model_describe(args):
    r = session(args).get(f"/api/v1/models/{args.name}/versions")
    render_table([r["model"]], ["id", "name", "description", "num_versions"])
    render_table([{"version": v["version"], "checkpoint": v["checkpoint"]["uuid"], "name": v["name"]}
                  for v in r["model_versions"]], ["version", "checkpoint", "name"])


def model_register(args):
    v = session(args).post(f"/api/v1/models/{args.name}/versions", {"checkpoint_uuid": args.uuid})["model_version"]
    print(f"Registered version {v['version']} of model {args.name}")


def model_delete(args):
    session(args).delete(f"/api/v1/models/{args.name}")


# ---------------------------------------------------------------------------- templates
def template_list(args):
    render_table(session(args).get("/api/v1/templates")["templates"], ["name", "config"], args.json)


def template_describe(args):
    print(yaml.safe_dump(session(args).get(f"/api/v1/templates/{args.name}")["template"]["config"]))


def template_set(args):
    session(args).put(f"/api/v1/templates/{args.name}", {"config": _read_config(args.template_file)})
    print(f"Set template {args.name}")


def template_remove(args):
    session(args).delete(f"/api/v1/templates/{args.name}")


# ---------------------------------------------------------------------------- cluster
def agent_list(args):
    rows = []
    for a in session(args).get("/api/v1/agents")["agents"]:
        rows.append({"id": a["id"], "resource_pool": a["resource_pool"], "enabled": a["enabled"],
                     "slots": len(a["slots"]), "containers": sum(1 for s in a["slots"].values() if s["container"])})
    render_table(rows, ["id", "resource_pool", "enabled", "slots", "containers"], args.json)


def agent_enable(enable: bool):
    def f(args):
        session(args).post(f"/api/v1/agents/{args.agent_id}/{'enable' if enable else 'disable'}",
                           {"drain": bool(getattr(args, "drain", False))})
    return f


def slot_list(args):
    rows = []
    for a in session(args).get("/api/v1/agents")["agents"]:
        for sid, sl in a["slots"].items():
            rows.append({"agent_id": a["id"], "slot_id": sid, "enabled": sl["enabled"],
                         "type": sl["device"].get("type"), "uuid": sl["device"].get("uuid"),
                         "allocation": (sl["container"] or {}).get("id")})
    render_table(rows, ["agent_id", "slot_id", "enabled", "type", "uuid", "allocation"], args.json)


def slot_enable(enable: bool):
    def f(args):
        session(args).post(f"/api/v1/agents/{args.agent_id}/slots/{args.slot_id}/{'enable' if enable else 'disable'}")
    return f


def resource_pool_list(args):
    render_table(session(args).get("/api/v1/resource-pools")["resource_pools"],
                 ["name", "num_agents", "slots_available", "slots_used", "scheduler_type", "slot_type"], args.json)


def job_list(args):
    render_table(session(args).get("/api/v1/job-queues")["jobs"],
                 ["job_id", "name", "state", "slots", "priority", "weight", "resource_pool", "position"], args.json)


def job_update(args):
    u: Dict[str, Any] = {"job_id": args.job_id}
    if args.priority is not None:
        u["priority"] = args.priority
    if args.weight is not None:
        u["weight"] = args.weight
    session(args).post("/api/v1/job-queues", {"updates": [u]})


def task_list(args):
    render_table(session(args).get("/api/v1/tasks")["tasks"], ["task_id", "type", "state", "name"], args.json)


def task_logs(args):
    _follow_logs(session(args), f"/api/v1/tasks/{args.task_id}/logs", follow=args.follow)


def cmd_run(kind: str, path: str):
    def f(args):
        s = session(args)
        body: Dict[str, Any] = {"config": {"resources": {"slots": args.slots}}}
        if getattr(args, "entrypoint", None):
            body["entrypoint"] = args.entrypoint
        if getattr(args, "experiment_ids", None):
            body["experiment_ids"] = args.experiment_ids
        if getattr(args, "context", None):
            from determined_clone_amd.util import tar_directory

            body["files"] = base64.b64encode(tar_directory(args.context)).decode()
        t = s.post(f"/api/v1/{path}", body)[path[:-1]]
        print(f"Launched {kind.lower()} {t['id']}")
        if kind == "COMMAND" and not args.detach:
            _follow_logs(s, f"/api/v1/tasks/{t['id']}/logs")
    return f


def cmd_list(path: str):
    def f(args):
        render_table(session(args).get(f"/api/v1/{path}")[path], ["id", "state", "entrypoint", "slots"], args.json)
    return f


def cmd_kill(path: str):
    def f(args):
        session(args).post(f"/api/v1/{path}/{args.task_id}/kill")
    return f


def _wait_service(s: Session, path: str, task_id: str, timeout: float = 120.0) -> str:
    """Proxy URL of a running NTSC task once its service registered (``/proxy/<task_id>/``)."""
    t0 = time.time()
    while time.time() - t0 < timeout:
        t = s.get(f"/api/v1/{path}/{task_id}")[path[:-1]]
        if t.get("state") == "TERMINATED":
            raise SystemExit(f"task {task_id} terminated")
        if t.get("service_ready"):
            return f"{s.master}/proxy/{task_id}/"
        time.sleep(0.5)
    raise SystemExit(f"task {task_id}: service not ready after {timeout:.0f}s")


def ntsc_open(path: str):
    """det notebook|tensorboard open ID: print (and try to open) the proxied URL."""
    def f(args):
        s = session(args)
        url = _wait_service(s, path, args.task_id) + f"?token={s.token}"
        print(url)
        if not args.no_browser:
            import webbrowser

            webbrowser.open(url)
    return f


def shell_open(args):
    """det shell open ID: interactive session over the master proxy (stdin lines -> terminal)."""
    import threading

    s = session(args)
    base = _wait_service(s, "shells", args.task_id).rstrip("/")
    state = {"next": 0, "closed": False}

    def pump() -> None:
        while not state["closed"]:
            out = s.get(base[len(s.master):] + "/output", params={"since": state["next"], "wait": 10})
            sys.stdout.write(out["data"])
            sys.stdout.flush()
            state["next"], state["closed"] = out["next"], out["closed"]

    th = threading.Thread(target=pump, daemon=True)
    th.start()
    try:
        for line in sys.stdin:
            s.post(base[len(s.master):] + "/input", {"data": line})
            if line.strip() == "exit":
                break
    except KeyboardInterrupt:
        pass
    time.sleep(0.5)
    state["closed"] = True


def shell_show_ssh_command(args):
    """det shell show-ssh-command ID [SSH_OPTS...]: the ssh command (e.g. for an IDE's remote
    interpreter) that reaches the shell task through the master's TCP tunnel as ProxyCommand
    (reference: cli/shell.py show_ssh_command). It needs an sshd serving the task's port in its
    container image; without one use ``det shell open`` / ``det shell run``."""
    import shlex

    s = session(args)
    t = s.get(f"/api/v1/shells/{args.task_id}")
    shell = t.get("shell", t)
    proxy = (f"{shlex.quote(sys.executable)} -m determined_clone_amd.cli.tunnel {s.master} %h"
             f" --token {s.token}")
    user = (shell.get("agent_user_group") or {}).get("agent_user") or os.environ.get("USER", "root")
    opts = " ".join(shlex.quote(o) for o in (args.ssh_opts or []))
    print(f"ssh -o {shlex.quote('ProxyCommand=' + proxy)} -o StrictHostKeyChecking=no "
          f"-o IdentitiesOnly=yes {opts + ' ' if opts else ''}{user}@{args.task_id}")


def shell_run(args):
    """det shell run ID -- CMD...: one command in the shell task's container."""
    s = session(args)
    base = _wait_service(s, "shells", args.task_id).rstrip("/")
    cmdline = " ".join(args.command[1:] if args.command[:1] == ["--"] else args.command)
    out = s.post(base[len(s.master):] + "/run", {"cmd": cmdline})
    sys.stdout.write(out["output"])
    sys.exit(out["exit_code"])


def workspace_list(args):
    render_table(session(args).get("/api/v1/workspaces")["workspaces"], ["id", "name", "num_projects", "archived"], args.json)


def workspace_create(args):
    w = session(args).post("/api/v1/workspaces", {"name": args.name})["workspace"]
    print(f"Created workspace {w['name']} (id {w['id']})")


def workspace_delete(args):
    s = session(args)
    w = [x for x in s.get("/api/v1/workspaces")["workspaces"] if x["name"] == args.name][0]
    s.delete(f"/api/v1/workspaces/{w['id']}")


def project_list(args):
    s = session(args)
    w = [x for x in s.get("/api/v1/workspaces")["workspaces"] if x["name"] == args.workspace][0]
    render_table(s.get(f"/api/v1/workspaces/{w['id']}/projects")["projects"], ["id", "name", "num_experiments"], args.json)


def project_create(args):
    s = session(args)
    w = [x for x in s.get("/api/v1/workspaces")["workspaces"] if x["name"] == args.workspace][0]
    p = s.post(f"/api/v1/workspaces/{w['id']}/projects", {"name": args.name})["project"]
    print(f"Created project {p['name']} (id {p['id']})")


def _serve_tunnels(args, s, task_id: str) -> None:
    import threading

    from determined_clone_amd.cli import tunnel

    port_map = tunnel.parse_port_map(args.publish)
    if not port_map:
        raise SystemExit("pass at least one -p LOCAL[:REMOTE]")
    with tunnel.listeners(s.master, s.token, task_id, port_map) as ports:
        for (local, remote), bound in zip(port_map.items(), ports):
            print(f"127.0.0.1:{bound} -> {task_id}:{remote}", flush=True)
        try:
            threading.Event().wait()
        except KeyboardInterrupt:
            pass


def task_tunnel(args):
    """det task tunnel TASK -p LOCAL[:REMOTE]: forward local ports to a running task's ports
    through the master (reference: `cli/proxy.py` _tunnel_task / --publish)."""
    _serve_tunnels(args, session(args), args.task_id)


def experiment_tunnel(args):
    """det experiment tunnel EXP -p ...: the experiment's first running trial."""
    s = session(args)
    trials = s.get(f"/api/v1/experiments/{args.experiment_id}/trials")["trials"]
    live = [t for t in trials if t.get("task_id") and t.get("state") in ("RUNNING", "ACTIVE")]
    if not live:
        raise SystemExit(f"experiment {args.experiment_id} has no running trial")
    _serve_tunnels(args, s, live[0]["task_id"])


def deploy_local(args):
    from determined_clone_amd.deploy import local

    {"cluster-up": local.cluster_up, "cluster-down": local.cluster_down,
     "master-up": local.master_up, "agent-up": local.agent_up}[args.deploy_cmd](args)


# ---------------------------------------------------------------------------- parser
def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="det", description="determined_clone_amd CLI")
    p.add_argument("-m", "--master", default=os.environ.get("DET_MASTER", "http://127.0.0.1:8080"))
    p.add_argument("-u", "--user", default=os.environ.get("DET_USER"))
    p.add_argument("--json", action="store_true", help="JSON output")
    sub = p.add_subparsers(dest="cmd")

    def cmd(parent, names, fn, help_=""):
        name, *aliases = names.split()
        sp = parent.add_parser(name, aliases=aliases, help=help_)
        sp.set_defaults(func=fn)
        return sp

    groups: Dict[str, Any] = {}

    def group(names, help_=""):
        name, *aliases = names.split()
        g = sub.add_parser(name, aliases=aliases, help=help_)
        groups[name] = g.add_subparsers(dest="subcmd")
        return groups[name]

    cmd(sub, "version", version)
    u = group("user u")
    sp = cmd(u, "login", user_login); sp.add_argument("username", nargs="?", default="admin"); sp.add_argument("--password")
    cmd(u, "logout", user_logout)
    cmd(u, "whoami", user_whoami)
    cmd(u, "list ls", user_list)
    sp = cmd(u, "create", user_create); sp.add_argument("username"); sp.add_argument("--admin", action="store_true"); sp.add_argument("--password")
    sp = cmd(u, "activate", user_set_active(True)); sp.add_argument("username")
    sp = cmd(u, "deactivate", user_set_active(False)); sp.add_argument("username")
    sp = cmd(u, "change-password", user_change_password); sp.add_argument("target_user", nargs="?"); sp.add_argument("--password", required=True)

    m = group("master")
    cmd(m, "info", master_info)
    cmd(m, "config", master_config)
    sp = cmd(m, "logs", master_logs); sp.add_argument("-f", "--follow", action="store_true"); sp.add_argument("--tail", type=int)

    e = group("experiment e")
    sp = cmd(e, "create", experiment_create)
    sp.add_argument("config_file"); sp.add_argument("model_def", nargs="?")
    sp.add_argument("--paused", action="store_true"); sp.add_argument("--test", "--test-mode", dest="test", action="store_true")
    sp.add_argument("--local", action="store_true",
                    help="run here instead of on the cluster (with --test: one batch; without: the whole trial)")
    sp.add_argument("--template"); sp.add_argument("--project-id", type=int)
    sp.add_argument("--config", action="append", help="override: key.path=value")
    sp.add_argument("-f", "--follow-first-trial", action="store_true")
    sp.add_argument("-p", "--publish", action="append", default=[],
                    help="LOCAL[:REMOTE]: forward a local port to the first trial's port (repeatable)")
    sp = cmd(e, "list ls", experiment_list); sp.add_argument("--all", "-a", action="store_true")
    for name, fn in (("describe", experiment_describe), ("config", experiment_config),
                     ("list-trials lt", experiment_list_trials), ("delete", experiment_delete),
                     ("activate", experiment_action("activate")), ("pause", experiment_action("pause")),
                     ("cancel", experiment_action("cancel")), ("kill", experiment_action("kill")),
                     ("archive", experiment_action("archive")), ("unarchive", experiment_action("unarchive"))):
        sp = cmd(e, name, fn); sp.add_argument("experiment_id", type=int)
    sp = cmd(e, "list-checkpoints lc", experiment_list_checkpoints); sp.add_argument("experiment_id", type=int); sp.add_argument("--best", type=int)
    sp = cmd(e, "wait", experiment_wait); sp.add_argument("experiment_id", type=int); sp.add_argument("--polling-interval", type=float, default=5)
    sp = cmd(e, "download", experiment_download); sp.add_argument("experiment_id", type=int); sp.add_argument("--top-n", type=int, default=1); sp.add_argument("--output-dir", default="checkpoints")
    sp = cmd(e, "preview-search", preview_search); sp.add_argument("config_file")
    for field in ("description", "name"):
        sp = cmd(e, f"set-{field}", experiment_set(field)); sp.add_argument("experiment_id", type=int); sp.add_argument("value")
    lab = e.add_parser("label").add_subparsers(dest="labelcmd")
    for name, add in (("add", True), ("remove", False)):
        sp = cmd(lab, name, experiment_label(add)); sp.add_argument("experiment_id", type=int); sp.add_argument("label")
    sp = cmd(e, "continue", experiment_continue); sp.add_argument("experiment_id", type=int)
    sp.add_argument("--config-file"); sp.add_argument("--config", action="append", help="override: key.path=value")
    sp.add_argument("-f", "--follow-first-trial", action="store_true")
    sp = cmd(e, "logs", experiment_logs); sp.add_argument("experiment_id", type=int)
    sp.add_argument("-f", "--follow", action="store_true"); sp.add_argument("--tail", type=int)
    sp = cmd(e, "move", experiment_move); sp.add_argument("experiment_id", type=int)
    sp.add_argument("workspace_name"); sp.add_argument("project_name")
    sp = cmd(e, "download-model-def", experiment_download_model_def); sp.add_argument("experiment_id", type=int)
    sp.add_argument("--output-dir", "-o")
    st = e.add_parser("set").add_subparsers(dest="setcmd")
    for field in ("description", "name"):
        sp = cmd(st, field, experiment_set(field)); sp.add_argument("experiment_id", type=int); sp.add_argument("value")
    for field, typ in (("max-slots", int), ("weight", float), ("priority", int)):
        sp = cmd(st, field, experiment_set_resource(field.replace("-", "_")))
        sp.add_argument("experiment_id", type=int); sp.add_argument("value", type=typ)
    sp = cmd(st, "gc-policy", experiment_set_gc_policy); sp.add_argument("experiment_id", type=int)
    for k in ("--save-experiment-best", "--save-trial-best", "--save-trial-latest"):
        sp.add_argument(k, type=int, required=True)

    t = group("trial t")
    sp = cmd(t, "describe", trial_describe); sp.add_argument("trial_id", type=int); sp.add_argument("--metrics", action="store_true")
    sp = cmd(t, "logs", trial_logs); sp.add_argument("trial_id", type=int); sp.add_argument("-f", "--follow", action="store_true"); sp.add_argument("--tail", type=int)
    sp = cmd(t, "kill", trial_kill); sp.add_argument("trial_id", type=int)
    sp = cmd(t, "download", trial_download); sp.add_argument("trial_id", type=int)
    pick = sp.add_mutually_exclusive_group(required=True)
    pick.add_argument("--best", action="store_true"); pick.add_argument("--latest", action="store_true")
    pick.add_argument("--uuid")
    sp.add_argument("--sort-by"); sp.add_argument("--smaller-is-better", type=lambda v: v.lower() != "false", default=True)
    sp.add_argument("-o", "--output-dir"); sp.add_argument("-q", "--quiet", action="store_true")

    c = group("checkpoint")
    sp = cmd(c, "describe", checkpoint_describe); sp.add_argument("uuid")
    sp = cmd(c, "download", checkpoint_download); sp.add_argument("uuid"); sp.add_argument("--output-dir", "-o")
    sp = cmd(c, "delete", checkpoint_delete); sp.add_argument("uuids", nargs="+")
    sp = cmd(c, "rm", checkpoint_rm); sp.add_argument("checkpoints_uuids", help="comma-separated")
    sp.add_argument("--glob", action="append", default=[])

    mo = group("model")
    sp = cmd(mo, "create", model_create); sp.add_argument("name"); sp.add_argument("--description")
    cmd(mo, "list ls", model_list)
    sp = cmd(mo, "describe", model_describe); sp.add_argument("name")
    sp = cmd(mo, "register-version", model_register); sp.add_argument("name"); sp.add_argument("uuid")
    sp = cmd(mo, "list-versions", model_list_versions); sp.add_argument("name")
    sp = cmd(mo, "delete", model_delete); sp.add_argument("name")

    tp = group("template tpl")
    cmd(tp, "list ls", template_list)
    sp = cmd(tp, "describe", template_describe); sp.add_argument("name")
    sp = cmd(tp, "set", template_set); sp.add_argument("name"); sp.add_argument("template_file")
    sp = cmd(tp, "remove rm", template_remove); sp.add_argument("name")

    a = group("agent a")
    cmd(a, "list ls", agent_list)
    sp = cmd(a, "enable", agent_enable(True)); sp.add_argument("agent_id")
    sp = cmd(a, "disable", agent_enable(False)); sp.add_argument("agent_id"); sp.add_argument("--drain", action="store_true")
    sl = group("slot s")
    cmd(sl, "list ls", slot_list)
    sp = cmd(sl, "enable", slot_enable(True)); sp.add_argument("agent_id"); sp.add_argument("slot_id", type=int)
    sp = cmd(sl, "disable", slot_enable(False)); sp.add_argument("agent_id"); sp.add_argument("slot_id", type=int)
    rp = group("resource-pool rp")
    cmd(rp, "list ls", resource_pool_list)
    j = group("job")
    cmd(j, "list ls", job_list)
    sp = cmd(j, "update", job_update); sp.add_argument("job_id"); sp.add_argument("--priority", type=int); sp.add_argument("--weight", type=float)
    tk = group("task")
    cmd(tk, "list ls", task_list)
    sp = cmd(tk, "logs", task_logs); sp.add_argument("task_id"); sp.add_argument("-f", "--follow", action="store_true")
    sp = cmd(tk, "tunnel", task_tunnel); sp.add_argument("task_id")
    sp.add_argument("-p", "--publish", action="append", default=[], help="LOCAL[:REMOTE] port (repeatable)")
    sp = cmd(groups["experiment"], "tunnel", experiment_tunnel); sp.add_argument("experiment_id", type=int)
    sp.add_argument("-p", "--publish", action="append", default=[], help="LOCAL[:REMOTE] port (repeatable)")

    for kind, names, path in (("COMMAND", "command cmd", "commands"), ("SHELL", "shell", "shells"),
                              ("NOTEBOOK", "notebook", "notebooks"), ("TENSORBOARD", "tensorboard", "tensorboards")):
        g = group(names)
        sp = cmd(g, "run" if kind == "COMMAND" else "start", cmd_run(kind, path))
        sp.add_argument("--slots", type=int, default=0)
        sp.add_argument("--context", "-c")
        if kind == "COMMAND":
            sp.add_argument("entrypoint", nargs=argparse.REMAINDER)
            sp.add_argument("-d", "--detach", action="store_true")
        if kind == "TENSORBOARD":
            sp.add_argument("experiment_ids", nargs="*", type=int)
        cmd(g, "list ls", cmd_list(path))
        sp = cmd(g, "kill", cmd_kill(path)); sp.add_argument("task_id")
        if kind in ("NOTEBOOK", "TENSORBOARD"):
            sp = cmd(g, "open", ntsc_open(path)); sp.add_argument("task_id")
            sp.add_argument("--no-browser", action="store_true")
        if kind == "SHELL":
            sp = cmd(g, "open", shell_open); sp.add_argument("task_id")
            for name in ("show-ssh-command", "show_ssh_command"):
                sp = cmd(g, name, shell_show_ssh_command); sp.add_argument("task_id")
                sp.add_argument("ssh_opts", nargs="*", help="additional ssh options")
            sp = cmd(g, "run", shell_run); sp.add_argument("task_id")
            sp.add_argument("command", nargs=argparse.REMAINDER)

    w = group("workspace")
    cmd(w, "list ls", workspace_list)
    sp = cmd(w, "create", workspace_create); sp.add_argument("name")
    sp = cmd(w, "delete", workspace_delete); sp.add_argument("name")
    sp = cmd(w, "describe", workspace_describe); sp.add_argument("name")
    sp = cmd(w, "archive", workspace_archive(True)); sp.add_argument("name")
    sp = cmd(w, "unarchive", workspace_archive(False)); sp.add_argument("name")
    pr = group("project p")
    sp = cmd(pr, "list ls", project_list); sp.add_argument("workspace")
    sp = cmd(pr, "create", project_create); sp.add_argument("workspace"); sp.add_argument("name")
    for name, fn in (("describe", project_describe), ("delete", project_delete),
                     ("archive", project_archive(True)), ("unarchive", project_archive(False))):
        sp = cmd(pr, name, fn); sp.add_argument("workspace"); sp.add_argument("name")

    from determined_clone_amd.cli import rbac as rbac_cli

    rbac_cli.register(cmd, group)

    from determined_clone_amd.cli import sso as sso_cli

    sso_cli.register(cmd, group)

    from determined_clone_amd.cli import extra as extra_cli

    extra_cli.register(cmd, group, groups.__getitem__)

    d = group("deploy")
    from determined_clone_amd.deploy import cli as deploy_cli

    deploy_cli.register(d)
    lo = d.add_parser("local").add_subparsers(dest="deploy_cmd")
    for name in ("cluster-up", "cluster-down", "master-up", "agent-up"):
        sp = lo.add_parser(name)
        sp.set_defaults(func=deploy_local)
        sp.add_argument("--master-port", type=int, default=8080)
        sp.add_argument("--agents", type=int, default=1)
        sp.add_argument("--artificial-slots", type=int, default=0)
        sp.add_argument("--slots-per-gpu", type=int, default=1)
        sp.add_argument("--storage-path", default=None)
        sp.add_argument("--state-dir", default=os.path.join(os.path.expanduser("~"), ".det-clone"))
    return p


def main(argv: Optional[List[str]] = None) -> int:
    p = build_parser()
    args = p.parse_args(argv)
    if not getattr(args, "func", None):
        p.print_help()
        return 1
    try:
        args.func(args)
    except (APIException, EnterpriseOnlyError) as e:
        print(f"Error: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
