"""The remaining v1 REST routes (reference: api.proto): bulk experiment actions, file tree,
metric streams, workloads, metric reports, user settings, slots, job stats, NTSC priority,
resource accounting, project/workspace archive + move, resource-pool bindings, route precedence."""
import base64
import json
import os
import shutil
import tempfile
import time

import pytest

from determined_clone_amd.agent import Agent
from determined_clone_amd.common.api import Session
from determined_clone_amd.errors import APIException
from determined_clone_amd.master import Master, MasterServer
from determined_clone_amd.util import tar_directory
from tests.test_cluster_e2e import MODEL_DEF

CFG = {"name": "api-extra", "entrypoint": "model_def:OneVar",
       "hyperparameters": {"global_batch_size": 4, "lr": 0.1},
       "searcher": {"name": "single", "metric": "val_loss", "max_length": {"batches": 4}},
       "min_validation_period": {"batches": 2}, "min_checkpoint_period": {"batches": 2},
       "resources": {"slots_per_trial": 1}, "max_restarts": 0, "labels": ["a"]}


@pytest.fixture(scope="module")
def env():
    tmp = tempfile.mkdtemp(prefix="det-api-")
    m = Master(os.path.join(tmp, "m.db"), checkpoint_storage={"type": "shared_fs", "host_path": os.path.join(tmp, "ckpt")})
    srv = MasterServer(m, "127.0.0.1", 0).start()
    agent = Agent(m.master_url, "agent-0", artificial_slots=2).start_background()
    s = Session(m.master_url)
    s.token = s.post("/api/v1/auth/login", {"username": "admin", "password": ""})["token"]
    ctx = os.path.join(tmp, "ctx")
    os.makedirs(os.path.join(ctx, "sub"))
    with open(os.path.join(ctx, "model_def.py"), "w") as f:
        f.write(MODEL_DEF)
    with open(os.path.join(ctx, "sub", "data.txt"), "w") as f:
        f.write("hello")
    body = {"config": CFG, "model_definition": base64.b64encode(tar_directory(ctx)).decode()}
    eid = s.post("/api/v1/experiments", body)["experiment"]["id"]
    t0 = time.time()
    while s.get(f"/api/v1/experiments/{eid}")["experiment"]["state"] != "COMPLETED":
        assert time.time() - t0 < 240
        time.sleep(0.5)
    yield m, s, eid, body
    agent.stop()
    srv.stop()
    shutil.rmtree(tmp, ignore_errors=True)


def test_files_labels_search_and_streams(env):
    m, s, eid, _ = env
    tree = s.get(f"/api/v1/experiments/{eid}/file_tree")["files"]
    names = {f["name"] for f in tree}
    assert {"model_def.py", "sub"} <= names
    sub = next(f for f in tree if f["name"] == "sub")
    assert sub["is_dir"] and sub["files"][0]["path"] == "sub/data.txt"
    f = s.post(f"/api/v1/experiments/{eid}/file", {"path": "sub/data.txt"})["file"]
    assert base64.b64decode(f) == b"hello"
    s.put(f"/api/v1/experiments/{eid}/labels/b")
    assert s.get(f"/api/v1/experiments/{eid}")["experiment"]["labels"] == ["a", "b"]
    s.delete(f"/api/v1/experiments/{eid}/labels/a")
    assert s.get("/api/v1/experiment/labels")["labels"] == ["b"]
    flt = {"filterGroup": {"kind": "group", "conjunction": "and", "children": [
        {"kind": "field", "columnName": "name", "operator": "contains", "value": "API-EXTRA"},
        {"kind": "field", "location": "LOCATION_TYPE_VALIDATIONS", "type": "COLUMN_TYPE_NUMBER",
         "columnName": "validation.val_loss.last", "operator": "notEmpty"}]}, "showArchived": False}
    res = s.get("/api/v1/experiments-search", params={"filter": json.dumps(flt), "sort": "id=desc"})["experiments"]
    assert res[0]["experiment"]["id"] == eid and res[0]["best_trial"] is not None
    flt["filterGroup"]["children"][0]["value"] = "no-such-name"
    assert s.get("/api/v1/experiments-search", params={"filter": json.dumps(flt)})["experiments"] == []
    with pytest.raises(Exception):  # malformed filter: 400, not an empty list
        s.get("/api/v1/experiments-search", params={"filter": '{"filterGroup": {"kind": "group"}}'})
    names = s.get("/api/v1/experiments/metrics-stream/metric-names", params={"ids": eid})
    assert "val_loss" in names["validation_metrics"] and "loss" in names["training_metrics"]
    assert s.get(f"/api/v1/experiments/{eid}/metrics-stream/batches",
                 params={"metric_type": "METRIC_TYPE_VALIDATION"})["batches"] == [2, 4]
    snap = s.get(f"/api/v1/experiments/{eid}/metrics-stream/trials-snapshot",
                 params={"metric_name": "val_loss", "metric_type": "METRIC_TYPE_VALIDATION", "batches_processed": 4})
    assert snap["trials"][0]["batches_processed"] == 4
    sample = s.get(f"/api/v1/experiments/{eid}/metrics-stream/trials-sample",
                   params={"metric_name": "loss", "metric_type": "METRIC_TYPE_TRAINING"})
    assert sample["trials"][0]["data"]


def test_trial_routes(env):
    m, s, eid, _ = env
    tid = s.get(f"/api/v1/experiments/{eid}/trials")["trials"][0]["id"]
    w = s.get(f"/api/v1/trials/{tid}/workloads")["workloads"]
    kinds = [next(iter(x)) for x in w]
    assert "training" in kinds and "validation" in kinds and "checkpoint" in kinds
    assert [x for x in s.get(f"/api/v1/trials/{tid}/workloads", params={"filter": "FILTER_OPTION_VALIDATION"})["workloads"]
            if "validation" not in x] == []
    s.post(f"/api/v1/trials/{tid}/validation_metrics",
           {"validation_metrics": {"steps_completed": 5, "avg_metrics": {"val_loss": 0.01}}})
    vm = s.get("/api/v1/trials/metrics/validation_metrics", params={"trial_ids": tid})["metrics"]
    assert vm[-1]["steps_completed"] == 5
    ts = s.get("/api/v1/trials/time-series", params={"trial_ids": tid, "metric_names": "val_loss"})["trials"][0]
    assert [p["steps_completed"] for p in ts["metrics"]["validation.val_loss"]][-1] == 5
    fields = s.get(f"/api/v1/trials/{tid}/logs/fields")
    assert "agent-0" in fields["agent_ids"]
    s.patch(f"/api/v1/trials/{tid}", {"tags": {"k": "v"}})
    ck = s.get(f"/api/v1/trials/{tid}/checkpoints")["checkpoints"][0]["uuid"]
    s.post("/api/v1/trial-source-info", {"trial_source_info": {"trial_id": tid, "checkpoint_uuid": ck}})
    assert s.get(f"/api/v1/checkpoints/{ck}/metrics")["metrics"]
    s.post(f"/api/v1/checkpoints/{ck}/metadata", {"checkpoint": {"metadata": {"note": "x"}}})
    assert s.get(f"/api/v1/checkpoints/{ck}")["checkpoint"]["metadata"]["note"] == "x"


def test_users_master_slots_jobs(env):
    m, s, eid, _ = env
    assert s.get("/api/v1/auth/user")["user"]["username"] == "admin"
    s.post("/api/v1/users/setting", {"settings": [{"key": "theme", "value": "dark"}]})
    assert s.get("/api/v1/users/setting")["settings"] == [{"key": "theme", "value": "dark", "store_path": ""}]
    s.post("/api/v1/users/setting/reset")
    assert s.get("/api/v1/users/setting")["settings"] == []
    assert s.get("/api/v1/users/determined/by-username")["user"]["username"] == "determined"
    assert s.get("/api/v1/users/1")["user"]["username"] == "admin"  # literal routes did not shadow {uid}
    assert s.get("/api/v1/master/telemetry")["enabled"] is False
    assert len(s.get("/api/v1/agents/agent-0/slots")["slots"]) == 2
    assert s.get("/api/v1/agents/agent-0/slots/1")["slot"]["id"] == "1"
    assert "results" in s.get("/api/v1/job-queues/stats")
    assert s.get("/api/v1/tasks/count") == {"commands": 0, "notebooks": 0, "shells": 0, "tensorboards": 0}
    raw = s.get("/api/v1/resources/allocation/raw")["resource_entries"]
    assert raw and raw[0]["slots"] == 1 and raw[0]["seconds"] > 0
    agg = s.get("/api/v1/resources/allocation/aggregated")["resource_entries"]
    assert agg[0]["seconds"] > 0 and "default" in agg[0]["by_resource_pool"]


def test_bulk_projects_workspaces_bindings(env):
    m, s, eid, body = env
    e2 = s.post("/api/v1/experiments", dict(body, activate=False))["experiment"]["id"]
    res = s.post("/api/v1/experiments/archive", {"experiment_ids": [eid, e2]})["results"]
    assert {r["id"]: bool(r["error"]) for r in res} == {eid: False, e2: True}  # e2 not terminal
    assert s.get(f"/api/v1/experiments/{eid}")["experiment"]["archived"] is True
    s.post("/api/v1/experiments/unarchive", {"filters": {"archived": True}})
    assert s.get(f"/api/v1/experiments/{eid}")["experiment"]["archived"] is False
    s.post("/api/v1/experiments/kill", {"experiment_ids": [e2]})
    ws = s.post("/api/v1/workspaces", {"name": "w2"})["workspace"]["id"]
    pid = s.post(f"/api/v1/workspaces/{ws}/projects", {"name": "p2"})["project"]["id"]
    assert s.post("/api/v1/experiments/move", {"experiment_ids": [eid], "destination_project_id": pid})["results"][0]["error"] == ""
    cols = {c["column"] for c in s.get(f"/api/v1/projects/{pid}/columns")["columns"]}
    assert "hp.lr" in cols and "validation_metrics.val_loss" in cols
    rng = s.get(f"/api/v1/projects/{pid}/experiments/metric-ranges")["ranges"]
    assert any(x["metrics_name"] == "validation_metrics.val_loss" for x in rng)
    s.put(f"/api/v1/projects/{pid}/notes", {"notes": [{"name": "n", "contents": "c"}]})
    s.post(f"/api/v1/projects/{pid}/archive")
    assert s.get(f"/api/v1/projects/{pid}")["project"]["archived"] is True
    s.post(f"/api/v1/projects/{pid}/move", {"destination_workspace_id": 1})
    s.post(f"/api/v1/workspaces/{ws}/archive")
    assert s.get(f"/api/v1/workspaces/{ws}")["workspace"]["archived"] is True
    s.post("/api/v1/resource-pools/default/workspace-bindings", {"workspace_ids": [ws]})
    assert s.get("/api/v1/resource-pools/default/workspace-bindings")["workspace_ids"] == [ws]
    assert s.get("/api/v1/workspaces/1/available-resource-pools")["resource_pool_names"] == []
    s.request("DELETE", "/api/v1/resource-pools/default/workspace-bindings", {"workspace_ids": [ws]})
    assert s.get("/api/v1/workspaces/1/available-resource-pools")["resource_pool_names"] == ["default"]
    res = s.request("DELETE", "/api/v1/experiments/delete", {"experiment_ids": [e2]})["results"]
    assert res[0]["error"] == ""
    with pytest.raises(APIException):
        s.get(f"/api/v1/experiments/{e2}")


def _det(m, *argv):
    import io
    from contextlib import redirect_stdout

    from determined_clone_amd.cli import cli

    buf = io.StringIO()
    with redirect_stdout(buf):
        rc = cli.main(["-m", m.master_url, "-u", "admin", *argv])
    assert rc in (0, None), buf.getvalue()
    return buf.getvalue()


def test_extra_cli_commands(env, tmp_path, monkeypatch):
    m, s, eid, _ = env
    monkeypatch.setenv("HOME", str(tmp_path))  # token cache
    out = _det(m, "resources", "raw")
    assert out.splitlines()[0].startswith("allocation_id,task_id,kind")
    assert "period_start" in _det(m, "res", "agg")
    assert len(_det(m, "dev", "auth-token").strip()) > 10
    assert '"cluster_id"' in _det(m, "dev", "curl", "/api/v1/master")
    assert "/api/v1/tasks/count" in _det(m, "dev", "bindings", "list")
    _det(m, "workspace", "create", "cliws")
    _det(m, "rp", "bindings", "add", "default", "cliws")
    assert "cliws" in _det(m, "rp", "bindings", "list-workspaces", "default")
    _det(m, "rp", "bindings", "replace", "default")
    assert "default" in _det(m, "workspace", "list-pools", "Uncategorized")
    _det(m, "project", "create", "cliws", "cp")
    assert "cp" in _det(m, "workspace", "list-projects", "cliws")
    _det(m, "project", "edit", "cliws", "cp", "--description", "d")
    assert "(none)" in _det(m, "project", "list-experiments", "cliws", "cp")
    cfgf = tmp_path / "tpl.yaml"
    cfgf.write_text("resources:\n  slots_per_trial: 1\n")
    _det(m, "template", "create", "t1", str(cfgf))
    _det(m, "template", "set-value", "t1", "resources.priority=7")
    assert "priority: 7" in _det(m, "template", "config", "t1")
    _det(m, "user", "create", "bob")
    _det(m, "user", "rename", "bob", "robert")
    _det(m, "user", "edit", "robert", "--display-name", "Rob")
    assert s.get("/api/v1/users/robert/by-username")["user"]["display_name"] == "Rob"
    tid = s.get(f"/api/v1/experiments/{eid}/trials")["trials"][0]["id"]
    bundle = _det(m, "trial", "support-bundle", str(tid), "-o", str(tmp_path)).strip()
    import tarfile

    with tarfile.open(bundle) as tf:
        assert {"trial.json", "metrics.json", "logs.txt"} <= set(tf.getnames())
    _det(m, "master", "config", "set", "--log-level", "info")
    assert "scheduler" in _det(m, "master", "config", "show")


def test_sdk_projects_workspaces_pools(env):
    from determined_clone_amd.experimental import client

    m, s, eid, _ = env
    d = client.Determined(session=s)
    ws = d.create_workspace("sdkws")
    p = ws.create_project("sdkp")
    p.set_description("desc")
    p.add_note("n1", "hello")
    assert p.list_notes()[-1]["name"] == "n1"
    p.archive()
    p.reload()
    assert p.archived and p.description == "desc"
    pool = d.get_resource_pool("default")
    pool.add_bindings(["sdkws"])
    assert pool.list_workspaces() == ["sdkws"]
    assert [x.name for x in ws.list_pools()] == ["default"]
    pool.replace_bindings([])
    assert [x.name for x in d.list_resource_pools()] == ["default"]
    p.move_to_workspace("Uncategorized")
    ws.archive()
