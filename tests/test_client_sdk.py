"""Python client SDK against an in-process master + agent."""
import os
import shutil
import tempfile

import pytest
import yaml

from determined_clone_amd.agent import Agent
from determined_clone_amd.experimental import client
from determined_clone_amd.master import Master, MasterServer

from test_cluster_e2e import BASE, MODEL_DEF


@pytest.fixture(scope="module")
def det():
    tmp = tempfile.mkdtemp(prefix="det-sdk-")
    m = Master(os.path.join(tmp, "m.db"), checkpoint_storage={"type": "shared_fs", "host_path": os.path.join(tmp, "ckpt")})
    srv = MasterServer(m, "127.0.0.1", 0).start()
    agent = Agent(m.master_url, "agent-0", artificial_slots=2).start_background()
    ctx = os.path.join(tmp, "ctx")
    os.makedirs(ctx)
    with open(os.path.join(ctx, "model_def.py"), "w") as f:
        f.write(MODEL_DEF)
    d = client.Determined(m.master_url, "admin", "")
    yield d, ctx, tmp, m
    agent.stop()
    srv.stop()
    shutil.rmtree(tmp, ignore_errors=True)


def test_experiment_lifecycle_and_checkpoints(det, tmp_path):
    d, ctx, tmp, m = det
    cfg = yaml.safe_load(BASE)
    cfg["searcher"] = {"name": "grid", "metric": "val_loss", "max_length": {"batches": 8}}
    cfg["hyperparameters"]["lr"] = {"type": "categorical", "vals": [0.01, 0.1]}
    exp = d.create_experiment(cfg, ctx)
    assert exp.wait(interval=0.5, timeout=240) == client.ExperimentState.COMPLETED
    trials = exp.list_trials()
    assert len(trials) == 2
    t = d.get_trial(trials[0].id)
    assert t.hparams["lr"] in (0.01, 0.1)
    vals = list(t.stream_validation_metrics())
    assert [v.steps_completed for v in vals] == [4, 8] and "val_loss" in vals[-1].metrics
    assert any("validated" in line for line in t.logs())
    top = exp.top_checkpoint()
    assert top.validation_metrics["avg_metrics"]["val_loss"] == min(
        c.validation_metrics["avg_metrics"]["val_loss"] for c in exp.list_checkpoints()
        if c.validation_metrics.get("avg_metrics"))
    ck = d.get_checkpoint(top.uuid)
    ck.add_metadata({"tag": "best"})
    assert d.get_checkpoint(top.uuid).metadata["tag"] == "best"
    path = ck.download(str(tmp_path / "ck"))
    assert os.path.exists(os.path.join(path, "state_dict.pth"))
    assert t.select_checkpoint(latest=True).steps_completed == 8
    exp.set_name("renamed")
    exp.add_label("sdk")
    exp.reload()
    assert exp.name == "renamed" and "sdk" in exp.labels
    assert any(e.id == exp.id for e in d.list_experiments(labels=["sdk"]))
    code = exp.download_code(str(tmp_path / "code"))
    assert os.path.exists(os.path.join(code, "model_def.py"))


def test_models_users_workspaces(det):
    d, ctx, tmp, m = det
    assert d.whoami().username == "admin"
    u = d.create_user("alice", password="pw")
    assert d.get_user_by_name("alice").user_id == u.user_id
    ws = d.create_workspace("team")
    assert d.get_workspace("team").id == ws.id
    model = d.create_model("clf", description="demo", labels=["a"])
    assert d.get_model("clf").model_id == model.model_id
    cfg = yaml.safe_load(BASE)
    cfg["searcher"] = {"name": "single", "metric": "val_loss", "max_length": {"batches": 4}}
    exp = d.create_experiment(cfg, ctx)
    exp.wait(interval=0.5, timeout=240)
    v = model.register_version(exp.top_checkpoint().uuid)
    assert v.version == 1 and model.get_version().version == 1
    model.add_metadata({"k": 1})
    assert d.get_model("clf").metadata == {"k": 1}
    assert "a" in d.get_model_labels()
    assert [mm.name for mm in d.list_models()] == ["clf"]
