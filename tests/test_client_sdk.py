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


# every public name the reference's experimental/client.py re-exports (client.py:54-76) plus its
# module-level functions
REFERENCE_NAMES = [
    "Session", "OrderBy", "Checkpoint", "CheckpointOrderBy", "CheckpointSortBy", "CheckpointState",
    "DownloadMode", "Determined", "Experiment", "ExperimentOrderBy", "ExperimentSortBy",
    "ExperimentState", "TrainingMetrics", "TrialMetrics", "ValidationMetrics", "Model", "ModelOrderBy",
    "ModelSortBy", "Oauth2ScimClient", "Project", "Trial", "TrialOrderBy", "TrialSortBy", "TrialState",
    "User", "Workspace", "login", "create_experiment", "get_experiment", "list_experiments",
    "create_user", "get_user_by_id", "get_user_by_name", "get_session_username", "whoami", "logout",
    "list_users", "get_trial", "get_checkpoint", "get_workspace", "list_workspaces",
    "create_workspace", "delete_workspace", "create_model", "get_model", "get_model_by_id",
    "get_models", "list_models", "get_model_labels", "list_oauth_clients", "add_oauth_client",
    "remove_oauth_client", "stream_trials_metrics", "iter_trials_metrics",
    "stream_trials_training_metrics", "stream_trials_validation_metrics",
]


def test_reference_public_names_exist():
    missing = [n for n in REFERENCE_NAMES if not hasattr(client, n)]
    assert not missing, missing
    # enum values match the reference bindings' wire values
    assert client.OrderBy.ASC.value == "ORDER_BY_ASC" and client.OrderBy.DESCENDING.value == "ORDER_BY_DESC"
    assert client.ExperimentSortBy.SEARCHER_METRIC_VAL.value == "SORT_BY_SEARCHER_METRIC_VAL"
    assert client.TrialSortBy.BEST_VALIDATION_METRIC.value == "SORT_BY_BEST_VALIDATION_METRIC"
    assert client.ModelSortBy.NUM_VERSIONS.value == "SORT_BY_NUM_VERSIONS"
    assert client.CheckpointSortBy.BATCH_NUMBER.value == "SORT_BY_BATCH_NUMBER"
    assert client.DownloadMode("master") is client.DownloadMode.MASTER
    with pytest.warns(FutureWarning):
        assert client.TrialOrderBy.DESC.value == "ORDER_BY_DESC"


def test_sorted_lists_with_enums(det):
    """each sorted list accepts the reference's SortBy / OrderBy enums."""
    d, ctx, tmp, m = det
    cfg = yaml.safe_load(BASE)
    cfg["searcher"] = {"name": "grid", "metric": "val_loss", "max_length": {"batches": 4}}
    cfg["hyperparameters"]["lr"] = {"type": "categorical", "vals": [0.01, 0.1, 0.5]}
    exp = d.create_experiment(cfg, ctx)
    assert exp.wait(interval=0.5, timeout=240) == client.ExperimentState.COMPLETED
    exp.set_description("zzz")
    # trials
    ids = [t.id for t in exp.list_trials(sort_by=client.TrialSortBy.ID, order_by=client.OrderBy.DESC)]
    assert ids == sorted(ids, reverse=True) and len(ids) == 3
    best = exp.list_trials(sort_by=client.TrialSortBy.BEST_VALIDATION_METRIC, order_by=client.OrderBy.ASC)
    assert len(best) == 3
    for key in client.TrialSortBy:
        assert len(exp.list_trials(sort_by=key, order_by=client.OrderBy.ASC)) == 3
    # experiments
    d.create_experiment(dict(cfg, searcher={"name": "single", "metric": "val_loss",
                                            "max_length": {"batches": 4}}), ctx).wait(interval=0.5, timeout=240)
    eids = [e.id for e in d.list_experiments(sort_by=client.ExperimentSortBy.ID, order_by=client.OrderBy.DESC)]
    assert eids == sorted(eids, reverse=True) and len(eids) >= 2
    for key in client.ExperimentSortBy:
        assert len(d.list_experiments(sort_by=key, order_by=client.OrderBy.ASC)) == len(eids)
    by_trials = d.list_experiments(sort_by=client.ExperimentSortBy.NUM_TRIALS, order_by=client.OrderBy.DESC)
    assert by_trials[0].id == exp.id  # 3 trials beats 1
    # checkpoints
    cks = exp.list_checkpoints(sort_by=client.CheckpointSortBy.BATCH_NUMBER, order_by=client.OrderBy.ASC)
    steps = [c.steps_completed for c in cks]
    assert steps == sorted(steps) and cks
    for key in client.CheckpointSortBy:
        assert len(exp.list_checkpoints(sort_by=key, order_by=client.OrderBy.DESC)) == len(cks)
    met = exp.list_checkpoints(sort_by=client.CheckpointSortBy.SEARCHER_METRIC, order_by=client.OrderBy.ASC)
    vals = [c.validation_metrics["avg_metrics"]["val_loss"] for c in met if c.validation_metrics.get("avg_metrics")]
    assert vals == sorted(vals)
    t0 = exp.list_trials()[0]
    assert len(t0.list_checkpoints(sort_by=client.CheckpointSortBy.END_TIME, order_by=client.OrderBy.DESC)) >= 1
    # models
    d.create_model("m-b", description="second")
    d.create_model("m-a", description="first")
    names = [x.name for x in d.list_models(sort_by=client.ModelSortBy.NAME, order_by=client.OrderBy.DESC)]
    assert names == sorted(names, reverse=True)
    for key in client.ModelSortBy:
        assert len(d.list_models(sort_by=key, order_by=client.OrderBy.ASC)) == len(names)
    # model version reload / iter_metrics, tensorboard files
    mdl = d.get_model("m-a")
    v = mdl.register_version(exp.top_checkpoint().uuid)
    v.set_notes("hello")
    v.notes = None
    v.reload()
    assert v.notes == "hello"
    assert list(v.iter_metrics()) == []  # no task reported using this version
    exp.delete_tensorboard_files()
