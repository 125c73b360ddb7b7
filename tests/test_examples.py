"""Run the shipped examples end to end on an in-process master + CPU agent (reference e2e_tests
run the tutorials the same way)."""
import base64
import os
import shutil
import tempfile
import time

import pytest
import yaml

from determined_clone_amd.agent import Agent
from determined_clone_amd.common.api import Session
from determined_clone_amd.master import Master, MasterServer
from determined_clone_amd.util import tar_directory

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")


@pytest.fixture(scope="module")
def cluster():
    tmp = tempfile.mkdtemp(prefix="det-ex-")
    m = Master(os.path.join(tmp, "m.db"), checkpoint_storage={"type": "shared_fs", "host_path": os.path.join(tmp, "ckpt")})
    srv = MasterServer(m, "127.0.0.1", 0).start()
    agent = Agent(m.master_url, "agent-0", artificial_slots=4).start_background()
    s = Session(m.master_url)
    s.token = s.post("/api/v1/auth/login", {"username": "admin", "password": ""})["token"]
    yield s
    agent.stop()
    srv.stop()
    shutil.rmtree(tmp, ignore_errors=True)


def _run(s, ctx_dir, cfg, timeout=300):
    body = {"config": cfg, "model_definition": base64.b64encode(tar_directory(ctx_dir)).decode()}
    eid = s.post("/api/v1/experiments", body)["experiment"]["id"]
    t0 = time.time()
    while time.time() - t0 < timeout:
        st = s.get(f"/api/v1/experiments/{eid}")["experiment"]["state"]
        if st in ("COMPLETED", "CANCELED", "ERROR"):
            return eid, st
        time.sleep(0.5)
    raise TimeoutError(st)


def test_mnist_tutorial_on_cluster(cluster):
    s = cluster
    cfg = yaml.safe_load(open(os.path.join(EX, "mnist_pytorch", "const.yaml")))
    cfg["searcher"]["max_length"] = {"batches": 30}
    cfg["min_validation_period"] = {"batches": 30}
    cfg.pop("records_per_epoch", None)
    eid, st = _run(s, os.path.join(EX, "mnist_pytorch"), cfg)
    assert st == "COMPLETED"
    t = s.get(f"/api/v1/experiments/{eid}/trials")["trials"][0]
    val = s.get(f"/api/v1/trials/{t['id']}/metrics", params={"group": "validation"})["metrics"]
    assert val[-1]["steps_completed"] == 30
    assert val[-1]["metrics"]["accuracy"] > 0.5  # synthetic MNIST is learnable


def test_core_api_hpsearch_on_cluster(cluster):
    s = cluster
    cfg = yaml.safe_load(open(os.path.join(EX, "core_api", "3_hpsearch.yaml")))
    cfg["searcher"]["max_length"] = 20
    cfg["searcher"]["max_trials"] = 4
    eid, st = _run(s, os.path.join(EX, "core_api"), cfg)
    assert st == "COMPLETED"
    trials = s.get(f"/api/v1/experiments/{eid}/trials")["trials"]
    assert len(trials) == 4 and all(t["state"] == "COMPLETED" for t in trials)


def _import_example(name, mod):
    import importlib.util
    import sys

    path = os.path.join(EX, name, mod + ".py")
    spec = importlib.util.spec_from_file_location(f"ex_{name}_{mod}", path)
    m = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = m
    spec.loader.exec_module(m)
    return m


def test_cifar_trial_local(tmp_path):
    from determined_clone_amd import pytorch
    from determined_clone_amd.common.storage import SharedFSStorageManager

    m = _import_example("cifar10_asha", "model_def")
    hp = {"global_batch_size": 16, "learning_rate": 0.01, "width": 16, "hidden": 64}
    with pytorch.init(hparams=hp, exp_conf={}) as ctx:
        ctx._core.checkpoint._storage_manager = SharedFSStorageManager(str(tmp_path))
        t = m.CIFARTrial(ctx)
        ctrl = pytorch.Trainer(t, ctx).fit(max_length=pytorch.Batch(3), checkpoint_policy="none",
                                           test_mode=True)
    assert ctrl.state.batches_trained >= 1


def test_gpt2_deepspeed_trial_local(tmp_path):
    from determined_clone_amd import pytorch
    from determined_clone_amd.common.storage import SharedFSStorageManager
    from determined_clone_amd.pytorch import deepspeed as det_ds

    m = _import_example("gpt2_deepspeed", "gpt2_trial")
    hp = {"model": "tiny", "seq_len": 32,
          "overwrite_deepspeed_args": {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": False},
                                       "scheduler": {"params": {"warmup_num_steps": 2, "total_num_steps": 10}}}}
    with det_ds.init(hparams=hp, exp_conf={}) as ctx:
        ctx._core.checkpoint._storage_manager = SharedFSStorageManager(str(tmp_path))
        t = m.GPT2Trial(ctx)
        c = det_ds.Trainer(t, ctx).fit(max_length=pytorch.Batch(3), checkpoint_policy="none")
    assert c.state.batches_trained == 3 and t.engine.global_steps == 3


def test_gpt2_pipeline_example_on_cluster(cluster):
    """The GPT-2 DeepSpeed example as a 2-stage pipeline over 2 slots: launch layer ->
    torch.distributed.run -> DeepSpeedTrial with a PipelineEngine (gloo on CPU slots)."""
    s = cluster
    cfg = yaml.safe_load(open(os.path.join(EX, "gpt2_deepspeed", "pipe.yaml")))
    cfg["hyperparameters"].update({"model": "tiny", "seq_len": 32, "pipe_parallel_size": 2})
    cfg["hyperparameters"]["overwrite_deepspeed_args"] = {
        "train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2,
        "bf16": {"enabled": False}, "zero_optimization": {"stage": 0},
        "scheduler": {"params": {"warmup_num_steps": 2, "total_num_steps": 10}}}
    cfg["resources"]["slots_per_trial"] = 2
    cfg["searcher"]["max_length"] = {"batches": 4}
    cfg["min_validation_period"] = {"batches": 4}
    eid, st = _run(s, os.path.join(EX, "gpt2_deepspeed"), cfg)
    t = s.get(f"/api/v1/experiments/{eid}/trials")["trials"][0]
    if st != "COMPLETED":
        logs = s.get(f"/api/v1/trials/{t['id']}/logs")["logs"]
        raise AssertionError("\n".join(l["log"] for l in logs[-60:]))
    val = s.get(f"/api/v1/trials/{t['id']}/metrics", params={"group": "validation"})["metrics"]
    assert val[-1]["steps_completed"] == 4 and val[-1]["metrics"]["lm_loss"] > 0
