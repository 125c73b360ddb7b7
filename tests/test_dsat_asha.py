"""DeepSpeed autotune, second half (reference: harness/determined/pytorch/dsat; tests in
harness/tests/experiment/... dsat and e2e_tests deepspeed autotune): the ASHA search over DeepSpeed
configurations, the model-profile memory model, the user-facing helpers (get_ds_config_from_hparams,
dsat_reporting_context), the native engine's autotuning hook, and both torchvision examples
(DeepSpeedTrial and Core API) searched on an in-process master + CPU agent."""
import json
import os
import pathlib
import shutil
import tempfile
import uuid

import pytest
import torch
import yaml

from determined_clone_amd.pytorch import dsat
from determined_clone_amd.pytorch.dsat import _defaults, _utils
from determined_clone_amd.pytorch.dsat import __main__ as dsat_main

ROOT = pathlib.Path(__file__).resolve().parents[1]
EXAMPLE = ROOT / "examples" / "deepspeed_autotune" / "torchvision"

# simulated hardware: micro batches above CAP[stage] run out of memory; throughput grows with the
# micro batch and saturates, stage 3 pays for its gathers, overlap_comm helps a little
CAP = {1: 40, 2: 60, 3: 90}


def _throughput(stage: int, mbs: int, zero_cfg: dict) -> float:
    base = {1: 1.0, 2: 0.97, 3: 0.8}[stage]
    bonus = 1.05 if zero_cfg.get("overlap_comm") else 1.0
    return base * bonus * 1000.0 * mbs / (mbs + 16.0)


def _drive(method, model_info, max_rounds=500):
    """Run a search method against the simulator until it shuts down; returns created hparams."""
    created = []
    pending = list(method.initial_operations(None))
    shutdown = False
    for _ in range(max_rounds):
        if not pending:
            break
        op = pending.pop(0)
        if op.kind == "Shutdown":
            shutdown = True
            continue
        if op.kind != "Create":
            continue
        hp = op.hparams
        created.append(hp)
        ow = hp[_defaults.OVERWRITE_KEY]
        rid = uuid.UUID(str(op.request_id))
        if (ow.get("autotuning") or {}).get("model_info"):
            pending += method.on_validation_completed(None, rid, dict(model_info), 1)
            continue
        stage = ow["zero_optimization"]["stage"]
        mbs = ow["train_micro_batch_size_per_gpu"]
        assert ow["autotuning"]["enabled"] and ow["autotuning"]["end_profile_step"] == 5
        if mbs > CAP[stage]:
            pending += method.on_trial_exited_early(None, rid, "INVALID_HP")
        else:
            res = {"throughput": _throughput(stage, mbs, ow["zero_optimization"]),
                   "latency": 1.0 / mbs}
            pending += method.on_validation_completed(None, rid, res, 5)
    return created, shutdown


def test_memory_model_bounds_micro_batch_per_stage():
    info = {"num_params": 10_000_000_000, "activation_mem_per_gpu": 2 * 2 ** 30,
            "gpu_mem": 288 * 2 ** 30}
    caps = _utils.approx_max_mbs_per_stage(info, [0, 1, 2, 3], dp=8, max_mbs=4096)
    # 16 B/param unpartitioned vs 16/8 B/param fully partitioned: more room as the stage grows
    assert caps[0] < caps[1] < caps[2] < caps[3]
    assert caps[3] == int((0.9 * 288 * 2 ** 30 - 10e9 * 2) // (2 * 2 ** 30))
    assert _utils.approx_max_mbs_per_stage({}, [1], 8, 64) == {1: 64}


def test_asha_search_profiles_promotes_and_finds_the_best():
    info = {"num_params": 100, "activation_mem_per_gpu": 100, "gpu_mem": 10_000,
            "trainable_num_params": 100}
    m = dsat.ASHADSATSearchMethod({"deepspeed_config": "ds_config.json"}, "throughput",
                                  zero_stages=(1, 2, 3), max_trials=40, max_concurrent_trials=1,
                                  max_mbs=128, seed=3, divisor=2, min_binary_search_trials=2,
                                  max_rungs=3)
    created, shutdown = _drive(m, info)
    assert shutdown
    # the model-profile trial first, then exactly max_trials - 1 profiling trials
    assert created[0][_defaults.OVERWRITE_KEY]["autotuning"]["model_info"]["profile"]
    assert len(created) == 40
    assert all(hp[_defaults.USE_DSAT_MODE_KEY] for hp in created)
    # the profile's numbers bound the binary searches ((9000 - 100 params * 16 B) / 100 B per sample)
    assert max(hp[_defaults.OVERWRITE_KEY]["train_micro_batch_size_per_gpu"] for hp in created[1:]) <= 74
    assert max(lin.rung for lin in m.lineages) >= 1  # successive halving promoted someone
    best = m.best()
    res = [r for r in m.results() if not r["oom"]]
    assert best["throughput"] == max(r["metric"] for r in res)
    assert best["train_micro_batch_size_per_gpu"] <= CAP[best["zero_stage"]]
    # the binary searches converge onto large micro batches (throughput grows with it)
    assert best["train_micro_batch_size_per_gpu"] >= 20
    assert any(r["oom"] for r in m.results())


def test_asha_state_round_trip(tmp_path):
    m = dsat.ASHADSATSearchMethod({}, "throughput", zero_stages=(1, 2), max_trials=6,
                                  max_concurrent_trials=2, max_mbs=32, seed=0)
    ops = m.initial_operations(None)
    rid = uuid.UUID(str(ops[0].request_id))
    m.on_validation_completed(None, rid, {"num_params": 10, "activation_mem_per_gpu": 1,
                                          "gpu_mem": 100}, 1)
    m.save_method_state(tmp_path)
    m2 = dsat.ASHADSATSearchMethod({}, "throughput", zero_stages=(1, 2), max_trials=6,
                                   max_concurrent_trials=2, max_mbs=32, seed=0)
    m2.load_method_state(tmp_path)
    assert [vars(a) == vars(b) for a, b in zip(m.lineages, m2.lineages)] and m2.created == m.created
    assert m2.stage_hi == m.stage_hi and m2.rng.random() == m.rng.random()


def test_profile_failure_falls_back_to_max_mbs():
    m = dsat.ASHADSATSearchMethod({}, "latency", zero_stages=(2,), max_trials=3,
                                  max_concurrent_trials=1, max_mbs=16, seed=0)
    ops = m.initial_operations(None)
    nxt = m.on_trial_exited_early(None, uuid.UUID(str(ops[0].request_id)), "ERRORED")
    creates = [o for o in nxt if o.kind == "Create"]
    assert creates and creates[0].hparams[_defaults.OVERWRITE_KEY]["train_micro_batch_size_per_gpu"] == 8


def test_random_search_early_stopping_and_test_method():
    m = dsat.DSATSearchMethod({}, "random", zero_stages=(1,), max_trials=50,
                              max_concurrent_trials=1, max_mbs=64, seed=1, early_stopping=3)
    created, shutdown = _drive_plain(m)
    assert shutdown and len(created) < 50
    t = dsat.DSATSearchMethod({}, "_test", zero_stages=(1, 2), max_trials=6, max_concurrent_trials=6)
    ops = t.initial_operations(None)
    mbs = [o.hparams[_defaults.OVERWRITE_KEY]["train_micro_batch_size_per_gpu"] for o in ops if o.kind == "Create"]
    assert mbs == [1, 2, 3, 4, 5, 6]


def _drive_plain(method):
    created, pending, shutdown = [], list(method.initial_operations(None)), False
    while pending:
        op = pending.pop(0)
        if op.kind == "Shutdown":
            shutdown = True
        if op.kind != "Create":
            continue
        created.append(op.hparams)
        ow = op.hparams[_defaults.OVERWRITE_KEY]
        mbs, stage = ow["train_micro_batch_size_per_gpu"], ow["zero_optimization"]["stage"]
        rid = uuid.UUID(str(op.request_id))
        if mbs > CAP[stage]:
            pending += method.on_trial_exited_early(None, rid, "INVALID_HP")
        else:
            pending += method.on_validation_completed(None, rid, {"throughput": float(mbs % 7)}, 5)
    return created, shutdown


def test_get_ds_config_from_hparams_merges_overwrites(tmp_path):
    (tmp_path / "ds.json").write_text(json.dumps({
        "train_batch_size": 256, "zero_optimization": {"stage": 1, "overlap_comm": True},
        "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}}))
    hp = {"deepspeed_config": "ds.json", "overwrite_deepspeed_args": {
        "zero_optimization": {"stage": 2}, "optimizer": {"params": {"lr": 5e-4}}}}
    cfg = dsat.get_ds_config_from_hparams(hp, tmp_path)
    assert cfg["zero_optimization"] == {"stage": 2, "overlap_comm": True}
    assert cfg["optimizer"] == {"type": "Adam", "params": {"lr": 5e-4}}
    with pytest.raises(KeyError):
        dsat.get_ds_config_from_hparams({}, tmp_path)
    assert dsat.get_batch_config_from_mbs_gas_and_slots(
        {"train_micro_batch_size_per_gpu": 8, "gradient_accumulation_steps": 2}, 4) == {
        "train_batch_size": 64, "train_micro_batch_size_per_gpu": 8, "gradient_accumulation_steps": 2}
    z = dsat.get_random_zero_optim_config(3)
    assert z["stage"] == 3 and {"reduce_bucket_size", "overlap_comm", "allgather_partitions"} <= set(z)


class _Rec:
    def __init__(self):
        self.val, self.done = [], []


def test_dsat_reporting_context_reports_engine_results(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    rec = _Rec()

    class Train:
        def report_validation_metrics(self, steps_completed, metrics):
            rec.val.append((steps_completed, metrics))

    class Op:
        length = 7

        def report_completed(self, m):
            rec.done.append(m)

    class Dist:
        rank = 0

    class Ctx:
        train, distributed = Train(), Dist()

    with pytest.raises(SystemExit):
        with dsat.dsat_reporting_context(Ctx(), Op()):
            (tmp_path / _defaults.AUTOTUNING_RESULTS_PATH).write_text(json.dumps({"throughput": 5.0}))
            raise SystemExit(0)
    assert rec.val == [(7, {"throughput": 5.0})] and rec.done == [{"throughput": 5.0}]


def test_engine_autotuning_hook_measures_and_exits(tmp_path, monkeypatch):
    from determined_clone_amd.pytorch import deepspeed as det_ds

    monkeypatch.chdir(tmp_path)
    cfg = {"train_micro_batch_size_per_gpu": 4, "optimizer": {"type": "Adam", "params": {"lr": 1e-3}},
           "autotuning": {"enabled": True, "start_profile_step": 2, "end_profile_step": 4}}
    eng, _, _, _ = det_ds.initialize(model=torch.nn.Linear(8, 2), config=cfg)
    steps = 0
    with pytest.raises(SystemExit):
        for steps in range(1, 100):
            eng.backward(eng(torch.randn(4, 8)).pow(2).mean())
            eng.step()
    assert steps == 4
    res = json.loads((tmp_path / _defaults.AUTOTUNING_RESULTS_PATH).read_text())
    assert res["throughput"] > 0 and res["latency"] > 0 and res["train_micro_batch_size_per_gpu"] == 4
    cfg["autotuning"] = {"enabled": True, "model_info": {"profile": True}}
    eng, _, _, _ = det_ds.initialize(model=torch.nn.Linear(8, 2), config=cfg)
    with pytest.raises(SystemExit):
        eng.backward(eng(torch.randn(4, 8)).pow(2).mean())
        eng.step()
    info = json.loads((tmp_path / _defaults.MODEL_INFO_PROFILING_PATH).read_text())
    assert info["num_params"] == 18 and info["gpu_mem"] > 0 and info["activation_mem_per_gpu"] >= 1
    # the stale results file of the earlier run was removed when this engine was built
    assert not (tmp_path / _defaults.AUTOTUNING_RESULTS_PATH).exists()


def test_full_experiment_config_merges_best():
    cfg = {"name": "x", "hyperparameters": {"deepspeed_config": "ds.json",
                                            "overwrite_deepspeed_args": {"train_batch_size": 64, "fp16": {"enabled": False}}},
           "searcher": {"name": "single", "max_length": 10}}
    out = dsat_main.full_experiment_config(cfg, {"zero_stage": 2, "train_micro_batch_size_per_gpu": 12,
                                                 "zero_optimization": {"stage": 2, "overlap_comm": True}})
    ow = out["hyperparameters"]["overwrite_deepspeed_args"]
    assert ow == {"fp16": {"enabled": False}, "train_micro_batch_size_per_gpu": 12,
                  "zero_optimization": {"stage": 2, "overlap_comm": True}}
    assert out["searcher"] == cfg["searcher"]


# ------------------------------------------------------------------------------ on a cluster
@pytest.fixture()
def cluster():
    from determined_clone_amd.agent import Agent
    from determined_clone_amd.common.api import Session
    from determined_clone_amd.master import Master, MasterServer

    tmp = tempfile.mkdtemp(prefix="det-dsat2-")
    m = Master(os.path.join(tmp, "m.db"), checkpoint_storage={"type": "shared_fs", "host_path": os.path.join(tmp, "ckpt")})
    srv = MasterServer(m, "127.0.0.1", 0).start()
    agent = Agent(m.master_url, "agent-0", artificial_slots=2).start_background()
    s = Session(m.master_url)
    s.token = s.post("/api/v1/auth/login", {"username": "admin", "password": ""})["token"]
    yield s, tmp
    agent.stop()
    srv.stop()
    shutil.rmtree(tmp, ignore_errors=True)


def _cpu_example(tmp: str, variant: str) -> tuple:
    """The example directory with the CPU-sized model (tiny ResNet, 64 px: BatchNorm needs more than one value per channel at micro batch 1; fp32, 1 slot)."""
    ctx = os.path.join(tmp, variant)
    shutil.copytree(EXAMPLE / variant, ctx)
    with open(os.path.join(ctx, "deepspeed.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["resources"]["slots_per_trial"] = 1
    cfg["searcher"]["max_length"] = 4
    cfg["hyperparameters"].update(model_name="resnet_tiny", image_size=64, num_classes=10,
                                  report_rate=2, checkpoint_rate=2)
    cfg["hyperparameters"]["overwrite_deepspeed_args"] = {"bf16": {"enabled": False}}
    cfg_path = os.path.join(tmp, f"{variant}.yaml")
    with open(cfg_path, "w") as f:
        yaml.safe_dump(cfg, f)
    return ctx, cfg_path


def _wait(s, eid, timeout=300):
    import time

    t0 = time.time()
    while time.time() - t0 < timeout:
        st = s.get(f"/api/v1/experiments/{eid}")["experiment"]["state"]
        if st in ("COMPLETED", "ERROR", "CANCELED"):
            return st
        time.sleep(1)
    return "TIMEOUT"


def test_asha_on_deepspeed_trial_example(cluster, capsys):
    s, tmp = cluster
    ctx, cfg_path = _cpu_example(tmp, "deepspeed_trial")
    rc = dsat_main.main(["asha", cfg_path, ctx, "-z", "1", "2", "-mt", "5", "-mct", "2",
                         "--start-profile-step", "1", "--end-profile-step", "2", "--max-mbs", "8",
                         "--min-binary-search-trials", "1", "--max-rungs", "2",
                         "--searcher-dir", os.path.join(tmp, "dsat_a"), "--run-full-experiment"],
                        session=s)
    assert rc == 0
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    if out["best"] is None:  # show why the profiling trials produced nothing
        for t in s.get(f"/api/v1/experiments/{out['experiment_id']}/trials")["trials"]:
            lines = [e["log"] for e in s.get(f"/api/v1/trials/{t['id']}/logs")["logs"]]
            first = next((i for i, ln in enumerate(lines) if "Traceback" in ln), 0)
            print(t["id"], t["state"], "\n".join(lines[first:first + 40]))
    assert out["best"] is not None and out["best"]["train_micro_batch_size_per_gpu"] >= 1
    assert len(out["trials"]) == 4  # + the model-profile trial = max_trials
    trials = s.get(f"/api/v1/experiments/{out['experiment_id']}/trials")["trials"]
    assert len(trials) == 5
    # the model-profile trial (micro batch 1) and every profiling trial ran to completion
    assert all(t["state"] == "COMPLETED" for t in trials), [t["state"] for t in trials]
    # the full-length experiment with the winning settings runs to completion
    assert _wait(s, out["full_experiment_id"]) == "COMPLETED"
    exp = s.get(f"/api/v1/experiments/{out['full_experiment_id']}")
    hp = exp["experiment"]["config"]["hyperparameters"]
    def plain(v):  # the master stores hyperparameters in expconf form ({"type": "const", "val"})
        if isinstance(v, dict):
            return plain(v["val"]) if v.get("type") == "const" and "val" in v else {k: plain(x) for k, x in v.items()}
        return v

    ow = plain(hp["overwrite_deepspeed_args"])
    assert ow["train_micro_batch_size_per_gpu"] == out["best"]["train_micro_batch_size_per_gpu"]
    assert ow["zero_optimization"]["stage"] == out["best"]["zero_stage"]


def test_binary_on_core_api_example(cluster, capsys):
    s, tmp = cluster
    ctx, cfg_path = _cpu_example(tmp, "core_api")
    rc = dsat_main.main(["binary", cfg_path, ctx, "-z", "1", "-mt", "3", "-mct", "2",
                         "--start-profile-step", "1", "--end-profile-step", "2", "--max-mbs", "4",
                         "--searcher-dir", os.path.join(tmp, "dsat_b")], session=s)
    assert rc == 0
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    # every trial reported the engine's measurements through dsat_reporting_context
    assert [t["mbs"] for t in out["trials"]] == [1, 2, 4] and all(t["metric"] for t in out["trials"])
    assert out["best"]["train_micro_batch_size_per_gpu"] in (1, 2, 4)


@pytest.mark.gpu
def test_engine_autotuning_hook_on_gpu(tmp_path, monkeypatch):
    """CUDA branch of the hook: activation bytes from the device allocator's peak, device memory
    from the MI355X's properties, bf16 ZeRO-2 engine."""
    from determined_clone_amd.models import resnet
    from determined_clone_amd.pytorch import deepspeed as det_ds

    monkeypatch.chdir(tmp_path)
    cfg = {"train_micro_batch_size_per_gpu": 8, "bf16": {"enabled": True},
           "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "zero_optimization": {"stage": 2},
           "autotuning": {"enabled": True, "model_info": {"profile": True}}}
    model = resnet.to_mi355x_layout(resnet.resnet18_bottleneck_tiny(num_classes=10))
    eng, _, _, _ = det_ds.initialize(model=model, config=cfg)
    x = torch.randn(8, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device="cuda")
    with pytest.raises(SystemExit):
        eng.backward(torch.nn.functional.cross_entropy(eng(x).float(), y))
        eng.step()
    info = json.loads((tmp_path / _defaults.MODEL_INFO_PROFILING_PATH).read_text())
    assert info["gpu_mem"] == torch.cuda.get_device_properties(0).total_memory
    assert info["activation_mem_per_gpu"] > 8 * 3 * 64 * 64 * 2  # at least the input images
    cfg["autotuning"] = {"enabled": True, "start_profile_step": 1, "end_profile_step": 3}
    eng, _, _, _ = det_ds.initialize(model=model, config=cfg)
    with pytest.raises(SystemExit):
        for _ in range(10):
            eng.backward(torch.nn.functional.cross_entropy(eng(x).float(), y))
            eng.step()
    res = json.loads((tmp_path / _defaults.AUTOTUNING_RESULTS_PATH).read_text())
    assert res["throughput"] > 0 and res["zero_stage"] == 2
