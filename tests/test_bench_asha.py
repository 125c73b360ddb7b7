"""ASHA trials/hr bench (tools/bench_asha.py) end to end on CPU slots, and the agent's GPU sharing."""
import json
import os
import subprocess
import sys

from determined_clone_amd.agent.agent import share_devices

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_share_devices_maps_slots_to_physical_gpus():
    devs = [{"id": 0, "uuid": "g0", "type": "rocm"}, {"id": 1, "uuid": "g1", "type": "rocm"}]
    slots = share_devices(devs, 2)
    assert [s["id"] for s in slots] == [0, 1, 2, 3]
    assert [s["device_index"] for s in slots] == [0, 0, 1, 1]
    assert len({s["uuid"] for s in slots}) == 4
    cpu = share_devices([{"id": 0, "uuid": "c", "type": "cpu"}], 4)
    assert len(cpu) == 1


def test_bench_asha_cpu_plumbing(tmp_path):
    out = subprocess.run(
        [sys.executable, os.path.join(ROOT, "tools", "bench_asha.py"), "--cpu", "--max-trials", "4",
         "--max-concurrent", "2", "--epochs", "2", "--records-per-epoch", "256", "--batch", "64",
         "--timeout", "300"],
        capture_output=True, text=True, timeout=420, cwd=str(tmp_path))
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["metric"] == "ASHA trials/hr"
    assert res["experiment_state"] == "COMPLETED"
    assert res["trials_completed"] == 4
    assert res["value"] > 0
    assert 0 < res["startup_share"] < 1 and res["startup_mean_s"] > 0
    assert res["allocations"] >= 4 and len(res["validation_error_quartiles"]) == 5


def test_detect_devices_max_gpus(monkeypatch):
    from determined_clone_amd.agent import agent as A

    phys = [{"id": i, "uuid": f"g{i}", "type": "rocm"} for i in range(8)]
    monkeypatch.setattr(A, "_detect_physical", lambda artificial_slots=0: [dict(d) for d in phys])
    devs = A.detect_devices(0, slots_per_gpu=4, max_gpus=2)
    assert len(devs) == 8 and {d["device_index"] for d in devs} == {0, 1}
    assert len(A.detect_devices(0, 1, 0)) == 8


def test_synthetic_cifar_is_learnable_but_noisy():
    import numpy as np

    from determined_clone_amd.models.cifar import SyntheticCIFAR10

    tr, va = SyntheticCIFAR10(2000, seed=0), SyntheticCIFAR10(500, seed=1, label_noise=0.0)
    assert tr.x.dtype == np.float16 and tr[0][0].shape == (3, 32, 32)
    # the batched fetch (DataLoader __getitems__ + cifar.collate) equals per-record fetching
    import torch

    from determined_clone_amd.models.cifar import collate

    bx, by = collate(tr.__getitems__([5, 0, 17]))
    rx, ry = torch.utils.data.default_collate([tr[5], tr[0], tr[17]])
    assert torch.equal(bx, rx) and torch.equal(by, ry)
    # nearest-class-mean on raw pixels is far from perfect (position jitter + low signal) ...
    means = np.stack([tr.x[tr.y == c].astype(np.float32).mean(0) for c in range(10)])
    pred = ((va.x.astype(np.float32)[:, None] - means[None]) ** 2).sum((2, 3, 4)).argmin(1)
    acc = (pred == va.y).mean()
    assert 0.15 < acc < 0.95, acc


def test_bench_asha_sixteen_trials_on_eight_fake_gpus(tmp_path):
    """BASELINE config "16 concurrent trials gang-scheduled across 8 MI355X" --
    the agent reports 8 ROCm devices with 2 slots each (trials run on the CPU here): 16 trials
    run at once, never more than 2 on one GPU, all 8 GPUs used."""
    out = subprocess.run(
        [sys.executable, os.path.join(ROOT, "tools", "bench_asha.py"), "--cpu", "--fake-gpus", "8",
         "--slots-per-gpu", "2", "--max-trials", "16", "--max-concurrent", "16", "--epochs", "1",
         "--records-per-epoch", "128", "--batch", "64", "--timeout", "600"],
        capture_output=True, text=True, timeout=900, cwd=str(tmp_path))
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["experiment_state"] == "COMPLETED" and res["trials_completed"] == 16
    assert res["n_gpus"] == 8 and res["config"]["slots_per_gpu"] == 2
    assert res["max_concurrent_trials"] == 16 and res["max_trials_per_gpu"] <= 2
    assert res["gpus_used"] == 8
