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
