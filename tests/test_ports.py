"""Rendezvous port registry (reference: `master/internal/portregistry`): unique c10d ports per
multi-container allocation on its chief agent, carried to the launcher through the cluster info."""
import json

from determined_clone_amd import _info
from determined_clone_amd.agent import runtime
from determined_clone_amd.launch import torch_distributed as td
from determined_clone_amd.master.ports import PortRegistry


def test_registry_per_agent_reuse():
    r = PortRegistry(base=30000, span=3)
    assert r.acquire("a", "x") == 30000
    assert r.acquire("a", "x") == 30000  # idempotent per allocation
    assert r.acquire("a", "y") == 30001
    assert r.acquire("b", "z") == 30000  # other agent: independent
    r.release("x")
    assert r.acquire("a", "w") == 30000  # freed port reused
    assert r.in_use("a") == {30000, 30001}
    r.acquire("a", "v")
    try:
        r.acquire("a", "u")
        raise AssertionError("expected exhaustion")
    except RuntimeError as e:
        assert "no free rendezvous port" in str(e)


def _spec(rank, port):
    return {"allocation_id": "e.1.a", "task_id": "e.1", "kind": "TRIAL", "slots": [0],
            "container_rank": rank, "num_containers": 2, "rendezvous_port": port,
            "cluster_info": {"master_url": "http://m:8080", "cluster_id": "c", "agent_id": "",
                             "slot_ids": [], "task_id": "e.1", "allocation_id": "e.1.a",
                             "session_token": "t", "task_type": "TRIAL"},
            "environment": {}}


def test_port_reaches_the_launcher(tmp_path):
    devices = [{"id": 0, "uuid": "g0", "type": "rocm", "device_index": 0}]
    _, env = runtime.build_task(_spec(1, 29417), "http://m:8080", "agent-1", devices, str(tmp_path),
                                container_addrs=["10.0.0.1", "10.0.0.2"], base_env={})
    info = _info.ClusterInfo.from_dict(json.loads(env["DET_CLUSTER_INFO"]))
    assert info.rendezvous_port == 29417 and info.container_addrs == ["10.0.0.1", "10.0.0.2"]
    assert _info.ClusterInfo.from_dict(info.to_dict()).rendezvous_port == 29417
    cmd = td.create_launch_cmd(2, 1, info.container_rank, info.container_addrs[0],
                               info.rendezvous_port, [], ["python3", "train.py"])
    assert cmd[cmd.index("--master-port") + 1] == "29417"


def test_master_assigns_distinct_ports_on_shared_chief(tmp_path):
    from determined_clone_amd.master.core import Allocation, Master
    from determined_clone_amd.master.rm import AllocationRequest

    m = Master(str(tmp_path / "m.db"))
    started = []
    m.rm.start_containers = lambda req, specs: started.append(specs)
    for aid in ("c1", "c2"):
        m.allocations[aid] = Allocation(aid, aid, "COMMAND", spec={"kind": "COMMAND"})
        req = AllocationRequest(aid, aid, aid, 16)
        req.placements = [{"agent_id": "node-a", "slots": list(range(8))},
                          {"agent_id": "node-b", "slots": list(range(8))}]
        m._on_alloc_start(req)
    p1, p2 = (s[0]["rendezvous_port"] for s in started)
    assert p1 != p2 and all(s["rendezvous_port"] == p1 for s in started[0])
    m._allocation_done(m.allocations["c1"], 0, "done")
    assert p1 not in m.ports.in_use("node-a")


def test_shared_gpu_slots_split_the_cpu_thread_budget(tmp_path, monkeypatch):
    """--slots-per-gpu > 1: each single-slot trial gets its share of the agent's CPU threads
    (OMP_NUM_THREADS), unless the experiment's environment sets it."""
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    devices = [{"id": i, "uuid": f"g0-{i}", "type": "rocm", "device_index": 0} for i in range(8)]
    spec = dict(_spec(0, 29417), num_containers=1, slots=[3])
    _, env = runtime.build_task(spec, "http://m:8080", "agent-1", devices, str(tmp_path), base_env={})
    assert env["OMP_NUM_THREADS"] == "2"
    spec["environment"] = {"environment_variables": ["OMP_NUM_THREADS=5"]}
    _, env = runtime.build_task(spec, "http://m:8080", "agent-1", devices, str(tmp_path), base_env={})
    assert env["OMP_NUM_THREADS"] == "5"
    # one slot per GPU: unchanged (inherits the base environment)
    one = [{"id": 0, "uuid": "g0", "type": "rocm", "device_index": 0}]
    _, env = runtime.build_task(dict(spec, slots=[0], environment={}), "http://m:8080", "agent-1", one,
                                str(tmp_path), base_env={})
    assert "OMP_NUM_THREADS" not in env
