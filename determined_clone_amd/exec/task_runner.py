"""``python -m determined_clone_amd.exec.task_runner`` -- run ONE container of a task outside an
agent: the command of a Kubernetes pod (``master/rm_kubernetes.py``) and of a Slurm/PBS job step
(``master/rm_dispatcher.py``).

Reference: the entrypoint the Kubernetes RM writes into its pods
(`master/internal/rm/kubernetesrm/spec.go`: fetch context, export ``DET_*``, exec the task) and the
HPC launcher's per-node wrapper. Inputs come from the environment:

* ``DET_TASK_SPEC``  -- the task spec (base64 JSON, ``agent/runtime.encode_spec``);
* ``DET_MASTER``     -- master URL; ``DET_SESSION_TOKEN`` -- task session token;
* ``DET_CONTAINER_RANK`` (optional) -- overrides the spec's rank, for job steps that learn it from
  the launcher (``SLURM_NODEID`` / ``PBS_VNODENUM`` are read too);
* ``DET_CONTAINER_ADDR`` (optional) -- this container's address (a pod's ``status.podIP`` through
  the downward API); default: the host's primary address.

A multi-container task rendezvouses through the master's allocation all-gather: every container
posts ``(rank, address)`` and builds ``container_addrs`` in rank order, so ``exec.launch`` points
``torch.distributed.run`` at the chief's address. Devices are whatever the container sees (the
Kubernetes AMD GPU device plugin / Slurm GRES already restrict it). Exit code = the task's.
"""
import logging
import os
import socket
import subprocess
import sys
import tempfile
from typing import List

from determined_clone_amd.agent import agent as agent_mod
from determined_clone_amd.agent import runtime
from determined_clone_amd.common.api import Session
from determined_clone_amd.util import routable_address

logger = logging.getLogger("determined_clone_amd.exec.task_runner")


def _rank_from_env(default: int) -> int:
    for k in ("DET_CONTAINER_RANK", "SLURM_NODEID", "PBS_VNODENUM", "PBS_NODENUM"):
        v = os.environ.get(k)
        if v is not None and v.strip().isdigit():
            return int(v)
    return default


def rendezvous(session: Session, alloc_id: str, rank: int, n: int, addr: str) -> List[str]:
    """Container addresses in rank order, exchanged through the master (all containers block
    until all ``n`` have posted)."""
    got = session.post(f"/api/v1/allocations/{alloc_id}/all_gather",
                       {"request_uuid": "det-rendezvous", "num_peers": n,
                        "data": {"rank": rank, "addr": addr}}, timeout=660)["data"]
    by_rank = {int(d["rank"]): d["addr"] for d in got}
    if sorted(by_rank) != list(range(n)):
        raise RuntimeError(f"rendezvous of {alloc_id} incomplete: ranks {sorted(by_rank)} of {n}")
    return [by_rank[i] for i in range(n)]


def main() -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    spec = runtime.decode_spec(os.environ["DET_TASK_SPEC"])
    master = os.environ.get("DET_MASTER") or spec["cluster_info"]["master_url"]
    session = Session(master, token=os.environ.get("DET_SESSION_TOKEN")
                      or spec["cluster_info"].get("session_token"))
    spec["container_rank"] = _rank_from_env(int(spec.get("container_rank", 0)))
    spec.pop("slots", None)  # the container owns every device it can see
    n = int(spec.get("num_containers", 1))
    addrs = None
    if n > 1:
        addrs = rendezvous(session, spec["allocation_id"], spec["container_rank"], n, routable_address())
    agent_id = os.environ.get("DET_AGENT_ID") or socket.gethostname()
    devices = agent_mod.detect_devices()
    wd = tempfile.mkdtemp(prefix="det-task-")
    ctx_dir = os.path.join(wd, "context")
    runtime.fetch_context(session, spec["task_id"], ctx_dir)
    cmd, env = runtime.build_task(spec, master, agent_id, devices, ctx_dir, container_addrs=addrs)
    proc = subprocess.Popen(cmd, cwd=ctx_dir, env=env, stdout=subprocess.PIPE,
                            stderr=subprocess.STDOUT)
    return runtime.pump_logs(proc, session, spec, agent_id)


if __name__ == "__main__":
    sys.exit(main())
