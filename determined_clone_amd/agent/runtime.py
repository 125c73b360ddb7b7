"""Task runtime shared by every place a task container runs: the agent (a process group per task),
a Kubernetes pod (``exec.task_runner`` as the pod's command) and a Slurm/PBS job step
(``exec.task_runner`` under ``srun`` / ``pbsdsh``).

Reference: the Go agent's container lifecycle (`agent/internal/container`) and the entrypoint
script the Kubernetes RM bakes into its pods (`master/internal/rm/kubernetesrm/spec.go`): fetch
the task's context directory, export the ``DET_*`` environment and the cluster-info document,
start ``exec.launch`` (trials) or the task's entrypoint (commands), and ship stdout/stderr lines to
the master's task-log API.
"""
import base64
import json
import logging
import os
import subprocess
import sys
import time
from typing import Any, Dict, List, Optional, Tuple

logger = logging.getLogger("determined_clone_amd.agent")

FRAMEWORK_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# sources the context directory's startup-hook.sh, then execs the task (reference entrypoint.sh)
ENTRYPOINT_SH = os.path.join(FRAMEWORK_ROOT, "determined_clone_amd", "exec", "entrypoint.sh")
STARTUP_HOOK = "startup-hook.sh"


def with_startup_hook(cmd: List[str], ctx_dir: str, entrypoint_sh: str = ENTRYPOINT_SH) -> List[str]:
    """``cmd`` run through the entrypoint wrapper when the context directory has a
    ``startup-hook.sh`` (for trials and every NTSC task, like the reference's entrypoints)."""
    if os.path.isfile(os.path.join(ctx_dir, STARTUP_HOOK)):
        return ["bash", entrypoint_sh] + list(cmd)
    return list(cmd)


def fetch_context(session: Any, task_id: str, ctx_dir: str) -> None:
    """Download and unpack the task's context directory (model definition) from the master."""
    os.makedirs(ctx_dir, exist_ok=True)
    try:
        blob = session.get(f"/api/v1/tasks/{task_id}/context").get("b64_tgz")
        if blob:
            from determined_clone_amd.util import untar_to

            untar_to(base64.b64decode(blob), ctx_dir)
    except Exception as e:
        logger.warning(f"could not fetch context for {task_id}: {e}")


def _user_env(spec: Dict[str, Any]) -> Dict[str, str]:
    user_env = (spec.get("environment") or {}).get("environment_variables") or {}
    if isinstance(user_env, list):
        user_env = dict(x.split("=", 1) for x in user_env if "=" in x)
    elif isinstance(user_env, dict) and ("rocm" in user_env or "cpu" in user_env or "cuda" in user_env):
        user_env = dict(x.split("=", 1) for x in (user_env.get("rocm") or user_env.get("cpu") or [])
                        if "=" in x)
    return {str(k): str(v) for k, v in user_env.items()}


def assigned_devices(spec: Dict[str, Any], devices: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    """The agent's devices given to this container (``spec["slots"]``; all when absent)."""
    slot_ids = spec.get("slots")
    return list(devices) if slot_ids is None else [d for d in devices if d["id"] in set(slot_ids)]


def build_task(spec: Dict[str, Any], master_url: str, agent_id: str,
               devices: List[Dict[str, Any]], ctx_dir: str,
               container_addrs: Optional[List[str]] = None,
               base_env: Optional[Dict[str, str]] = None) -> Tuple[List[str], Dict[str, str]]:
    """``(argv, env)`` of the process that runs one container of the task ``spec`` on ``devices``
    (the slots the container was given). ``container_addrs`` are the rendezvous addresses of a
    multi-container task, in container-rank order (default: all on this host)."""
    alloc = spec["allocation_id"]
    task_id = spec["task_id"]
    info = dict(spec["cluster_info"])
    info["agent_id"] = agent_id
    slot_ids = spec.get("slots")
    mine = devices if slot_ids is None else [d for d in devices if d["id"] in set(slot_ids)]
    info["slot_ids"] = [d["id"] for d in mine] if slot_ids is None else list(slot_ids)
    info["gpu_uuids"] = [d["uuid"] for d in mine if d["type"] == "rocm"]
    n = int(spec.get("num_containers", 1))
    if n > 1:
        info["rendezvous"] = {"container_addrs": list(container_addrs or ["127.0.0.1"] * n),
                              "container_rank": int(spec.get("container_rank", 0))}
        if spec.get("rendezvous_port"):
            info["rendezvous"]["port"] = int(spec["rendezvous_port"])
    env = dict(os.environ if base_env is None else base_env)
    env.update(_user_env(spec))
    env["DET_CLUSTER_INFO"] = json.dumps(info)
    env["DET_CONTEXT_DIR"] = ctx_dir
    env["DET_MASTER"] = master_url
    env["DET_AGENT_ID"] = agent_id
    env["DET_ALLOCATION_ID"] = alloc
    env["DET_TASK_ID"] = task_id
    if spec.get("proxy_secret"):
        env["DET_TASK_PROXY_SECRET"] = str(spec["proxy_secret"])
    env["PYTHONUNBUFFERED"] = "1"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PYTHONPATH"] = os.pathsep.join([ctx_dir, FRAMEWORK_ROOT] + ([env["PYTHONPATH"]] if env.get("PYTHONPATH") else []))
    if any(d["type"] == "rocm" for d in mine):
        phys = sorted({int(d.get("device_index", d["id"])) for d in mine})
        if spec["kind"] == "TRIAL" and len(mine) > 1 and len(phys) < len(mine):
            # RCCL needs one rank per device: a multi-slot trial must not land on two shares
            # of the same GPU.
            raise RuntimeError(f"task {task_id}: {len(mine)} slots map to only {len(phys)} "
                               "GPU(s); --slots-per-gpu > 1 supports single-slot trials only")
        env["HIP_VISIBLE_DEVICES"] = ",".join(str(i) for i in phys)
        if len(devices) > len({int(d.get("device_index", d["id"])) for d in devices}):
            # --slots-per-gpu > 1: many single-slot trials share this node's cores. Split the
            # agent's CPU-thread budget among the slots, or each trial process starts a full
            # OpenMP / torch intra-op pool (16 trials x 16 threads on a 16-core share).
            budget = int(os.environ.get("OMP_NUM_THREADS") or len(os.sched_getaffinity(0)))
            if "OMP_NUM_THREADS" not in _user_env(spec):
                env["OMP_NUM_THREADS"] = str(max(1, budget * len(mine) // len(devices)))
    else:
        env["DET_SLOTS"] = str(max(len(mine), 1))
        # CPU slots: give each task its share of the host's cores so concurrent trials do not
        # oversubscribe the CPU with one full-size OpenMP pool each.
        share = max(1, (os.cpu_count() or 1) * max(len(mine), 1) // max(len(devices), 1))
        env.setdefault("OMP_NUM_THREADS", str(share))
    if spec["kind"] == "TRIAL":
        cmd = [sys.executable, "-m", "determined_clone_amd.exec.launch"]
    else:
        cmd = list(spec.get("entrypoint") or ["true"])
        if cmd and cmd[0] in ("python", "python3"):
            cmd[0] = sys.executable
    return with_startup_hook(cmd, ctx_dir), env


def pump_logs(proc: subprocess.Popen, session: Any, spec: Dict[str, Any], agent_id: str) -> int:
    """Ship the process's output lines to the master (batched) until it exits; its exit code."""
    alloc = spec["allocation_id"]
    task_id = spec["task_id"]
    buf: List[Dict[str, Any]] = []
    last = time.time()

    def flush() -> None:
        nonlocal buf, last
        if buf:
            try:
                session.post("/api/v1/task/logs", {"logs": buf})
            except Exception as e:
                logger.warning(f"log shipping failed: {e}")
            buf = []
        last = time.time()

    for raw in iter(proc.stdout.readline, b""):
        line = raw.decode(errors="replace").rstrip("\n")
        rank = None
        if line.startswith("[rank"):
            try:
                rank = int(line[line.index("=") + 1: line.index("]")])
            except ValueError:
                rank = None
        buf.append({"task_id": task_id, "allocation_id": alloc, "agent_id": agent_id,
                    "log": line, "timestamp": time.time(), "rank_id": rank,
                    "container_id": str(spec.get("container_rank", 0))})
        if len(buf) >= 200 or time.time() - last > 1.0:
            flush()
    code = proc.wait()
    flush()
    return code


def encode_spec(spec: Dict[str, Any]) -> str:
    """Task spec as one environment-variable-safe string (``DET_TASK_SPEC``)."""
    return base64.b64encode(json.dumps(spec).encode()).decode()


def decode_spec(s: str) -> Dict[str, Any]:
    return json.loads(base64.b64decode(s.encode()).decode())
