"""HPC launcher resource manager: trials and tasks run as Slurm or PBS batch jobs.

Reference: the "dispatcher" resource manager (`master/internal/rm/dispatcherrm`, driven through the
HPE launcher) and the expconf `slurm` / `pbs` sections (`schemas/expconf/v0/hpc-cluster-slurm.json`:
``slots_per_node``, ``gpu_type``, ``sbatch_args``; `hpc-cluster-pbs.json`: ``slots_per_node``,
``pbsbatch_args``). Here the workload manager is driven directly through its CLI:

* an allocation is handed to the workload manager as soon as it is requested -- Slurm/PBS own the
  queue, priorities and node placement (the reference defers to them the same way); the job has
  ``ceil(slots / slots_per_node)`` nodes, one container (one ``exec.task_runner`` process) per
  node, ``slots_per_node`` GPUs per node (``--gpus-per-node`` / ``--gres=gpu:<type>:<n>`` on
  Slurm, ``select=<nodes>:ngpus=<n>`` on PBS);
* the batch script exports the task spec (``DET_TASK_SPEC``) and starts one task runner per node
  (``srun --ntasks-per-node=1`` / ``pbsdsh -u``); each learns its container rank from
  ``SLURM_NODEID`` / ``PBS_NODENUM`` and the containers rendezvous through the master;
* job state is polled (``squeue`` + ``sacct`` / ``qstat -f -F json``): RUNNING -> containers
  RUNNING; finished -> TERMINATED with the job's exit code; kill = ``scancel`` / ``qdel``;
* resource pools are the Slurm partitions / PBS queues (``sinfo`` / ``qstat -Q``).
"""
import json
import logging
import os
import re
import shlex
import subprocess
import sys
import tempfile
import threading
import time
from typing import Any, Callable, Dict, List, Optional

from determined_clone_amd.agent.runtime import FRAMEWORK_ROOT, encode_spec
from determined_clone_amd.master.rm import AllocationRequest, ResourceManager

logger = logging.getLogger("determined_clone_amd.master.rm_dispatcher")

SLURM_DONE = {"COMPLETED", "FAILED", "CANCELLED", "TIMEOUT", "NODE_FAIL", "OUT_OF_MEMORY",
              "PREEMPTED", "BOOT_FAIL", "DEADLINE"}


def _export(k: str, v: str) -> str:
    # PYTHONPATH keeps the job's own value (shell expansion); everything else is quoted verbatim
    return f'export {k}="{v}"' if k == "PYTHONPATH" else f"export {k}={shlex.quote(v)}"


class _Job:
    __slots__ = ("alloc_id", "job_id", "n", "node_ids", "running", "done", "killed", "submitted")

    def __init__(self, alloc_id: str, job_id: str, n: int) -> None:
        self.alloc_id, self.job_id, self.n = alloc_id, job_id, n
        self.node_ids: List[str] = []
        self.running = self.done = self.killed = False
        self.submitted = time.time()


class DispatcherResourceManager(ResourceManager):
    def __init__(self, config: Dict[str, Any], scheduler: str = "priority", fit: str = "best",
                 preemption: bool = True,
                 on_start: Optional[Callable[[AllocationRequest], None]] = None,
                 on_preempt: Optional[Callable[[AllocationRequest], None]] = None,
                 start_watcher: bool = True) -> None:
        super().__init__(scheduler, fit, preemption, on_start, on_preempt)
        self.config = dict(config)
        self.kind = config.get("type", "slurm")
        if self.kind not in ("slurm", "pbs"):
            raise ValueError(f"dispatcher RM: unknown workload manager {self.kind!r}")
        self.slots_per_node = int(config.get("slots_per_node", 8))
        self.slot_type = config.get("slot_type", "rocm")
        self.gres_syntax = bool(config.get("gres_supported", False))
        self.python = config.get("python", sys.executable)
        self.job_dir = config.get("job_storage_root") or tempfile.mkdtemp(prefix="det-hpc-")
        os.makedirs(self.job_dir, exist_ok=True)
        self.poll_interval = float(config.get("poll_interval", 2.0))
        self.default_pool = config.get("default_compute_resource_pool")
        self.on_container_event: Optional[Callable[..., None]] = None
        self.jobs: Dict[str, _Job] = {}
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        if start_watcher:
            self._thread = threading.Thread(target=self._watch, daemon=True, name="hpc-rm")
            self._thread.start()

    # ------------------------------------------------------------------ CLI
    def _run(self, argv: List[str], input_text: Optional[str] = None) -> str:
        p = subprocess.run(argv, capture_output=True, text=True, input=input_text, timeout=60)
        if p.returncode != 0:
            raise RuntimeError(f"{' '.join(argv)}: exit {p.returncode}: {p.stderr.strip()[:300]}")
        return p.stdout

    # ------------------------------------------------------------------ requests
    def _per_node(self, req: AllocationRequest) -> int:
        hpc = (req.hpc or {}).get(self.kind) or {}
        return int(hpc.get("slots_per_node") or self.slots_per_node)

    def schedule(self) -> None:
        """Hand every pending request to the workload manager (it owns the queue)."""
        starts: List[AllocationRequest] = []
        with self._lock:
            for alloc_id in list(self.pending):
                req = self.pending.pop(alloc_id)
                per = max(1, self._per_node(req))
                n = max(1, -(-req.slots // per))
                left = req.slots
                req.placements = []
                for i in range(n):
                    k = min(per, left)
                    left -= k
                    req.placements.append({"agent_id": f"{self.kind}-node{i}", "slots": list(range(k))})
                req.start_time = time.time()
                self.running[alloc_id] = req
                starts.append(req)
        for r in starts:
            if self.on_start:
                self.on_start(r)

    def release(self, alloc_id: str) -> None:
        with self._lock:
            self.pending.pop(alloc_id, None)
            self.running.pop(alloc_id, None)

    # ------------------------------------------------------------------ batch scripts
    def batch_script(self, req: AllocationRequest, spec: Dict[str, Any], nodes: int) -> str:
        hpc = (req.hpc or {}).get(self.kind) or {}
        per = len(spec.get("slots") or [])
        alloc = spec["allocation_id"]
        name = re.sub(r"[^A-Za-z0-9_.-]", "_", f"det-{alloc}")[:60]
        out = os.path.join(self.job_dir, f"{name}.%j.out" if self.kind == "slurm" else f"{name}.out")
        pool = req.pool if req.pool and req.pool != "default" else self.default_pool
        lines = ["#!/bin/bash"]
        exports = {
            "DET_TASK_SPEC": encode_spec(spec),
            "DET_MASTER": spec["cluster_info"]["master_url"],
            "DET_SESSION_TOKEN": spec["cluster_info"].get("session_token", ""),
            "HSA_ENABLE_IPC_MODE_LEGACY": "0",
            "PYTHONPATH": os.pathsep.join([self.config.get("framework_root", FRAMEWORK_ROOT),
                                           "${PYTHONPATH:-}"]),
        }
        runner = f"{shlex.quote(self.python)} -m determined_clone_amd.exec.task_runner"
        if self.kind == "slurm":
            lines += [f"#SBATCH --job-name={name}", f"#SBATCH --nodes={nodes}",
                      "#SBATCH --ntasks-per-node=1", f"#SBATCH --output={out}"]
            if per and self.slot_type != "cpu":
                gpu_type = hpc.get("gpu_type")
                if self.gres_syntax:
                    lines.append(f"#SBATCH --gres=gpu:{gpu_type + ':' if gpu_type else ''}{per}")
                else:
                    lines.append(f"#SBATCH --gpus-per-node={gpu_type + ':' if gpu_type else ''}{per}")
            elif per:
                lines.append(f"#SBATCH --cpus-per-task={per}")
            if pool:
                lines.append(f"#SBATCH --partition={pool}")
            lines += [f"#SBATCH {a}" for a in (self.config.get("sbatch_args") or []) + (hpc.get("sbatch_args") or [])]
            lines += [_export(k, v) for k, v in exports.items()]
            lines.append(f"srun --kill-on-bad-exit=1 --ntasks-per-node=1 {runner}")
        else:
            sel = f"select={nodes}" + (f":ngpus={per}" if per and self.slot_type != "cpu" else
                                       (f":ncpus={per}" if per else ""))
            lines += [f"#PBS -N {name}", f"#PBS -l {sel}", "#PBS -j oe", f"#PBS -o {out}"]
            if pool:
                lines.append(f"#PBS -q {pool}")
            lines += [f"#PBS {a}" for a in (self.config.get("pbsbatch_args") or []) + (hpc.get("pbsbatch_args") or [])]
            lines += [_export(k, v) for k, v in exports.items()]
            env = " ".join(f"{k}={shlex.quote(v)}" for k, v in exports.items() if k != "PYTHONPATH")
            if nodes > 1:
                # pbsdsh does not forward the environment: pass it on the command line; each
                # task learns its rank from PBS_VNODENUM
                lines.append(f"pbsdsh -u -- /usr/bin/env {env} {runner}")
            else:
                lines.append(f"DET_CONTAINER_RANK=0 {runner}")
        return "\n".join(lines) + "\n"

    def start_containers(self, req: AllocationRequest, specs: List[Dict[str, Any]]) -> None:
        spec = dict(specs[0])
        spec["container_rank"] = 0
        script = self.batch_script(req, spec, len(specs))
        path = os.path.join(self.job_dir, re.sub(r"[^A-Za-z0-9_.-]", "_", f"det-{req.alloc_id}.sh"))
        with open(path, "w") as f:
            f.write(script)
        try:
            if self.kind == "slurm":
                out = self._run(["sbatch", "--parsable", path])
                job_id = out.strip().split(";")[0]
            else:
                job_id = self._run(["qsub", path]).strip()
        except Exception as e:
            logger.error(f"job submission for {req.alloc_id} failed: {e}")
            j = _Job(req.alloc_id, "", len(specs))
            j.node_ids = [s["agent_id"] for s in specs]
            self._finish(j, 1)
            return
        j = _Job(req.alloc_id, job_id, len(specs))
        j.node_ids = [s["agent_id"] for s in specs]
        with self._lock:
            self.jobs[req.alloc_id] = j
        logger.info(f"allocation {req.alloc_id}: {self.kind} job {job_id} ({len(specs)} node(s))")

    def kill_containers(self, alloc_id: str, placements: List[Dict[str, Any]]) -> None:
        j = self.jobs.get(alloc_id)
        if j is None or j.done:
            return
        j.killed = True
        try:
            self._run(["scancel", j.job_id] if self.kind == "slurm" else ["qdel", j.job_id])
        except Exception as e:
            logger.warning(f"could not cancel job {j.job_id}: {e}")

    # ------------------------------------------------------------------ job state
    def _slurm_states(self, ids: List[str]) -> Dict[str, Any]:
        states: Dict[str, Any] = {}
        out = self._run(["squeue", "-h", "-j", ",".join(ids), "-o", "%i|%T"]) if ids else ""
        for line in out.splitlines():
            if "|" in line:
                jid, st = line.strip().split("|", 1)
                states[jid] = (st.strip(), None)
        missing = [i for i in ids if i not in states]
        if missing:
            acct = self._run(["sacct", "-n", "-P", "-X", "-j", ",".join(missing), "-o", "JobID,State,ExitCode"])
            for line in acct.splitlines():
                parts = line.strip().split("|")
                if len(parts) >= 3:
                    st = parts[1].split()[0] if parts[1] else "UNKNOWN"
                    code, _, sig = parts[2].partition(":")
                    ec = int(code) if code.isdigit() else 1
                    if sig.isdigit() and int(sig) and not ec:
                        ec = 128 + int(sig)
                    states[parts[0]] = (st, ec)
        return states

    def _pbs_states(self, ids: List[str]) -> Dict[str, Any]:
        states: Dict[str, Any] = {}
        if not ids:
            return states
        out = self._run(["qstat", "-x", "-f", "-F", "json"] + ids)
        jobs = (json.loads(out or "{}").get("Jobs") or {})
        for jid, j in jobs.items():
            st = j.get("job_state", "")
            code = j.get("Exit_status")
            states[jid] = ({"Q": "PENDING", "H": "PENDING", "W": "PENDING", "R": "RUNNING",
                            "E": "RUNNING", "F": "COMPLETED", "X": "COMPLETED"}.get(st, st),
                           int(code) if code is not None else None)
        return states

    def _event(self, j: _Job, state: str, code: Optional[int] = None) -> None:
        if self.on_container_event is None:
            return
        for node in j.node_ids:
            try:
                self.on_container_event(node, j.alloc_id, state, code)
            except Exception:
                logger.exception(f"container event for job {j.job_id} failed")

    def _finish(self, j: _Job, code: int) -> None:
        if j.done:
            return
        j.done = True
        with self._lock:
            self.jobs.pop(j.alloc_id, None)
        if not j.running:
            j.running = True
            self._event(j, "RUNNING")
        self._event(j, "TERMINATED", 137 if j.killed and code == 0 else code)

    def sync_jobs(self) -> None:
        with self._lock:
            jobs = [j for j in self.jobs.values() if not j.done]
        if not jobs:
            return
        ids = [j.job_id for j in jobs]
        states = self._slurm_states(ids) if self.kind == "slurm" else self._pbs_states(ids)
        for j in jobs:
            st, code = states.get(j.job_id, (None, None))
            if st is None:
                continue
            if st in ("RUNNING", "COMPLETING") and not j.running:
                j.running = True
                self._event(j, "RUNNING")
            elif st in SLURM_DONE or (self.kind == "pbs" and st == "COMPLETED"):
                self._finish(j, code if code is not None else (0 if st == "COMPLETED" else 1))

    def _watch(self) -> None:
        err = None
        while not self._stop.is_set():
            try:
                self.sync_jobs()
                err = None
            except Exception as e:
                if str(e) != err:
                    logger.warning(f"{self.kind} job poll failed: {e}")
                err = str(e)
            self._stop.wait(self.poll_interval)

    def close(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)

    # ------------------------------------------------------------------ views
    def pools(self) -> List[Dict[str, Any]]:
        out = []
        try:
            if self.kind == "slurm":
                for line in self._run(["sinfo", "-h", "-o", "%R|%D|%G"]).splitlines():
                    part, nodes, gres = (line.split("|") + ["", "", ""])[:3]
                    m = re.search(r"gpu(?::[^:(]+)?:(\d+)", gres)
                    per = int(m.group(1)) if m else 0
                    out.append({"name": part.strip(), "num_agents": int(nodes or 0),
                                "slots_available": per * int(nodes or 0), "slots_used": 0,
                                "type": "RESOURCE_POOL_TYPE_STATIC", "scheduler_type": "slurm",
                                "slot_type": self.slot_type if per else "cpu"})
            else:
                for line in self._run(["qstat", "-Q"]).splitlines()[2:]:
                    if line.strip():
                        out.append({"name": line.split()[0], "num_agents": 0, "slots_available": 0,
                                    "slots_used": 0, "type": "RESOURCE_POOL_TYPE_STATIC",
                                    "scheduler_type": "pbs", "slot_type": self.slot_type})
        except Exception as e:
            logger.warning(f"could not list {self.kind} partitions: {e}")
        with self._lock:
            used = sum(r.slots for r in self.running.values())
        if out:
            out[0]["slots_used"] = used
        return out or [{"name": self.default_pool or "default", "num_agents": 0, "slots_available": 0,
                        "slots_used": used, "type": "RESOURCE_POOL_TYPE_STATIC",
                        "scheduler_type": self.kind, "slot_type": self.slot_type}]

    def queue(self) -> List[Dict[str, Any]]:
        rows = super().queue()
        for r in rows:
            j = self.jobs.get(r["allocation_id"])
            r["hpc_job_id"] = j.job_id if j else None
            if j is not None and not j.running:
                r["state"] = "QUEUED"
        return rows
