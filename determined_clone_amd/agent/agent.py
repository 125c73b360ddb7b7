"""Agent: reports this host's MI355X slots to the master and runs tasks on them.

Reference: `agent/internal` (Go; Docker container runtime, rocm-smi/nvidia-smi detection).
Here a task is a process group (no Docker in this image): the agent fetches the task's context
directory from the master, sets ``HIP_VISIBLE_DEVICES`` to the assigned slots, ``DET_*`` env and
the cluster-info document, starts ``exec.launch``, ships stdout/stderr lines to the master, and
reports RUNNING / TERMINATED(exit code). Kill = SIGTERM to the process group, SIGKILL after a
grace period.

Devices: KFD topology via the native module (`native/scheduler.cpp: detect_kfd_gpus`), falling
back to ``rocm-smi --json``; CPU-only hosts expose ``--artificial-slots`` CPU slots.

GPU sharing (``--slots-per-gpu K``, MI355X-specific): one MI355X has 256 CUs and 288 GB of HBM3E, far
more than a small HP-search trial (e.g. the CIFAR-10 CNN of the adaptive_asha config) can use, so
the agent may expose each physical GPU as K schedulable slots. Trials placed on slots of the same
GPU run as separate processes on separate HIP queues of that device (time-sliced / co-resident
waves), which is how 16 concurrent ASHA trials fit on 8 GPUs. Slot ``i`` maps to physical device
``i // K``; ``HIP_VISIBLE_DEVICES`` lists the distinct physical devices of the task's slots.
"""
import argparse
import json
import logging
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time
from typing import Any, Dict, List, Optional

from determined_clone_amd.agent import runtime
from determined_clone_amd.common.api import Session

logger = logging.getLogger("determined_clone_amd.agent")


def share_devices(devs: List[Dict[str, Any]], slots_per_gpu: int) -> List[Dict[str, Any]]:
    """Expose each ROCm device as ``slots_per_gpu`` slots (see module docstring)."""
    out: List[Dict[str, Any]] = []
    for d in devs:
        d = dict(d, device_index=d["id"])
        k = slots_per_gpu if d["type"] == "rocm" else 1
        for j in range(max(1, k)):
            out.append(dict(d, id=len(out), uuid=d["uuid"] if k <= 1 else f"{d['uuid']}/{j}",
                            share=j, shares=k))
    return out


def pci_address(domain: Any, location_id: Any) -> Optional[str]:
    """KFD topology ``domain`` + ``location_id`` (bus << 8 | device << 3 | function) ->
    ``dddd:bb:dd.f``, the form of ``/dev/dri/by-path/pci-<address>-{card,render}``."""
    try:
        loc = int(location_id)
        dom = int(domain or 0)
    except (TypeError, ValueError):
        return None
    return f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7:x}"


def detect_devices(artificial_slots: int = 0, slots_per_gpu: int = 1,
                   max_gpus: int = 0) -> List[Dict[str, Any]]:
    devs = _detect_physical(artificial_slots)
    if max_gpus > 0:  # the first N ROCm devices (e.g. a 1/2/4/8-GPU run on one node)
        gpus = [d for d in devs if d["type"] == "rocm"][:max_gpus]
        devs = gpus or devs
    return share_devices(devs, slots_per_gpu) if slots_per_gpu > 1 else devs


def _detect_physical(artificial_slots: int = 0) -> List[Dict[str, Any]]:
    if artificial_slots > 0:
        return [{"id": i, "uuid": f"cpu-{i}", "type": "cpu", "brand": "artificial"} for i in range(artificial_slots)]
    devs: List[Dict[str, Any]] = []
    try:
        from determined_clone_amd.native import load

        for g in load().detect_kfd_gpus(""):
            devs.append({"id": int(g["index"]), "uuid": g.get("unique_id") or g["index"],
                         "type": "rocm", "brand": "AMD", "gfx_target": g.get("gfx_target"),
                         "cu_count": int(g.get("cu_count") or 0),
                         "vram_bytes": int(g.get("vram_bytes") or 0),
                         # PCI address + DRM render minor: which /dev/dri nodes a container of
                         # this slot gets (agent/containers.py rocm_device_paths)
                         "pci_bus": pci_address(g.get("domain"), g.get("location_id")),
                         "render_minor": int(g["drm_render_minor"]) if g.get("drm_render_minor") else None})
    except Exception as e:  # pragma: no cover - no native module / no KFD
        logger.debug(f"KFD detection failed: {e}")
    if not devs and shutil.which("rocm-smi"):
        try:
            out = subprocess.run(["rocm-smi", "--showuniqueid", "--showbus", "--json"],
                                 capture_output=True, text=True, timeout=30).stdout
            for k, v in sorted(json.loads(out).items()):
                if k.startswith("card"):
                    devs.append({"id": int(k[4:]), "uuid": v.get("Unique ID", k), "type": "rocm",
                                 "brand": "AMD"})
        except Exception:  # pragma: no cover
            pass
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis and devs:
        keep = {int(x) for x in vis.split(",") if x.strip().isdigit()}
        devs = [d for d in devs if d["id"] in keep]
    if not devs:
        devs = [{"id": 0, "uuid": "cpu-0", "type": "cpu", "brand": "cpu"}]
    return devs


class _Task:
    def __init__(self, spec: Dict[str, Any], proc: subprocess.Popen, workdir: str) -> None:
        self.spec = spec
        self.proc = proc
        self.workdir = workdir
        self.killed = False


def _names_image(spec: Dict[str, Any]) -> bool:
    """True when the task's experiment config chose a container image (``environment.image``)."""
    c = spec.get("container") or {}
    img = c.get("image")
    return bool(img if not isinstance(img, dict) else any(img.values()))


class Agent:
    def __init__(self, master_url: str, agent_id: Optional[str] = None, pool: str = "default",
                 artificial_slots: int = 0, label: str = "", username: str = "admin",
                 password: str = "", workdir: Optional[str] = None, slots_per_gpu: int = 1,
                 max_gpus: int = 0, container_runtime: str = "process",
                 container_socket: Optional[str] = None, dev_root: str = "/dev") -> None:
        self.session = Session(master_url)
        tok = self.session.post("/api/v1/auth/login", {"username": username, "password": password})["token"]
        self.session.token = tok
        self.master_url = self.session.master
        self.id = agent_id or socket.gethostname()
        self.pool = pool
        self.label = label
        self.devices = detect_devices(artificial_slots, slots_per_gpu, max_gpus)
        self.tasks: Dict[str, _Task] = {}
        self.workdir = workdir or tempfile.mkdtemp(prefix="det-clone-agent-")
        os.makedirs(self.workdir, exist_ok=True)  # the zygote binds its socket here right away
        self._stop = threading.Event()
        self._lock = threading.Lock()
        # container runtime (agent/containers.py): Docker / Podman / Apptainer, or None = tasks
        # run as process groups (also the fallback of "auto" when no daemon answers)
        from determined_clone_amd.agent import containers

        self.containers = containers.make_runtime(container_runtime, self.id, container_socket, dev_root)
        # "auto": containers only for tasks whose config names an image (environment.image);
        # tasks without one keep the process runtime (zygote, per-agent MIOpen DB), so an agent
        # on a host where a daemon answers does not move every task into a default image it may
        # not be able to pull
        self.container_auto = (container_runtime or "auto").lower() == "auto"
        # allocations whose container is being created (pull / create / start on a worker thread)
        # -> killed-while-launching flag
        self._launching: Dict[str, threading.Event] = {}
        # pre-warmed fork server for task processes (exec/zygote.py), started in the background
        self.zygote = None
        self._zygote_done = threading.Event()
        threading.Thread(target=self._start_zygote, daemon=True).start()

    def _start_zygote(self) -> None:
        from determined_clone_amd.exec.zygote import ZygoteClient

        try:
            self.zygote = ZygoteClient.start(self.workdir)
        except Exception as e:  # plain subprocesses still work
            logger.warning(f"zygote unavailable: {e}")
        finally:
            self._zygote_done.set()

    def register(self) -> None:
        self.session.post("/api/v1/agents/register", {
            "agent_id": self.id, "slots": self.devices, "resource_pool": self.pool,
            "label": self.label, "addresses": ["127.0.0.1"]})

    # ------------------------------------------------------------------ task lifecycle
    def _start(self, spec: Dict[str, Any]) -> None:
        alloc = spec["allocation_id"]
        wd = os.path.join(self.workdir, alloc.replace("/", "_"))
        ctx_dir = os.path.join(wd, "context")
        runtime.fetch_context(self.session, spec["task_id"], ctx_dir)
        if self.containers is not None and (not self.container_auto or _names_image(spec)):
            # off the action loop: an image pull can take minutes and must not stall kills, other
            # starts or the master long-poll (reference: the agent pulls asynchronously)
            killed = threading.Event()
            with self._lock:
                self._launching[spec["allocation_id"]] = killed
            threading.Thread(target=self._start_container, args=(spec, wd, ctx_dir, killed),
                             daemon=True, name=f"launch-{spec['allocation_id']}").start()
            return
        cmd, env = runtime.build_task(spec, self.master_url, self.id, self.devices, ctx_dir)
        if "MIOPEN_USER_DB_PATH" not in env:
            # one writable MIOpen find DB + kernel cache per agent, seeded from the shipped MI355X
            # files: what one trial compiles or finds, every later trial of the agent reuses
            from determined_clone_amd.ops import miopen_db

            db, cache = miopen_db.task_dirs(self.workdir)
            miopen_db.configure(env, db, cache)
        proc = None
        # a task that arrives while the zygote is still importing waits for it: a cold
        # subprocess would pay the same imports (and compete with the zygote for the CPU)
        self._zygote_done.wait(timeout=60)
        why = None
        if self.zygote is not None:
            from determined_clone_amd.exec.zygote import incompatible_reason

            why = incompatible_reason(env, skip_paths=[runtime.FRAMEWORK_ROOT])
            if why:
                logger.info(f"task {spec['task_id']}: plain subprocess, not the zygote ({why})")
        if self.zygote is not None and not why and len(cmd) >= 3 and cmd[0] == sys.executable and cmd[1] == "-m":
            try:
                proc = self.zygote.spawn(cmd[2], cmd[3:], env, ctx_dir)
            except Exception as e:
                logger.warning(f"zygote spawn failed ({e}); starting {cmd[2]} as a subprocess")
        if proc is None:
            env["DET_SPAWN_TIME"] = repr(time.time())
            proc = subprocess.Popen(cmd, cwd=ctx_dir, env=env, stdout=subprocess.PIPE,
                                    stderr=subprocess.STDOUT, start_new_session=True)
        t = _Task(spec, proc, wd)
        with self._lock:
            self.tasks[alloc] = t
        self._event(alloc, "RUNNING")
        threading.Thread(target=self._pump, args=(t,), daemon=True).start()

    def _start_container(self, spec: Dict[str, Any], wd: str, ctx_dir: str,
                         killed: Optional[threading.Event] = None) -> None:
        """Run the task in a container (agent/containers.py): same command and DET_* environment
        as the process runtime, seen through the container's mounts and device mapping. Runs on a
        worker thread per allocation; a failure (pull, create, start) is reported as TERMINATED 1
        and a kill that arrived meanwhile stops the container as soon as it exists."""
        alloc = spec["allocation_id"]
        try:
            base = {k: v for k, v in os.environ.items() if k.startswith("DET_MASTER_CERT")}
            cmd, env = runtime.build_task(spec, self.master_url, self.id, self.devices, ctx_dir, base_env=base)
            if "MIOPEN_USER_DB_PATH" not in env:
                # the agent's MIOpen find DB + kernel cache, bind-mounted at the same path, so
                # containerised trials reuse what earlier trials found / compiled
                from determined_clone_amd.ops import miopen_db

                db, cache = miopen_db.task_dirs(self.workdir)
                miopen_db.configure(env, db, cache)
                spec = dict(spec)
                c = dict(spec.get("container") or {})
                c["bind_mounts"] = list(c.get("bind_mounts") or []) + [
                    {"host_path": os.path.dirname(db), "container_path": os.path.dirname(db),
                     "read_only": False}]
                spec["container"] = c
            mine = runtime.assigned_devices(spec, self.devices)
            if killed is not None and killed.is_set():
                raise RuntimeError("killed before its container started")
            proc = self.containers.launch(spec, cmd, env, ctx_dir, mine, runtime.FRAMEWORK_ROOT)
        except Exception as e:
            logger.warning(f"container launch of {alloc} failed: {e}")
            with self._lock:
                self._launching.pop(alloc, None)
            self._event(alloc, "TERMINATED", 137 if killed is not None and killed.is_set() else 1)
            shutil.rmtree(wd, ignore_errors=True)
            return
        t = _Task(spec, proc, wd)
        with self._lock:
            self.tasks[alloc] = t
            self._launching.pop(alloc, None)
        self._event(alloc, "RUNNING")
        threading.Thread(target=self._pump, args=(t,), daemon=True).start()
        if killed is not None and killed.is_set():  # kill arrived during the pull / create
            self._kill(alloc)

    def _reattach(self) -> None:
        """After an agent restart: follow this agent's containers that are still running and
        report the exit of those that ended while no agent watched them (reference
        docker.go ReattachContainer)."""
        if self.containers is None:
            return
        for labels, proc, code in self.containers.reattach():
            from determined_clone_amd.agent import containers

            alloc = labels.get(containers.LABEL_ALLOC)
            if not alloc or alloc in self.tasks:
                continue
            if code is not None:
                logger.info(f"container of {alloc} exited ({code}) while the agent was down")
                self._event(alloc, "TERMINATED", code)
                proc.remove()
                continue
            logger.info(f"re-attached to the running container of {alloc}")
            spec = {"allocation_id": alloc, "task_id": labels.get(containers.LABEL_TASK, alloc)}
            t = _Task(spec, proc, os.path.join(self.workdir, alloc.replace("/", "_")))
            with self._lock:
                self.tasks[alloc] = t
            self._event(alloc, "RUNNING")
            threading.Thread(target=self._pump, args=(t,), daemon=True).start()

    def _pump(self, t: _Task) -> None:
        alloc = t.spec["allocation_id"]
        code = runtime.pump_logs(t.proc, self.session, t.spec, self.id)
        with self._lock:
            self.tasks.pop(alloc, None)
        self._event(alloc, "TERMINATED", code if not t.killed else (code or 137))
        remove = getattr(t.proc, "remove", None)
        if remove is not None:  # container: delete it once its exit is reported
            try:
                remove()
            except Exception as e:
                logger.warning(f"removing the container of {alloc}: {e}")
        shutil.rmtree(t.workdir, ignore_errors=True)

    def _signal(self, t: _Task, sig: int) -> bool:
        """SIGTERM / SIGKILL the task: its process group, or its container."""
        from determined_clone_amd.agent import containers

        if isinstance(t.proc, containers.ContainerProcess):  # Docker / Podman: via the daemon
            try:
                t.proc.send_signal(signal.Signals(sig).name)
            except Exception as e:
                logger.warning(f"signalling container: {e}")
                return False
            return True
        try:
            os.killpg(t.proc.pid, sig)
        except ProcessLookupError:
            return False
        return True

    def _kill(self, alloc: str, grace: float = 10.0) -> None:
        with self._lock:
            t = self.tasks.get(alloc)
            launching = self._launching.get(alloc)
        if t is None:
            if launching is not None:
                launching.set()  # _start_container stops it once it exists
            return
        t.killed = True
        if not self._signal(t, signal.SIGTERM):
            return

        def hard() -> None:
            time.sleep(grace)
            if t.proc.poll() is None:
                self._signal(t, signal.SIGKILL)

        threading.Thread(target=hard, daemon=True).start()

    def _event(self, alloc: str, state: str, exit_code: Optional[int] = None) -> None:
        try:
            self.session.post(f"/api/v1/agents/{self.id}/events",
                              {"allocation_id": alloc, "state": state, "exit_code": exit_code})
        except Exception as e:
            logger.warning(f"event report failed: {e}")

    # ------------------------------------------------------------------ main loop
    def run(self) -> None:
        self.register()
        self._reattach()
        while not self._stop.is_set():
            try:
                acts = self.session.get(f"/api/v1/agents/{self.id}/actions",
                                        params={"timeout_seconds": 5}, timeout=30)["actions"]
            except Exception as e:
                logger.warning(f"master unreachable: {e}; re-registering")
                time.sleep(1)
                try:
                    self.register()
                except Exception:
                    pass
                continue
            for a in acts:
                try:
                    if a["type"] == "start":
                        self._start(a["spec"])
                    elif a["type"] == "kill":
                        self._kill(a["allocation_id"])
                except Exception:
                    logger.exception(f"failed to handle action {a.get('type')}")
                    if a.get("type") == "start":
                        self._event(a["spec"]["allocation_id"], "TERMINATED", 1)

    def start_background(self) -> "Agent":
        self.register()
        self._reattach()
        threading.Thread(target=self.run, daemon=True, name=f"agent-{self.id}").start()
        return self

    def stop(self) -> None:
        self._stop.set()
        for alloc in list(self.tasks):
            self._kill(alloc, grace=2.0)
        if self.zygote is not None:
            self.zygote.close()


def main() -> None:
    ap = argparse.ArgumentParser("det-clone-agent")
    ap.add_argument("--master-url", default=os.environ.get("DET_MASTER", "http://127.0.0.1:8080"))
    ap.add_argument("--agent-id", default=None)
    ap.add_argument("--resource-pool", default="default")
    ap.add_argument("--artificial-slots", type=int, default=0)
    ap.add_argument("--label", default="")
    ap.add_argument("--slots-per-gpu", type=int, default=1,
                    help="expose each MI355X as this many slots (HP-search trials sharing a GPU)")
    ap.add_argument("--max-gpus", type=int, default=0, help="use only the first N GPUs (0 = all)")
    ap.add_argument("--container-runtime", default="process",
                    choices=["auto", "docker", "podman", "apptainer", "process"],
                    help="run tasks in containers: process (default) = process groups; auto = Docker "
                         "or Podman when its socket answers, for tasks whose config sets "
                         "environment.image (others stay process groups)")
    ap.add_argument("--container-socket", default=None, help="Docker / Podman API unix socket")
    ap.add_argument("--master-cert-file", default=None,
                    help="CA / self-signed cert of an HTTPS master, or 'noverify'")
    ap.add_argument("--master-cert-name", default=None,
                    help="host name the master's certificate was issued for")
    args = ap.parse_args()
    logging.basicConfig(level=logging.INFO)
    # the agent's own Session and every task it launches (tasks inherit the agent environment)
    # verify the master the same way
    if args.master_cert_file:
        os.environ["DET_MASTER_CERT_FILE"] = os.path.abspath(args.master_cert_file) \
            if args.master_cert_file.lower() != "noverify" else "noverify"
    if args.master_cert_name:
        os.environ["DET_MASTER_CERT_NAME"] = args.master_cert_name
    Agent(args.master_url, args.agent_id, args.resource_pool, args.artificial_slots, args.label,
          slots_per_gpu=args.slots_per_gpu, max_gpus=args.max_gpus,
          container_runtime=args.container_runtime, container_socket=args.container_socket).run()


if __name__ == "__main__":
    main()
