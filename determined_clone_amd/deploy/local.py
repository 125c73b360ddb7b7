"""``det deploy local``: run master + agent(s) as local background processes
(reference: `harness/determined/deploy/local/cluster_utils.py`, which uses Docker containers; this
image has no Docker, so they are plain processes with pid files under ``--state-dir``)."""
import os
import signal
import subprocess
import sys
import time

from determined_clone_amd.common.api import Session


def _pidfile(state_dir: str, name: str) -> str:
    return os.path.join(state_dir, f"{name}.pid")


def _spawn(args_list, state_dir: str, name: str) -> int:
    os.makedirs(state_dir, exist_ok=True)
    log = open(os.path.join(state_dir, f"{name}.log"), "ab")
    p = subprocess.Popen(args_list, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    with open(_pidfile(state_dir, name), "w") as f:
        f.write(str(p.pid))
    return p.pid


def master_up(args) -> None:
    cmd = [sys.executable, "-m", "determined_clone_amd.master", "--port", str(args.master_port),
           "--db", os.path.join(args.state_dir, "master.db")]
    if args.storage_path:
        cmd += ["--checkpoint-dir", args.storage_path]
    _spawn(cmd, args.state_dir, "master")
    url = f"http://127.0.0.1:{args.master_port}"
    for _ in range(120):
        try:
            Session(url, max_retries=0).get("/api/v1/master")
            print(f"master up at {url}")
            return
        except Exception:
            time.sleep(0.5)
    raise RuntimeError("master did not come up; see " + os.path.join(args.state_dir, "master.log"))


def agent_up(args) -> None:
    for i in range(args.agents):
        cmd = [sys.executable, "-m", "determined_clone_amd.agent", "--master-url",
               f"http://127.0.0.1:{args.master_port}", "--agent-id", f"agent-{i}"]
        if args.artificial_slots:
            cmd += ["--artificial-slots", str(args.artificial_slots)]
        if getattr(args, "slots_per_gpu", 1) > 1:
            cmd += ["--slots-per-gpu", str(args.slots_per_gpu)]
        _spawn(cmd, args.state_dir, f"agent-{i}")
    print(f"{args.agents} agent(s) started")


def cluster_up(args) -> None:
    master_up(args)
    agent_up(args)


def cluster_down(args) -> None:
    for fn in sorted(os.listdir(args.state_dir)) if os.path.isdir(args.state_dir) else []:
        if not fn.endswith(".pid"):
            continue
        path = os.path.join(args.state_dir, fn)
        try:
            pid = int(open(path).read().strip())
            os.killpg(pid, signal.SIGTERM)
        except (ValueError, ProcessLookupError, PermissionError):
            pass
        os.remove(path)
    print("cluster down")
