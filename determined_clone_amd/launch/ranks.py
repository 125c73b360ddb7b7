"""Self-launch for single-node benchmark and tool scripts: ``--gpus N`` without a launcher.

A script that is started as ``python script.py --gpus N`` (no ``torch.distributed.run`` around it)
calls :func:`run_as_ranks` before it touches the GPU; that starts
``torch.distributed.run --nnodes=1 --nproc-per-node N`` on the same script as a CHILD process
(never an exec: a process that initialised HIP must not replace itself), forwards the ranks'
output, and returns the exit code. Only JSON lines (``{...}``) are collected, and exactly one is
expected from rank 0 by default; it is printed last so a caller reading the final JSON line gets
it. The ranks find RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, as under the
reference's ``launch/torch_distributed.py`` for a multi-slot trial.
"""
import os
import signal
import socket
import subprocess
import sys
from typing import List, Optional, Sequence


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def needs_launch(nproc: int) -> bool:
    """True when ``nproc`` ranks were asked for and this process is not one of them."""
    return nproc > 1 and "RANK" not in os.environ


def run_as_ranks(script: str, argv: Sequence[str], nproc: int, expect_json: Optional[int] = 1,
                 env: Optional[dict] = None) -> int:
    """Run ``script argv`` as ``nproc`` local ranks; returns 0 only if every rank exited 0 and
    ``expect_json`` JSON lines (None: any number) were printed."""
    cmd: List[str] = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                      "--nproc-per-node", str(nproc), "--master-addr", "127.0.0.1",
                      "--master-port", str(free_port()), os.path.abspath(script), *argv]
    child_env = dict(os.environ if env is None else env)
    # dmabuf IPC: the host driver has no legacy IPC, RCCL needs this in every rank
    child_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    child = subprocess.Popen(cmd, env=child_env, stdout=subprocess.PIPE, text=True)

    def _forward(signum, _frame):  # a timeout that signals us reaches the ranks as well
        child.send_signal(signum)

    old = {s: signal.signal(s, _forward) for s in (signal.SIGTERM, signal.SIGINT)}
    json_lines: List[str] = []
    try:
        assert child.stdout is not None
        for line in child.stdout:
            if line.startswith("{"):
                json_lines.append(line)
            else:
                sys.stdout.write(line)
                sys.stdout.flush()
        rc = child.wait()
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    for line in json_lines:
        sys.stdout.write(line)
    sys.stdout.flush()
    if rc != 0:
        print(f"{os.path.basename(script)}: torch.distributed.run exited with {rc}", file=sys.stderr)
        return rc if rc > 0 else 1
    if expect_json is not None and len(json_lines) != expect_json:
        print(f"{os.path.basename(script)}: expected {expect_json} JSON line(s), got "
              f"{len(json_lines)}", file=sys.stderr)
        return 1
    return 0
