"""DeepSpeedTrial launch layer (reference: `harness/determined/launch/deepspeed.py`).

The reference starts DeepSpeed's launcher (pdsh/ssh fan-out) under a pid_server with one
pid_client per worker. Here the engine is native (``pytorch.deepspeed``), so the per-node launcher is
``torch.distributed.run`` (one process per MI355X, RCCL over xGMI) and -- for multi-node jobs --
every worker runs under ``dca-pidwatch client`` reporting to a ``dca-pidwatch server`` on the node, so
a crashed worker on any node tears the job down within seconds instead of hanging in a
collective. Entry: ``python -m determined_clone_amd.launch.deepspeed [torchrun args --] --trial
module:Class`` or ``... -- script args``.
"""
import os
import sys
import tempfile
from typing import List

from determined_clone_amd import _info
from determined_clone_amd.launch import torch_distributed


def _script(argv: List[str]) -> List[str]:
    if argv and argv[0] == "--trial":
        return [sys.executable, "-m", "determined_clone_amd.exec.harness", argv[1]] + argv[2:]
    return argv


def main(argv: List[str]) -> int:
    override: List[str] = []
    if "--" in argv:
        i = argv.index("--")
        override, rest = argv[:i], argv[i + 1:]
    else:
        rest = argv
    script = _script(rest)
    info = _info.get_cluster_info()
    nodes = len(info.container_addrs) if info else 1
    if nodes <= 1:
        return torch_distributed.main(override + ["--"] + script)
    from determined_clone_amd.exec import pid_server

    procs = max(len(info.slot_ids), 1)
    sock = os.path.join(tempfile.gettempdir(), f"dca-pidwatch-{os.getpid()}.sock")
    worker = [pid_server.binary(), "client", sock, "--"] + script
    launch = [sys.executable, "-m", "determined_clone_amd.launch.torch_distributed"] + override + ["--", *worker]
    return pid_server.main(["--grace-period", "5", "--signal-children", sock, str(procs), "--", *launch])


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
