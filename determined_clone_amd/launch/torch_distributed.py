"""Torch-distributed launch layer (reference: `harness/determined/launch/torch_distributed.py`).

Starts one process per assigned MI355X slot with ``torch.distributed.run`` (RCCL over xGMI on one
node, rendezvous on 127.0.0.1), prefixes every line with its rank (``wrap_rank``), and — like the
reference's pid_server — tears the whole group down as soon as one rank fails
(``--max-restarts 0``). Multi-node: container rank/addresses from the cluster info.
"""
import os
import socket
import subprocess
import sys
from typing import List

from determined_clone_amd import _info

C10D_PORT = int(os.environ.get("C10D_PORT", "29400"))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def create_launch_cmd(num_nodes: int, proc_per_node: int, node_rank: int, master_addr: str,
                      port: int, override_args: List[str], script: List[str]) -> List[str]:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", str(num_nodes),
           "--nproc-per-node", str(proc_per_node), "--node-rank", str(node_rank),
           "--max-restarts", "0", "--master-addr", master_addr, "--master-port", str(port)]
    cmd += override_args
    if script and script[0] == sys.executable and len(script) > 2 and script[1] == "-m":
        cmd += ["--module", script[2]] + script[3:]
    elif script and script[0].endswith("python3") or (script and script[0].endswith("python")):
        cmd += script[1:]
    else:
        cmd += ["--no-python"] + script
    return cmd


def main(argv: List[str]) -> int:
    override: List[str] = []
    if "--" in argv:
        i = argv.index("--")
        override, script = argv[:i], argv[i + 1:]
    else:
        script = argv
    info = _info.get_cluster_info()
    if info is None:
        nodes, procs, rank, addr = 1, int(os.environ.get("DET_SLOTS", "1")), 0, "127.0.0.1"
    else:
        nodes = len(info.container_addrs)
        procs = max(len(info.slot_ids), 1)
        rank = info.container_rank
        addr = info.container_addrs[0] if nodes > 1 else "127.0.0.1"
    # multi-node: the port the master reserved for this allocation on the chief's host
    # (master/ports.py), so concurrent jobs sharing a chief node never collide
    port = ((info.rendezvous_port if info is not None else None) or C10D_PORT) if nodes > 1 else _free_port()
    cmd = create_launch_cmd(nodes, procs, rank, addr, port, override, script)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PYTHONUNBUFFERED"] = "1"
    proc = subprocess.Popen(cmd, env=env)
    return proc.wait()


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
