"""``python -m determined_clone_amd.exec.pid_server [opts] ADDR NUM_WORKERS -- CMD...``

Thin entry point for the native ``dca-pidwatch server`` (native/pidwatch.cpp): runs the launch layer
CMD and tears the whole job down when any worker that registered through ``pid_client`` exits
without a graceful shutdown (reference: `harness/determined/exec/pid_server.py`, `ipc.PIDServer`).
"""
import subprocess
import sys
from typing import List


def binary() -> str:
    from determined_clone_amd.native import build

    return str(build.build_pidwatch())


def main(argv: List[str]) -> int:
    return subprocess.call([binary(), "server"] + argv)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
