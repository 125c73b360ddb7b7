"""``python -m determined_clone_amd.exec.pid_client ADDR -- CMD...``: run one worker under the
native ``dca-pidwatch client`` (registers its pid with the pid server, keepalives, graceful-exit
byte; reference: `harness/determined/exec/pid_client.py`, `ipc.PIDClient`)."""
import subprocess
import sys
from typing import List

from determined_clone_amd.exec.pid_server import binary


def main(argv: List[str]) -> int:
    return subprocess.call([binary(), "client"] + argv)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
