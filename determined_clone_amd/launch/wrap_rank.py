"""Prefix every output line of a worker with its rank (reference:
`harness/determined/launch/wrap_rank.py`), so the master's log viewer can filter by rank.

``python -m determined_clone_amd.launch.wrap_rank RANK|ENVVAR -- CMD...``: RANK may be a number or the
name of an environment variable holding it (``RANK``, ``LOCAL_RANK``...). Lines are split on ``\\n``
AND ``\\r`` so tqdm-style progress bars become separate log lines.
"""
import os
import re
import subprocess
import sys
import threading
from typing import BinaryIO, Iterator, List

_split = re.compile(rb"([\r\n])")
LIMIT = 8191


def iter_lines(fd: BinaryIO) -> Iterator[bytes]:
    buf = b""
    while True:
        chunk = fd.read1(4096) if hasattr(fd, "read1") else fd.read(4096)
        if not chunk:
            break
        buf += chunk
        parts = _split.split(buf)
        buf = parts.pop()  # unterminated tail
        for i in range(0, len(parts), 2):
            yield parts[i] + b"\n"
        while len(buf) > LIMIT:
            yield buf[:LIMIT] + b"\n"
            buf = buf[LIMIT:]
    if buf:
        yield buf + b"\n"


def _pump(src: BinaryIO, dst: BinaryIO, prefix: bytes) -> None:
    for line in iter_lines(src):
        dst.write(prefix + line)
        dst.flush()


def resolve_rank(spec: str) -> str:
    return spec if spec.isdigit() else os.environ.get(spec, "?")


def main(argv: List[str]) -> int:
    if "--" not in argv or argv.index("--") != 1:
        print("usage: wrap_rank RANK|ENVVAR -- CMD...", file=sys.stderr)
        return 2
    rank = resolve_rank(argv[0])
    cmd = argv[2:]
    prefix = f"[rank={rank}] ".encode()
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, bufsize=0)
    ts = [threading.Thread(target=_pump, args=(p.stdout, sys.stdout.buffer, prefix), daemon=True),
          threading.Thread(target=_pump, args=(p.stderr, sys.stderr.buffer, prefix), daemon=True)]
    for t in ts:
        t.start()
    rc = p.wait()
    for t in ts:
        t.join()
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
