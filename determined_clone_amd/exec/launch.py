"""Default task entrypoint (reference: `harness/determined/exec/launch.py`).

Reads the experiment's ``entrypoint``:
* ``"pkg.module:TrialClass"`` (legacy class-based trial) -> ``exec.harness`` (wrapped in the
  torch-distributed launcher when the trial has more than one slot);
* anything else is a command line run as-is (it may itself call a launch layer, e.g.
  ``python3 -m determined_clone_amd.launch.torch_distributed python3 train.py``).
A single-slot class-based trial runs the harness in this process; anything else is started as a
subprocess (never exec'd, see the GPU-box rules) and its exit code is propagated.
"""
import os
import shlex
import subprocess
import sys
from typing import List

from determined_clone_amd import _info


def build_command(entrypoint, slots: int) -> List[str]:
    if isinstance(entrypoint, list):
        ep = entrypoint
    else:
        ep = shlex.split(entrypoint or "")
    if len(ep) == 1 and ":" in ep[0] and not ep[0].endswith(".py"):
        cmd = [sys.executable, "-m", "determined_clone_amd.exec.harness", ep[0]]
        if slots > 1:
            cmd = [sys.executable, "-m", "determined_clone_amd.launch.torch_distributed", "--"] + cmd
        return cmd
    if ep and ep[0] in ("python", "python3"):
        ep = [sys.executable] + ep[1:]
    return ep


def main() -> int:
    info = _info.get_cluster_info()
    if info is None:
        print("exec.launch must run inside a task (no cluster info)", file=sys.stderr)
        return 1
    cfg = info.trial._config if info.task_type == "TRIAL" else {}
    ep = cfg.get("entrypoint") if cfg else None
    if ep is None:
        ep = os.environ.get("DET_ENTRYPOINT", "")
    slots = len(info.slot_ids) if info.slot_ids else 1
    cmd = build_command(ep, slots)
    if not cmd:
        print("no entrypoint configured", file=sys.stderr)
        return 1
    if cmd[:3] == [sys.executable, "-m", "determined_clone_amd.exec.harness"]:
        # single-slot class-based trial: run the harness in this process (one interpreter start
        # per trial instead of two; with the agent's zygote this process is already warm)
        from determined_clone_amd.exec import harness

        return harness.main(cmd[3])
    proc = subprocess.Popen(cmd)
    try:
        return proc.wait()
    except KeyboardInterrupt:
        proc.terminate()
        return proc.wait()


if __name__ == "__main__":
    sys.exit(main())
