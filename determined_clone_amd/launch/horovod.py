"""``python -m determined_clone_amd.launch.horovod [--autohorovod] [horovodrun args] -- script...``

Reference: `harness/determined/launch/horovod.py` -- the default launch layer of Determined,
which runs the entrypoint under ``horovodrun`` (MPI/Gloo rendezvous over SSH between containers,
NCCL allreduce) when ``slots_per_trial > 1`` and as a plain subprocess otherwise.

Horovod is not part of this stack: the data-parallel allreduce is RCCL over xGMI through
``torch.distributed`` (``parallel/ddp.py``), one process per MI355X. This launcher keeps the
entrypoint contract so existing experiment configs run unchanged: a single slot runs the script
directly; several slots run it under ``launch.torch_distributed`` (same rank environment:
RANK / LOCAL_RANK / WORLD_SIZE, plus HOROVOD_RANK / HOROVOD_SIZE / HOROVOD_LOCAL_RANK aliases for
scripts that read them). ``horovodrun``-specific flags before ``--`` are accepted and ignored
with a warning.
"""
import logging
import os
import subprocess
import sys
from typing import List

from determined_clone_amd import _info
from determined_clone_amd.launch import torch_distributed

logger = logging.getLogger("determined_clone_amd.launch.horovod")


def _split(argv: List[str]):
    autohorovod = "--autohorovod" in argv
    argv = [a for a in argv if a != "--autohorovod"]
    if "--" in argv:
        i = argv.index("--")
        return autohorovod, argv[:i], argv[i + 1:]
    return autohorovod, [], argv


def main(argv: List[str]) -> int:
    _, hvd_args, script = _split(argv)
    if not script:
        print("usage: launch.horovod [--autohorovod] [horovodrun args] -- script ...", file=sys.stderr)
        return 1
    if hvd_args:
        logger.warning(f"ignoring horovodrun arguments {hvd_args}: RCCL via torch.distributed is used")
    info = _info.get_cluster_info()
    slots = len(info.slot_ids) if info and info.slot_ids else int(os.environ.get("DET_SLOTS", "1"))
    nodes = len(info.container_addrs) if info else 1
    if slots * nodes <= 1:
        if script[0] in ("python", "python3"):
            script = [sys.executable] + script[1:]
        return subprocess.Popen(script).wait()
    # horovod-style rank variables are derived from the torch.distributed ones in each rank
    return torch_distributed.main(["--", sys.executable, "-m", "determined_clone_amd.launch.horovod",
                                   "--rank-env-shim", "--"] + script)


def _rank_env_shim(script: List[str]) -> int:
    env = dict(os.environ)
    env["HOROVOD_RANK"] = env.get("RANK", "0")
    env["HOROVOD_SIZE"] = env.get("WORLD_SIZE", "1")
    env["HOROVOD_LOCAL_RANK"] = env.get("LOCAL_RANK", "0")
    env["HOROVOD_LOCAL_SIZE"] = env.get("LOCAL_WORLD_SIZE", "1")
    if script and script[0] in ("python", "python3"):
        script = [sys.executable] + script[1:]
    return subprocess.Popen(script, env=env).wait()


if __name__ == "__main__":
    if sys.argv[1:2] == ["--rank-env-shim"]:
        args = sys.argv[2:]
        sys.exit(_rank_env_shim(args[1:] if args[:1] == ["--"] else args))
    sys.exit(main(sys.argv[1:]))
