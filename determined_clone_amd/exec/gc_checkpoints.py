"""``python -m determined_clone_amd.exec.gc_checkpoints`` -- checkpoint garbage collection as a
task (reference: `harness/determined/exec/gc_checkpoints.py`: the master launches it with the
storage config and the storage ids to delete when an experiment's ``save_*`` policy or a
``det checkpoint rm`` drops checkpoints, so deletion runs where the storage is mounted).

Inputs: ``--storage-config`` / ``--delete`` / ``--globs`` (JSON files) or the ``DET_STORAGE_CONFIG``
/ ``DET_DELETE`` / ``DET_GLOB`` environment variables (JSON text), ``--delete-tensorboards``
(with ``--experiment-id``), ``--dry-run``. With globs only the matching files of each checkpoint
are removed; the remaining resources are printed as JSON (one line per checkpoint) so the caller
can update its registry.
"""
import argparse
import json
import logging
import os
import sys
from typing import Any, List, Optional

from determined_clone_amd.common import storage

logger = logging.getLogger("determined_clone_amd.exec.gc_checkpoints")


def _json_arg(val: str) -> Any:
    with open(val) as f:
        return json.load(f)


def _env_json(name: str, default: Any) -> Any:
    v = os.environ.get(name)
    return json.loads(v) if v else default


def mask(cfg: dict) -> dict:
    secret = ("secret", "key", "token", "password", "connection_string")
    return {k: ("***" if any(s in k for s in secret) and v else v) for k, v in cfg.items()}


def main(argv: Optional[List[str]] = None) -> int:
    p = argparse.ArgumentParser(description="checkpoint GC")
    p.add_argument("--experiment-id")
    p.add_argument("--log-level", default=os.getenv("DET_LOG_LEVEL", "INFO"),
                   choices=["DEBUG", "INFO", "WARNING", "ERROR"])
    p.add_argument("--storage-config", type=_json_arg, default=_env_json("DET_STORAGE_CONFIG", {}))
    p.add_argument("--delete", type=_json_arg, default=_env_json("DET_DELETE", []))
    p.add_argument("--globs", type=_json_arg, default=_env_json("DET_GLOB", []))
    p.add_argument("--delete-tensorboards", action="store_true",
                   default=bool(os.getenv("DET_DELETE_TENSORBOARDS")))
    p.add_argument("--dry-run", action="store_true", default="DET_DRY_RUN" in os.environ)
    a = p.parse_args(argv)
    logging.basicConfig(level=a.log_level, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    logger.info(f"checkpoint storage: {json.dumps(mask(a.storage_config))}")
    manager = storage.build(a.storage_config)
    ids = [s.strip() for s in a.delete]
    globs = [g.strip() for g in a.globs]
    for sid in ids:
        if a.dry_run:
            logger.info(f"dry run: would delete {sid} {globs or '(all files)'}")
            continue
        remaining = manager.delete(sid, globs or None)
        print(json.dumps({"storage_id": sid, "resources": remaining or {}}), flush=True)
        logger.info(f"deleted {sid}" + (f" (globs {globs})" if globs else ""))
    if a.delete_tensorboards and a.experiment_id:
        root = a.storage_config.get("host_path") or a.storage_config.get("container_path")
        if root and not a.dry_run:
            import glob as _g
            import shutil

            for d in _g.glob(os.path.join(root, a.storage_config.get("storage_path") or "", "tensorboard", "*",
                                          "experiment", str(a.experiment_id))):
                shutil.rmtree(d, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
