"""The MIOpen find / perf databases and kernel cache measured on MI355X and shipped in-tree
(``ops/tuned/miopen/{db,cache}``), and how processes use them.

PyTorch runs convolutions in MIOpen's immediate mode (``cudnn.benchmark=False``): the solver of
each convolution comes from the find DB (``*.ufdb.txt``), its tuning parameters from the perf DB
(``*.udb.txt``), its compiled kernels from the kernel cache (``*.ukdb``). With none of them for a
shape, MIOpen falls back to heuristic solvers and compiles kernels at the first call (seconds per
shape, in every fresh process). The shipped files hold the ResNet-50 (bs 1024, including the
space-to-depth stem) and CIFAR-10 search shapes.

* ``configure(env)`` -- point ``MIOPEN_USER_DB_PATH`` / ``MIOPEN_CUSTOM_CACHE_DIR`` at a directory
  pair (default: the shipped one) unless the environment already chose one.
* ``task_dirs(root)`` -- a writable copy under ``root`` seeded from the shipped files: the agent
  gives every task it starts the same copy, so kernels compiled or solvers found by one trial serve
  all later trials of the agent (reference analogue: the cluster-wide kernel caches a container
  image would bake in).
"""
import os
import shutil
from typing import Dict, MutableMapping, Optional, Tuple

SHIPPED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "miopen")


def shipped_dirs() -> Tuple[str, str]:
    return os.path.join(SHIPPED, "db"), os.path.join(SHIPPED, "cache")


def configure(env: Optional[MutableMapping[str, str]] = None, db_dir: Optional[str] = None,
              cache_dir: Optional[str] = None) -> Dict[str, str]:
    """Set the MIOpen DB / cache locations in ``env`` (default ``os.environ``) where unset;
    returns the two values in effect."""
    env = os.environ if env is None else env
    sdb, scache = shipped_dirs()
    env.setdefault("MIOPEN_USER_DB_PATH", db_dir or sdb)
    env.setdefault("MIOPEN_CUSTOM_CACHE_DIR", cache_dir or scache)
    return {"MIOPEN_USER_DB_PATH": env["MIOPEN_USER_DB_PATH"],
            "MIOPEN_CUSTOM_CACHE_DIR": env["MIOPEN_CUSTOM_CACHE_DIR"]}


def use_private_copy(tag: str = "proc", env: Optional[MutableMapping[str, str]] = None) -> Dict[str, str]:
    """Point MIOpen at a writable copy of the shipped files private to ``tag`` (e.g. one per rank)
    under the temp dir, unless the environment already chose a location. Benchmarks and tools use
    this so that find results / compiled kernels never land in the git-tracked shipped directory
    and no two processes of one job share one sqlite DB; only an explicit tuning run writes the
    shipped files."""
    import tempfile

    env = os.environ if env is None else env
    if "MIOPEN_USER_DB_PATH" in env:
        return configure(env)
    root = os.path.join(tempfile.gettempdir(), f"dca_miopen_{os.getuid()}", tag)
    db, cache = task_dirs(root)
    return configure(env, db, cache)


def task_dirs(root: str) -> Tuple[str, str]:
    """``(db_dir, cache_dir)`` under ``root``: created from the shipped files the first time,
    reused afterwards (files a task added are kept)."""
    out = []
    for src, name in zip(shipped_dirs(), ("db", "cache")):
        dst = os.path.join(root, "miopen", name)
        if not os.path.isdir(dst):
            tmp = dst + ".tmp"
            shutil.rmtree(tmp, ignore_errors=True)
            if os.path.isdir(src):
                shutil.copytree(src, tmp)
            else:
                os.makedirs(tmp)
            try:
                os.rename(tmp, dst)
            except OSError:  # another agent thread won the race
                shutil.rmtree(tmp, ignore_errors=True)
        out.append(dst)
    return out[0], out[1]
