"""Small helpers (reference: harness/determined/util.py, common/util.py)."""
import inspect
import io
import json
import math
import numbers
import os
import pathlib
import random
import tarfile
from typing import Any, Callable, Dict, Iterable, List, Optional

import numpy as np


def is_overridden(full_method: Callable, parent_class: type) -> bool:
    """True if ``full_method`` (a bound method) overrides the method of the same name."""
    name = full_method.__name__
    parent = getattr(parent_class, name, None)
    if parent is None:
        return True
    return getattr(full_method, "__func__", full_method) is not parent


def has_param(fn: Callable, name: str, pos: Optional[int] = None) -> bool:
    try:
        sig = inspect.signature(fn)
    except (TypeError, ValueError):
        return False
    if name in sig.parameters:
        return True
    if pos is not None:
        return len(sig.parameters) >= pos
    return False


def is_numerical_scalar(v: Any) -> bool:
    if isinstance(v, bool):
        return False
    if isinstance(v, numbers.Number):
        return True
    if isinstance(v, np.ndarray):
        return v.size == 1 and np.issubdtype(v.dtype, np.number)
    try:
        import torch

        if isinstance(v, torch.Tensor):
            return v.numel() == 1
    except ImportError:  # pragma: no cover
        pass
    return False


def to_python(v: Any) -> Any:
    """Metric values -> JSON-friendly python (numpy/torch scalars and arrays)."""
    try:
        import torch

        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    if isinstance(v, np.ndarray):
        return v.item() if v.size == 1 else v.tolist()
    if isinstance(v, np.generic):
        return v.item()
    if isinstance(v, dict):
        return {k: to_python(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [to_python(x) for x in v]
    if isinstance(v, float) and not math.isfinite(v):
        return v
    return v


def json_encode(obj: Any, **kw: Any) -> str:
    def default(o: Any) -> Any:
        o2 = to_python(o)
        if o2 is o:
            return str(o)
        return o2

    return json.dumps(obj, default=default, **kw)


def set_random_seeds(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed % (2**32))
    try:
        import torch

        torch.random.manual_seed(seed)
    except ImportError:  # pragma: no cover
        pass


def tar_directory(path: str, exclude: Iterable[str] = (".git", "__pycache__")) -> bytes:
    """Pack a model-definition directory (context directory upload)."""
    excl = set(exclude)
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tf:
        root = pathlib.Path(path)
        for p in sorted(root.rglob("*")):
            rel = p.relative_to(root)
            if any(part in excl for part in rel.parts):
                continue
            tf.add(str(p), arcname=str(rel), recursive=False)
    return buf.getvalue()


def untar_to(data: bytes, dest: str) -> None:
    os.makedirs(dest, exist_ok=True)
    with tarfile.open(fileobj=io.BytesIO(data), mode="r:gz") as tf:
        for m in tf.getmembers():
            target = os.path.realpath(os.path.join(dest, m.name))
            if not target.startswith(os.path.realpath(dest)):
                raise ValueError(f"unsafe path in context archive: {m.name}")
        tf.extractall(dest)


def merge_dicts(base: Dict[str, Any], override: Dict[str, Any]) -> Dict[str, Any]:
    """Recursive merge (override wins), used for templates and config defaults."""
    out = dict(base)
    for k, v in override.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = merge_dicts(out[k], v)
        else:
            out[k] = v
    return out


def write_user_code(path: pathlib.Path, on_cluster: bool) -> None:
    """Save the model definition next to a checkpoint (reference: util.write_user_code)."""
    src = os.environ.get("DET_CONTEXT_DIR")
    if not (on_cluster and src and os.path.isdir(src)):
        return
    dst = path / "code"
    dst.mkdir(parents=True, exist_ok=True)
    untar_to(tar_directory(src), str(dst))


def chunks(lst: List[Any], n: int) -> Iterable[List[Any]]:
    for i in range(0, len(lst), n):
        yield lst[i:i + n]


def routable_address() -> str:
    """This container's address as other hosts reach it: ``DET_CONTAINER_ADDR`` (e.g. a pod IP),
    else the source address of the default route, else 127.0.0.1 (no network)."""
    import socket

    a = os.environ.get("DET_CONTAINER_ADDR")
    if a:
        return a
    try:
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.connect(("10.255.255.255", 1))
            return s.getsockname()[0]
    except OSError:
        return "127.0.0.1"


# Header the master's /proxy/ route attaches when it forwards to an NTSC task's service; the
# service (exec/shell.py, notebook.py, tensorboard.py) refuses requests without it.
PROXY_SECRET_HEADER = "X-Det-Proxy-Secret"


def proxy_secret_ok(headers: Any) -> bool:
    """True when ``headers`` carry this task's ``DET_TASK_PROXY_SECRET`` (always true off-cluster,
    where no secret is set)."""
    import hmac

    secret = os.environ.get("DET_TASK_PROXY_SECRET")
    if not secret:
        return True
    return hmac.compare_digest(str(headers.get(PROXY_SECRET_HEADER) or ""), secret)



_marked = set()


def startup_mark(what: str, once: bool = True) -> None:
    """With ``DET_STARTUP_TRACE=1``: log ``what`` with the seconds since the agent spawned this task
    process (``DET_SPAWN_TIME``; else since process creation). The task's start-up timeline
    (``tools/bench_asha.py --trace`` averages the marks over a search's trials). GPU work queued
    so far is synchronised first, so a mark includes the device time of what precedes it."""
    if os.environ.get("DET_STARTUP_TRACE") != "1" or (once and what in _marked):
        return
    _marked.add(what)
    import logging
    import time

    import sys as _sys

    torch = _sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        torch.cuda.synchronize()
    if os.environ.get("DET_SPAWN_TIME"):
        since = time.time() - float(os.environ["DET_SPAWN_TIME"])
    else:
        try:
            import psutil

            since = time.time() - psutil.Process().create_time()
        except Exception:  # pragma: no cover - psutil missing
            since = float("nan")
    logging.getLogger("determined_clone_amd.startup").info(f"{what} at +{since:.3f}s")
