"""Loader for the in-tree HIP extension ``determined_clone_amd.ops._C``.

GPU tensors ALWAYS go through the HIP kernels: if the extension is missing on a machine with a GPU
the op raises (no silent eager fallback). CPU tensors use the PyTorch reference implementations
that the GPU numerics tests compare against.

A binary built from other sources than the ``csrc/`` next to it is refused: ``_C.source_hash`` (the
hash ``ops/build.py`` links in) must equal the hash of the tree (:class:`StaleExtensionError`).
``DCA_OPS_SO`` (an explicit A/B build of modified sources) skips the check.
"""
import importlib
import importlib.machinery
import importlib.util
import os
import sys
from typing import Any, Optional

_C: Optional[Any] = None
_err: Optional[BaseException] = None


class StaleExtensionError(ImportError):
    """``_C.so`` was not built from the ``csrc/`` sources of this tree."""


def check_fresh(mod: Any) -> None:
    """Raise :class:`StaleExtensionError` unless ``mod`` was built from the current sources."""
    from determined_clone_amd.ops import build

    if not build.CSRC.is_dir():  # installed without sources: nothing to compare against
        return
    want = build.source_hash()
    got = getattr(mod, "source_hash", "")
    if got != want:
        raise StaleExtensionError(
            f"{getattr(mod, '__file__', '_C')} is stale: built from sources {got[:12] or '<unknown>'}, "
            f"the tree has {want[:12]}; rebuild with `python -m determined_clone_amd.ops.build`")


def load() -> Any:
    global _C, _err
    if _C is not None:
        return _C
    import torch  # noqa: F401  (loads libc10_hip / libamdhip64 before the extension)

    alt = os.environ.get("DCA_OPS_SO")
    if alt:  # A/B builds: load this file as the extension (e.g. a variant built with other flags)
        loader = importlib.machinery.ExtensionFileLoader("determined_clone_amd.ops._C", alt)
        spec = importlib.util.spec_from_file_location("determined_clone_amd.ops._C", alt, loader=loader)
        _C = importlib.util.module_from_spec(spec)
        loader.exec_module(_C)
        sys.modules["determined_clone_amd.ops._C"] = _C
    try:
        if _C is None:
            if os.environ.get("DCA_AUTOBUILD", "1") == "1":
                from determined_clone_amd.ops import build

                if build.linked_hash() != build.source_hash():  # missing or stale: rebuild first
                    build.build()
            mod = importlib.import_module("determined_clone_amd.ops._C")
            check_fresh(mod)
            _C = mod
    except ImportError as e:
        _err = e
        if isinstance(e, StaleExtensionError):
            raise
        raise ImportError(
            "determined_clone_amd.ops._C is not built; run "
            "`python -m determined_clone_amd.ops.build`"
        ) from e
    import torch

    if torch.cuda.is_available():
        # replay the shipped tuned hipBLASLt/rocBLAS GEMM solutions (ops/gemm_tuning.py)
        from determined_clone_amd.ops import gemm_tuning

        gemm_tuning.enable()
    return _C


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False
