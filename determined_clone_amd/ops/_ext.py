"""Loader for the in-tree HIP extension ``determined_clone_amd.ops._C``.

GPU tensors ALWAYS go through the HIP kernels: if the extension is missing on a machine with a GPU
the op raises (no silent eager fallback). CPU tensors use the PyTorch reference implementations
that the GPU numerics tests compare against.
"""
import importlib
import importlib.machinery
import importlib.util
import os
import sys
from typing import Any, Optional

_C: Optional[Any] = None
_err: Optional[BaseException] = None


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
            _C = importlib.import_module("determined_clone_amd.ops._C")
    except ImportError as e:  # pragma: no cover - exercised only when the build is missing
        _err = e
        if os.environ.get("DCA_AUTOBUILD", "1") == "1":
            from determined_clone_amd.ops import build

            build.build()
            _C = importlib.import_module("determined_clone_amd.ops._C")
        else:
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
