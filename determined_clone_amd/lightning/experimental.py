"""``DetLogger``: a PyTorch Lightning logger that reports through Core API v2 (reference:
`harness/determined/lightning/experimental.py:12`).

Lightning is not part of this image, so the class subclasses Lightning's ``Logger`` when it is
importable and otherwise implements the same duck-typed surface (``experiment``, ``name``,
``version``, ``log_hyperparams``, ``log_metrics``, ``save``, ``finalize``) -- a Lightning
``Trainer(logger=DetLogger(...))`` only calls those. Rank-zero-only like the reference (the
``RANK`` environment variable decides; a Lightning install uses its own ``rank_zero_only``).
"""
import functools
import os
from typing import Any, Callable, Dict, Optional

from determined_clone_amd.experimental import core_v2

try:  # pragma: no cover - Lightning is not installed in this image
    from lightning.pytorch.loggers.logger import Logger as _LoggerBase
except ImportError:  # pragma: no cover
    _LoggerBase = object


def _rank_zero_only(fn: Callable[..., Any]) -> Callable[..., Any]:
    @functools.wraps(fn)
    def wrapped(*args: Any, **kwargs: Any) -> Any:
        if int(os.environ.get("RANK", os.environ.get("LOCAL_RANK", "0"))) != 0:
            return None
        return fn(*args, **kwargs)

    return wrapped


class DetLogger(_LoggerBase):  # type: ignore[misc,valid-type]
    def __init__(self, *, defaults: Optional[core_v2.DefaultConfig] = None,
                 unmanaged: Optional[core_v2.UnmanagedConfig] = None, client: Any = None) -> None:
        if _LoggerBase is not object:
            super().__init__()
        self._kwargs = {"defaults": defaults, "client": client, "unmanaged": unmanaged}
        self._initialized = False

    @property
    def experiment(self) -> None:
        """Starts (or resumes) the Core API v2 run on first use (rank 0 only)."""
        if int(os.environ.get("RANK", "0")) == 0 and not self._initialized:
            core_v2.init(**self._kwargs)
            self._initialized = True
        return None

    @property
    def name(self) -> str:
        return "DetLogger"

    @property
    def version(self) -> str:
        return "0.1"

    @_rank_zero_only
    def log_hyperparams(self, params: Any, *args: Any, **kwargs: Any) -> None:
        # hyper-parameters are part of the experiment config (DefaultConfig.hparams)
        pass

    @_rank_zero_only
    def log_metrics(self, metrics: Dict[str, float], step: Optional[int] = None) -> None:
        self.experiment  # noqa: B018 - lazily initialise like Lightning's logger contract
        core_v2.train.report_training_metrics(int(step or 0), dict(metrics))

    @_rank_zero_only
    def save(self) -> None:
        pass

    @_rank_zero_only
    def finalize(self, status: str) -> None:
        if self._initialized:
            core_v2.close()
            self._initialized = False
