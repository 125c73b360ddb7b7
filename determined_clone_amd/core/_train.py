"""TrainContext: metric reporting (reference: `harness/determined/core/_train.py`)."""
import enum
import logging
import math
import pathlib
from typing import Any, Dict, List, Optional, Set

from determined_clone_amd import util

logger = logging.getLogger("determined_clone_amd.core")


class EarlyExitReason(enum.Enum):
    INVALID_HP = "EXITED_REASON_INVALID_HP"
    USER_REQUESTED_STOP = "EXITED_REASON_USER_REQUESTED_STOP"


class TrainContext:
    def __init__(self, session: Any, trial_id: int, run_id: int, exp_id: int, dist: Any,
                 tensorboard_mode: Any = None, tensorboard_manager: Any = None,
                 tbd_writer: Any = None) -> None:
        self._session = session
        self._trial_id = trial_id
        self._run_id = run_id
        self._exp_id = exp_id
        self._dist = dist
        self._tensorboard_manager = tensorboard_manager
        self._tbd_writer = tbd_writer
        self._last_validation: Optional[int] = None

    def set_status(self, status: str) -> None:
        if self._session is not None:
            self._session.post(f"/api/v1/trials/{self._trial_id}/runner/metadata",
                               {"metadata": {"state": status}})

    def _get_last_validation(self) -> Optional[int]:
        if self._session is None:
            return None
        r = self._session.get(f"/api/v1/trials/{self._trial_id}")
        return (r.get("trial") or {}).get("latest_validation_steps")

    def _report_trial_metrics(self, group: str, steps_completed: int, metrics: Dict[str, Any],
                              batch_metrics: Optional[List[Dict[str, Any]]] = None) -> None:
        if self._dist.rank != 0:
            return
        body = {"metrics": {"trial_id": self._trial_id, "trial_run_id": self._run_id,
                            "steps_completed": int(steps_completed),
                            "avg_metrics": util.to_python(metrics),
                            "batch_metrics": util.to_python(batch_metrics) if batch_metrics else None},
                "group": group}
        self._session.post(f"/api/v1/trials/{self._trial_id}/metrics", body)
        if self._tbd_writer is not None:
            try:
                self._tbd_writer.on_metrics(group, steps_completed, metrics)
            except Exception:  # pragma: no cover - tensorboard is best effort
                logger.exception("tensorboard metric write failed")

    def report_training_metrics(self, steps_completed: int, metrics: Dict[str, Any],
                                batch_metrics: Optional[List[Dict[str, Any]]] = None) -> None:
        self._report_trial_metrics("training", steps_completed, metrics, batch_metrics)

    def report_validation_metrics(self, steps_completed: int, metrics: Dict[str, Any]) -> None:
        self._last_validation = steps_completed
        self._report_trial_metrics("validation", steps_completed, metrics)

    def report_metrics(self, group: str, steps_completed: int, metrics: Dict[str, Any]) -> None:
        self._report_trial_metrics(group, steps_completed, metrics)

    def get_tensorboard_path(self) -> pathlib.Path:
        if self._tensorboard_manager is not None:
            return self._tensorboard_manager.base_path
        return pathlib.Path("/tmp/tensorboard")

    def upload_tensorboard_files(self, selector: Any = None, mangler: Any = None) -> None:
        if self._tensorboard_manager is not None:
            self._tensorboard_manager.sync(selector, mangler)

    def report_early_exit(self, reason: EarlyExitReason) -> None:
        if self._dist.rank != 0 or self._session is None:
            return
        self._session.post(f"/api/v1/trials/{self._trial_id}/early_exit", {"reason": reason.value})

    def get_experiment_best_validation(self) -> Optional[float]:
        if self._session is None:
            return None
        try:
            r = self._session.get(f"/api/v1/experiments/{self._exp_id}/searcher/best_searcher_validation_metric")
        except Exception:
            return None
        return r.get("metric") if r else None


class DummyTrainContext(TrainContext):
    """Off-cluster: metrics are logged (and kept for inspection by tests)."""

    def __init__(self, tensorboard_path: Optional[pathlib.Path] = None) -> None:
        super().__init__(None, 0, 0, 0, None)
        self._tb_path = tensorboard_path
        self.reported: List[Dict[str, Any]] = []

    def set_status(self, status: str) -> None:
        logger.debug(f"status: {status}")

    def _get_last_validation(self) -> Optional[int]:
        return None

    def _report_trial_metrics(self, group, steps_completed, metrics, batch_metrics=None) -> None:
        m = util.to_python(metrics)
        self.reported.append({"group": group, "steps_completed": steps_completed, "metrics": m})
        shown = {k: (round(v, 6) if isinstance(v, float) and math.isfinite(v) else v) for k, v in m.items()}
        logger.info(f"[{group}] steps_completed={steps_completed} {shown}")

    def upload_tensorboard_files(self, selector: Any = None, mangler: Any = None) -> None:
        pass

    def report_early_exit(self, reason: EarlyExitReason) -> None:
        logger.info(f"early exit: {reason.value}")

    def get_experiment_best_validation(self) -> Optional[float]:
        return None

    def get_tensorboard_path(self) -> pathlib.Path:
        return self._tb_path or pathlib.Path("/tmp/tensorboard")
