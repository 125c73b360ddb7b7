"""Experimental Core API (reference: `harness/determined/core/_experimental.py`)."""
from typing import Any


class ExperimentalCoreContext:
    def __init__(self, session: Any, trial_id: int) -> None:
        self._session = session
        self._trial_id = trial_id

    def report_task_using_checkpoint(self, checkpoint: Any) -> None:
        uuid = getattr(checkpoint, "uuid", checkpoint)
        self._session.post(f"/api/v1/trials/{self._trial_id}/checkpoint_usage", {"checkpoint_uuid": uuid})

    def report_task_using_model_version(self, model_version: Any) -> None:
        ckpt = getattr(model_version, "checkpoint", None)
        if ckpt is not None:
            self.report_task_using_checkpoint(ckpt)


class DummyExperimentalCoreContext(ExperimentalCoreContext):
    def __init__(self) -> None:
        super().__init__(None, 0)

    def report_task_using_checkpoint(self, checkpoint: Any) -> None:
        pass

    def report_task_using_model_version(self, model_version: Any) -> None:
        pass
