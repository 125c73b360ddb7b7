"""SearcherContext / SearcherOperation (reference: `harness/determined/core/_searcher.py`).

Operations carry ABSOLUTE lengths (train until ``op.length`` units, validate, report), which makes
resuming after preemption trivial. The chief polls the master; workers receive the length from the
chief so all ranks train the same amount.
"""
import enum
import logging
from typing import Any, Iterator, Optional

logger = logging.getLogger("determined_clone_amd.core")


class Unit(enum.Enum):
    EPOCHS = "EPOCHS"
    RECORDS = "RECORDS"
    BATCHES = "BATCHES"


def _parse_searcher_units(experiment_config: dict) -> Optional[Unit]:
    searcher = experiment_config.get("searcher", {}) or {}
    if searcher.get("name") == "custom":
        u = searcher.get("unit")
        return Unit[u.upper()] if u else None
    length = searcher.get("max_length")
    if isinstance(length, dict) and len(length) == 1:
        return {"epochs": Unit.EPOCHS, "records": Unit.RECORDS, "batches": Unit.BATCHES}.get(next(iter(length)))
    return None


class SearcherOperation:
    def __init__(self, session: Any, trial_id: int, length: int, is_chief: bool) -> None:
        self._session = session
        self._trial_id = trial_id
        self._length = int(length)
        self._is_chief = is_chief
        self._completed = False

    @property
    def length(self) -> int:
        return self._length

    def report_progress(self, length: float) -> None:
        if not self._is_chief:
            raise RuntimeError("you must only call op.report_progress() from the chief worker")
        if self._completed and length != self._length:
            raise RuntimeError("you must not call op.report_progress() after op.report_completed()")
        self._session.post(f"/api/v1/trials/{self._trial_id}/progress", {"progress": float(length)})

    def report_completed(self, searcher_metric: Any) -> None:
        if not self._is_chief:
            raise RuntimeError("you must only call op.report_completed() from the chief worker")
        if self._completed:
            raise RuntimeError("you may only call op.report_completed() once")
        self._completed = True
        from determined_clone_amd.util import to_python

        self._session.post(f"/api/v1/trials/{self._trial_id}/searcher/completed_operation",
                           {"op": {"length": self._length}, "searcher_metric": to_python(searcher_metric)})


class SearcherMode(enum.Enum):
    WorkersAskChief = "WORKERS_ASK_CHIEF"
    ChiefOnly = "CHIEF_ONLY"


class SearcherContext:
    def __init__(self, session: Any, dist: Any, trial_id: int, run_id: int, allocation_id: str,
                 units: Optional[Unit] = None) -> None:
        self._session = session
        self._dist = dist
        self._trial_id = trial_id
        self._run_id = run_id
        self._allocation_id = allocation_id
        self._units = units

    def _get_searcher_op(self) -> Optional[SearcherOperation]:
        body = self._session.get(f"/api/v1/trials/{self._trial_id}/searcher/operation")
        if body.get("completed"):
            return None
        length = int(body["op"]["validate_after"]["length"])
        return SearcherOperation(self._session, self._trial_id, length, self._dist.rank == 0)

    def operations(self, searcher_mode: SearcherMode = SearcherMode.WorkersAskChief,
                   auto_ack: bool = True) -> Iterator[SearcherOperation]:
        searcher_mode = SearcherMode(searcher_mode)
        if self._dist.rank == 0:
            while True:
                op = self._get_searcher_op()
                if searcher_mode == SearcherMode.WorkersAskChief:
                    self._dist.broadcast(op.length if op else None)
                if op is None:
                    if auto_ack:
                        self.acknowledge_out_of_ops()
                    break
                yield op
                if not op._completed:
                    raise RuntimeError("you must call op.report_completed() on each operation")
        else:
            if searcher_mode != SearcherMode.WorkersAskChief:
                raise RuntimeError("operations(searcher_mode=ChiefOnly) called from a non-chief worker")
            while True:
                length = self._dist.broadcast(None)
                if length is None:
                    break
                yield SearcherOperation(self._session, self._trial_id, length, False)

    def acknowledge_out_of_ops(self) -> None:
        self._session.post(f"/api/v1/allocations/{self._allocation_id}/signals/ack_preemption")

    def get_configured_units(self) -> Optional[Unit]:
        return self._units


class DummySearcherOperation(SearcherOperation):
    def __init__(self, length: int, is_chief: bool) -> None:
        super().__init__(None, 0, length, is_chief)

    def report_progress(self, length: float) -> None:
        if not self._is_chief:
            raise RuntimeError("you must only call op.report_progress() from the chief worker")
        logger.debug(f"progress: {length}/{self._length}")

    def report_completed(self, searcher_metric: Any) -> None:
        if not self._is_chief:
            raise RuntimeError("you must only call op.report_completed() from the chief worker")
        if self._completed:
            raise RuntimeError("you may only call op.report_completed() once")
        self._completed = True
        logger.info(f"searcher op completed (length={self._length}, metric={searcher_metric})")


class DummySearcherContext(SearcherContext):
    """Off-cluster: one operation of ``length`` units."""

    def __init__(self, dist: Any, length: int = 1) -> None:
        super().__init__(None, dist, 0, 0, "", None)
        self._length = length

    def operations(self, searcher_mode: SearcherMode = SearcherMode.WorkersAskChief,
                   auto_ack: bool = True) -> Iterator[SearcherOperation]:
        op = DummySearcherOperation(self._length, self._dist.rank == 0)
        yield op
        if self._dist.rank == 0 and not op._completed:
            raise RuntimeError("you must call op.report_completed() on each operation")

    def acknowledge_out_of_ops(self) -> None:
        pass

    def get_configured_units(self) -> Optional[Unit]:
        return None
