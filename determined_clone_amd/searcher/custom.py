"""User-side custom searcher API: ``SearchMethod`` + ``LocalSearchRunner`` / ``RemoteSearchRunner``
(reference: `harness/determined/searcher/_search_method.py`, `_search_runner.py`,
`_remote_search_runner.py`).

An experiment configured with ``searcher: {name: custom}`` makes the master queue searcher EVENTS
(initial_operations, trial_created, validation_completed, trial_closed, trial_exited_early,
trial_progress) instead of deciding itself; a search runner long-polls
``GET /api/v1/experiments/{id}/searcher_events``, asks the user's :class:`SearchMethod` for
operations and posts them to ``POST /api/v1/experiments/{id}/searcher_operations``. Runner state is
persisted after every event (JSON, not pickle) so a crashed runner resumes and re-posts the
operations of the last event.
"""
import abc
import base64
import json
import logging
import os
import pathlib
import time
import uuid
from typing import Any, Dict, List, Optional, Sequence, Set, Tuple, Union

from determined_clone_amd.searcher.methods import Close, Create, Operation, Shutdown, ValidateAfter

logger = logging.getLogger("determined_clone_amd.searcher")


class Progress(Operation):
    """Report overall search progress (0..1) to the master."""

    kind = "Progress"

    def __init__(self, progress: float) -> None:
        self.progress = float(progress)


class ExitedReason:
    ERRORED = "ERRORED"
    USER_CANCELED = "USER_CANCELED"
    INVALID_HP = "INVALID_HP"

    @classmethod
    def from_master(cls, reason: Optional[str]) -> str:
        if reason in ("INVALID_HP", "INIT_INVALID_HP"):
            return cls.INVALID_HP
        if reason in ("USER_CANCELED", "USER_REQUESTED_STOP"):
            return cls.USER_CANCELED
        return cls.ERRORED


class SearcherState:
    """Bookkeeping the runner maintains for the search method (do not modify it in the method)."""

    def __init__(self) -> None:
        self.failures: Set[uuid.UUID] = set()
        self.trial_progress: Dict[uuid.UUID, float] = {}
        self.trials_closed: Set[uuid.UUID] = set()
        self.trials_created: Set[uuid.UUID] = set()
        self.last_event_id = 0
        self.experiment_id: Optional[int] = None
        self.experiment_completed = False
        self.experiment_failed = False

    def to_dict(self) -> Dict[str, Any]:
        return {
            "failures": [str(f) for f in self.failures],
            "trialProgress": {str(k): v for k, v in self.trial_progress.items()},
            "trialsClosed": [str(t) for t in self.trials_closed],
            "trialsCreated": [str(t) for t in self.trials_created],
            "lastEventId": self.last_event_id,
            "experimentId": self.experiment_id,
            "experimentCompleted": self.experiment_completed,
            "experimentFailed": self.experiment_failed,
        }

    def from_dict(self, d: Dict[str, Any]) -> None:
        self.failures = {uuid.UUID(f) for f in d.get("failures", [])}
        self.trial_progress = {uuid.UUID(k): v for k, v in d.get("trialProgress", {}).items()}
        self.trials_closed = {uuid.UUID(t) for t in d.get("trialsClosed", [])}
        self.trials_created = {uuid.UUID(t) for t in d.get("trialsCreated", [])}
        self.last_event_id = d.get("lastEventId", 0)
        self.experiment_id = d.get("experimentId")
        self.experiment_completed = d.get("experimentCompleted", False)
        self.experiment_failed = d.get("experimentFailed", False)


class SearchMethod(metaclass=abc.ABCMeta):
    """Implement a hyperparameter search by reacting to trial events with operations
    (:class:`Create`, :class:`ValidateAfter`, :class:`Close`, :class:`Shutdown`)."""

    @abc.abstractmethod
    def initial_operations(self, searcher_state: SearcherState) -> List[Operation]:
        pass

    @abc.abstractmethod
    def on_trial_created(self, searcher_state: SearcherState, request_id: uuid.UUID) -> List[Operation]:
        pass

    @abc.abstractmethod
    def on_validation_completed(self, searcher_state: SearcherState, request_id: uuid.UUID,
                                metric: Any, train_length: int) -> List[Operation]:
        pass

    @abc.abstractmethod
    def on_trial_closed(self, searcher_state: SearcherState, request_id: uuid.UUID) -> List[Operation]:
        pass

    @abc.abstractmethod
    def progress(self, searcher_state: SearcherState) -> float:
        pass

    @abc.abstractmethod
    def on_trial_exited_early(self, searcher_state: SearcherState, request_id: uuid.UUID,
                              exited_reason: str) -> List[Operation]:
        pass

    # -------- persistence (JSON; override *_method_state for method-specific fields)
    def save(self, searcher_state: SearcherState, path: pathlib.Path, *, experiment_id: int,
             operations: List[Operation]) -> None:
        path.mkdir(parents=True, exist_ok=True)
        (path / "searcher_state.json").write_text(json.dumps({
            "state": searcher_state.to_dict(), "experiment_id": experiment_id,
            "operations": [_op_to_wire(o) for o in operations]}))
        self.save_method_state(path)

    def save_method_state(self, path: pathlib.Path) -> None:
        pass

    def load(self, path: pathlib.Path) -> Tuple[SearcherState, int, List[Operation]]:
        d = json.loads((path / "searcher_state.json").read_text())
        st = SearcherState()
        st.from_dict(d["state"])
        self.load_method_state(path)
        return st, int(d["experiment_id"]), [_op_from_wire(o) for o in d.get("operations", [])]

    def load_method_state(self, path: pathlib.Path) -> None:
        pass


def _op_to_wire(op: Operation) -> Dict[str, Any]:
    d = op.to_dict()
    if "request_id" in d:
        d["request_id"] = str(d["request_id"])
    return d


def _op_from_wire(d: Dict[str, Any]) -> Operation:
    d = dict(d)
    kind = d.pop("kind")
    if kind == "Progress":
        return Progress(**d)
    return {"Create": Create, "ValidateAfter": ValidateAfter, "Close": Close, "Shutdown": Shutdown}[kind](**d)


class _ExperimentInactive(Exception):
    def __init__(self, state: str) -> None:
        super().__init__(state)
        self.state = state


TERMINAL = ("COMPLETED", "CANCELED", "ERROR", "DELETED")


class SearchRunner:
    def __init__(self, search_method: SearchMethod) -> None:
        self.search_method = search_method
        self.state = SearcherState()

    # ------------------------------------------------------------------ event dispatch
    def _get_operations(self, event: Dict[str, Any]) -> List[Operation]:
        kind = event["type"]
        sm, st = self.search_method, self.state
        if kind == "initial_operations":
            return sm.initial_operations(st)
        rid = uuid.UUID(event["request_id"]) if event.get("request_id") else None
        if kind == "trial_created":
            st.trials_created.add(rid)
            st.trial_progress[rid] = 0.0
            return sm.on_trial_created(st, rid)
        if kind == "trial_closed":
            st.trials_closed.add(rid)
            ops = sm.on_trial_closed(st, rid)
            return ops + [Progress(sm.progress(st))]
        if kind == "trial_exited_early":
            reason = ExitedReason.from_master(event.get("exited_reason"))
            if reason == ExitedReason.INVALID_HP:
                st.trial_progress.pop(rid, None)
            elif reason == ExitedReason.ERRORED:
                st.failures.add(rid)
            ops = sm.on_trial_exited_early(st, rid, reason)
            return ops + [Progress(sm.progress(st))]
        if kind == "validation_completed":
            if event.get("metric") is None:
                raise RuntimeError("validation_completed event without a metric")
            ops = sm.on_validation_completed(st, rid, event["metric"], int(event.get("validate_after_length", 0)))
            return ops + [Progress(sm.progress(st))]
        if kind == "trial_progress":
            st.trial_progress[rid] = float(event.get("partial_units", 0.0))
            return [Progress(sm.progress(st))]
        raise RuntimeError(f"Unsupported searcher event {event}")

    # ------------------------------------------------------------------ master I/O
    def get_events(self, session: Any, experiment_id: int) -> List[Dict[str, Any]]:
        return session.get(f"/api/v1/experiments/{experiment_id}/searcher_events")["searcher_events"]

    def post_operations(self, session: Any, experiment_id: int, event: Dict[str, Any],
                        operations: List[Operation]) -> None:
        body: Dict[str, Any] = {"triggered_by_event_id": event["id"], "searcher_operations": []}
        for op in operations:
            if isinstance(op, Progress):
                body["progress"] = op.progress
            else:
                body["searcher_operations"].append(_op_to_wire(op))
        session.post(f"/api/v1/experiments/{experiment_id}/searcher_operations", body)

    def _experiment_state(self, session: Any, experiment_id: int) -> str:
        return session.get(f"/api/v1/experiments/{experiment_id}")["experiment"]["state"]

    def run_experiment(self, experiment_id: int, session: Any,
                       prior_operations: Optional[List[Operation]] = None,
                       sleep_time: float = 0.2, timeout: Optional[float] = None) -> None:
        self.state.experiment_id = experiment_id
        t0 = time.time()
        while True:
            events = self.get_events(session, experiment_id)
            new = [e for e in events if e["id"] > self.state.last_event_id]
            # an event we already answered but whose ack may not have reached the master
            replay = [e for e in events if e["id"] <= self.state.last_event_id]
            if replay and prior_operations is not None:
                logger.info(f"re-posting operations for event {replay[-1]['id']}")
                self.post_operations(session, experiment_id, replay[-1], prior_operations)
                prior_operations = None
            for ev in new:
                ops = self._get_operations(ev)
                self.state.last_event_id = ev["id"]
                self.save_state(experiment_id, ops)
                self.post_operations(session, experiment_id, ev, ops)
            if not new:
                state = self._experiment_state(session, experiment_id)
                if state in TERMINAL:
                    self.state.experiment_completed = state == "COMPLETED"
                    self.state.experiment_failed = state == "ERROR"
                    self.save_state(experiment_id, [])
                    return
                if state == "PAUSED":
                    self._show_experiment_paused_msg()
                if timeout is not None and time.time() - t0 > timeout:
                    raise TimeoutError(f"experiment {experiment_id} still {state}")
                time.sleep(sleep_time)

    def save_state(self, experiment_id: int, operations: List[Operation]) -> None:
        pass

    def _show_experiment_paused_msg(self) -> None:
        pass


def _create_experiment(session: Any, exp_config: Union[Dict[str, Any], str],
                       model_dir: Union[str, pathlib.Path]) -> int:
    import yaml

    from determined_clone_amd.util import tar_directory

    cfg = yaml.safe_load(exp_config) if isinstance(exp_config, str) else dict(exp_config)
    cfg.setdefault("searcher", {})
    cfg["searcher"]["name"] = "custom"
    body = {"config": cfg,
            "model_definition": base64.b64encode(tar_directory(str(model_dir))).decode()}
    return int(session.post("/api/v1/experiments", body)["experiment"]["id"])


class LocalSearchRunner(SearchRunner):
    """Runs the search method in THIS process (e.g. a laptop) against a master; state lives under
    ``searcher_dir/exp_<id>/`` so re-running the script resumes the same experiment."""

    def __init__(self, search_method: SearchMethod, searcher_dir: Optional[pathlib.Path] = None,
                 session: Any = None) -> None:
        super().__init__(search_method)
        self.searcher_dir = pathlib.Path(searcher_dir or os.getcwd())
        if session is None:
            from determined_clone_amd.common.api import Session

            session = Session(os.environ.get("DET_MASTER", "http://127.0.0.1:8080"))
        self.session = session

    def run(self, exp_config: Union[Dict[str, Any], str], model_dir: Optional[str] = None,
            timeout: Optional[float] = None) -> int:
        exp_file = self.searcher_dir / "experiment_id"
        prior: Optional[List[Operation]] = None
        if exp_file.exists():
            experiment_id = int(exp_file.read_text())
            path = self._get_state_path(experiment_id)
            if (path / "searcher_state.json").exists():
                self.state, _, prior = self.search_method.load(path)
            logger.info(f"resuming custom search for experiment {experiment_id}")
        else:
            experiment_id = _create_experiment(self.session, exp_config, model_dir or os.getcwd())
            self.searcher_dir.mkdir(parents=True, exist_ok=True)
            exp_file.write_text(str(experiment_id))
        self.state.experiment_id = experiment_id
        self.run_experiment(experiment_id, self.session, prior, timeout=timeout)
        return experiment_id

    def load_state(self, experiment_id: int) -> Tuple[int, List[Operation]]:
        self.state, eid, ops = self.search_method.load(self._get_state_path(experiment_id))
        return eid, ops

    def save_state(self, experiment_id: int, operations: List[Operation]) -> None:
        self.search_method.save(self.state, self._get_state_path(experiment_id),
                                experiment_id=experiment_id, operations=operations)

    def _get_state_path(self, experiment_id: int) -> pathlib.Path:
        return self.searcher_dir / f"exp_{experiment_id}"

    def _show_experiment_paused_msg(self) -> None:
        logger.info(f"experiment {self.state.experiment_id} is paused; waiting for activation")


class RemoteSearchRunner(SearchRunner):
    """Runs the search method inside a Determined task (core.Context): state is checkpointed
    through ``core_context.checkpoint`` so the runner task itself can be preempted/resumed."""

    def __init__(self, search_method: SearchMethod, context: Any) -> None:
        super().__init__(search_method)
        self.context = context
        from determined_clone_amd import _info
        from determined_clone_amd.common.api import Session

        info = _info.get_cluster_info()
        self.session = Session(info.master_url if info else os.environ.get("DET_MASTER", ""))
        if info and getattr(info, "session_token", None):
            self.session.token = info.session_token
        self.info = info

    def run(self, exp_config: Union[Dict[str, Any], str], model_dir: Optional[str] = None,
            timeout: Optional[float] = None) -> int:
        prior = None
        latest = self.info.latest_checkpoint if self.info else None
        if latest is not None:
            eid, prior = self.load_state(latest)
        else:
            eid = _create_experiment(self.session, exp_config, model_dir or os.getcwd())
        self.state.experiment_id = eid
        self.run_experiment(eid, self.session, prior, timeout=timeout)
        return eid

    def load_state(self, storage_id: str) -> Tuple[int, List[Operation]]:
        with self.context.checkpoint.restore_path(storage_id) as path:
            self.state, eid, ops = self.search_method.load(pathlib.Path(path))
        return eid, ops

    def save_state(self, experiment_id: int, operations: List[Operation]) -> None:
        md = {"steps_completed": self.state.last_event_id}
        with self.context.checkpoint.store_path(md) as (path, _sid):
            self.search_method.save(self.state, pathlib.Path(path), experiment_id=experiment_id,
                                    operations=operations)
