"""Experiment and trial lifecycle (reference: `master/internal/experiment.go`, `trial.go`,
`restore.go`).

An Experiment owns a Searcher and turns its operations into trials:
* Create        -> a trial row + an allocation request (slots_per_trial, priority, weight)
* ValidateAfter -> the trial's current target length (served by GET .../searcher/operation)
* Close         -> the trial finishes once its process exits cleanly
* Shutdown      -> the experiment completes (or errors) when its trials are gone
Trial processes that exit with no outstanding operation and are not closed are "waiting" (e.g.
un-promoted ASHA trials); a later ValidateAfter restarts them from their latest checkpoint.
Non-zero exits are retried up to ``max_restarts``; preemption (pause, higher-priority work)
checkpoints and re-queues.
"""
import json
import logging
import threading
import time
import uuid
from typing import Any, Dict, List, Optional

from determined_clone_amd.master.db import DB, dec, now
from determined_clone_amd.master.rm import AllocationRequest
from determined_clone_amd.searcher import Searcher
from determined_clone_amd.searcher.methods import (Close, Create, ExitedReason, Shutdown,
                                                   ValidateAfter, make_search_method)

logger = logging.getLogger("determined_clone_amd.master")

ACTIVE, PAUSED, STOPPING_CANCELED, STOPPING_COMPLETED, STOPPING_ERROR = (
    "ACTIVE", "PAUSED", "STOPPING_CANCELED", "STOPPING_COMPLETED", "STOPPING_ERROR")
COMPLETED, CANCELED, ERROR = "COMPLETED", "CANCELED", "ERROR"
TERMINAL = {COMPLETED, CANCELED, ERROR}


class Trial:
    def __init__(self, exp: "Experiment", trial_id: int, request_id: str, hparams: Dict[str, Any],
                 seed: int) -> None:
        self.exp = exp
        self.id = trial_id
        self.request_id = request_id
        self.hparams = hparams
        self.seed = seed
        self.state = ACTIVE
        self.op: Optional[ValidateAfter] = None  # current target
        self.op_complete = True
        self.closed = False
        self.restarts = 0
        self.run_id = 0
        self.allocation_id: Optional[str] = None
        self.allocation_state: Optional[str] = None
        self.task_id = f"{exp.id}.{request_id}"
        self.latest_checkpoint: Optional[str] = None
        self.steps_completed = 0
        self.killed = False
        self.preempt_event = threading.Event()
        self.exited_early = False

    # searcher view served to the trial process
    def searcher_operation(self) -> Dict[str, Any]:
        if self.op is None:
            return {"op": None, "completed": True}
        return {"op": {"validate_after": {"length": self.op.length}},
                "completed": self.op_complete}

    def needs_run(self) -> bool:
        return (not self.op_complete or (self.closed and False)) and self.state not in TERMINAL

    def to_dict(self) -> Dict[str, Any]:
        row = self.exp.master.db.one("SELECT * FROM trials WHERE id=?", [self.id]) or {}
        return trial_row_to_api(row, self)


def trial_row_to_api(row: Dict[str, Any], t: Optional[Trial] = None) -> Dict[str, Any]:
    return {
        "id": row.get("id"), "experiment_id": row.get("experiment_id"),
        "request_id": row.get("request_id"), "hparams": dec(row.get("hparams"), {}),
        "state": (t.state if t else row.get("state")), "start_time": row.get("start_time"),
        "end_time": row.get("end_time"), "restarts": (t.restarts if t else row.get("restarts")),
        "seed": row.get("seed"), "run_id": row.get("run_id"),
        "steps_completed": row.get("steps_completed"), "latest_checkpoint": row.get("latest_checkpoint"),
        "best_validation": row.get("best_validation"),
        "latest_validation_steps": row.get("latest_validation_steps"),
        "summary_metrics": dec(row.get("summary_metrics"), {}), "task_id": row.get("task_id"),
        "runner_state": row.get("runner_state"), "progress": row.get("progress"),
        "searcher_op": (t.searcher_operation() if t else None),
    }


class Experiment:
    def __init__(self, master: Any, exp_id: int, config: Dict[str, Any], seed: int,
                 job_id: str) -> None:
        self.master = master
        self.id = exp_id
        self.config = config
        self.seed = seed
        self.job_id = job_id
        self.state = ACTIVE
        self.trials: Dict[str, Trial] = {}
        self.searcher = Searcher(seed, make_search_method(config["searcher"]), config["hyperparameters"])
        self.lock = threading.RLock()
        self.best_metric: Optional[float] = None
        self.shutdown = False
        res = config.get("resources") or {}
        self.slots_per_trial = int(res.get("slots_per_trial", 1))
        self.priority = int(res["priority"]) if res.get("priority") is not None else 42
        self.weight = float(res.get("weight") or 1.0)
        self.pool = res.get("resource_pool") or "default"
        self.max_slots = res.get("max_slots")
        self.created_at = time.time()  # job submission time (fair-share group age)
        self.smaller_is_better = bool(config["searcher"].get("smaller_is_better", True))

    # ------------------------------------------------------------------ searcher plumbing
    def start(self) -> None:
        with self.lock:
            self._process(self.searcher.initial_operations())
            self._persist()

    def _process(self, ops: List[Any]) -> None:
        for op in ops:
            if isinstance(op, Create):
                self._create_trial(op)
            elif isinstance(op, ValidateAfter):
                t = self.trials.get(op.request_id)
                if t is None:
                    continue
                t.op = op
                t.op_complete = False
                self._ensure_running(t)
            elif isinstance(op, Close):
                t = self.trials.get(op.request_id)
                if t is None:
                    continue
                t.closed = True
                if t.allocation_id is None and t.op_complete:
                    self._trial_closed(t)
            elif isinstance(op, Shutdown):
                self.shutdown = True
                if op.failure:
                    self._set_state(STOPPING_ERROR)
                elif op.cancel:
                    self._set_state(STOPPING_CANCELED)
                elif self.state in (ACTIVE, PAUSED):
                    self._set_state(STOPPING_COMPLETED)
        self._maybe_finish()

    def _create_trial(self, op: Create) -> None:
        seed = int(self.searcher.rng.randint(0, 2 ** 31 - 1))
        tid = self.master.db.insert("trials", {
            "experiment_id": self.id, "request_id": op.request_id, "hparams": op.hparams,
            "state": ACTIVE, "start_time": now(), "seed": seed,
            "task_id": f"{self.id}.{op.request_id}"})
        t = Trial(self, tid, op.request_id, op.hparams, seed)
        if op.checkpoint:
            t.latest_checkpoint = op.checkpoint
        self.trials[op.request_id] = t
        self._process(self.searcher.trial_created(op.request_id))

    # ------------------------------------------------------------------ unmanaged trials
    def add_unmanaged_trial(self, hparams: Optional[Dict[str, Any]] = None,
                            external_id: Optional[str] = None) -> Trial:
        """A trial whose process runs outside the cluster (Core API v2 ``unmanaged`` mode): no
        searcher operation and no allocation; it reports metrics / checkpoints / heartbeats
        itself. ``external_id`` makes the call idempotent (resume of the same external trial)."""
        with self.lock:
            if external_id is not None:
                row = self.master.db.one("SELECT request_id FROM trials WHERE experiment_id=? AND "
                                         "external_trial_id=?", [self.id, str(external_id)])
                if row is not None and row["request_id"] in self.trials:
                    return self.trials[row["request_id"]]
            rid = str(uuid.uuid4())
            tid = self.master.db.insert("trials", {
                "experiment_id": self.id, "request_id": rid, "hparams": hparams or {},
                "state": ACTIVE, "start_time": now(), "seed": 0, "task_id": f"{self.id}.{rid}",
                "external_trial_id": None if external_id is None else str(external_id)})
            t = Trial(self, tid, rid, hparams or {}, 0)
            self.trials[rid] = t
            return t

    def unmanaged_heartbeat(self, t: Trial, state: str) -> None:
        """RUNNING keeps the trial alive; COMPLETED / ERROR / CANCELED end it, and the
        experiment ends with its last trial."""
        with self.lock:
            if state not in TERMINAL or t.state in TERMINAL:
                return
            t.state = state
            self.master.db.update("trials", "id", t.id, {"state": state, "end_time": now()})
            if all(x.state in TERMINAL for x in self.trials.values()):
                final = COMPLETED if all(x.state == COMPLETED for x in self.trials.values()) else ERROR
                self._set_state(final)
                self.master.db.update("experiments", "id", self.id, {"end_time": now()})

    def _ensure_running(self, t: Trial) -> None:
        if self.state != ACTIVE or t.allocation_id is not None or t.state in TERMINAL:
            return
        if t.op_complete:
            return
        alloc_id = f"{t.task_id}.{t.run_id}"
        t.allocation_id = alloc_id
        t.allocation_state = "PENDING"
        t.preempt_event = threading.Event()
        req = AllocationRequest(alloc_id, t.task_id, self.job_id, self.slots_per_trial,
                                self.priority, self.weight, self.pool, True,
                                name=f"Trial {t.id} (Experiment {self.id})")
        req.max_slots = int(self.max_slots) if self.max_slots is not None else -1
        req.job_submit_time = self.created_at
        # HPC launcher options (expconf `slurm` / `pbs`: slots_per_node, gpu_type, sbatch_args)
        req.hpc = {"slurm": self.config.get("slurm") or {}, "pbs": self.config.get("pbs") or {}}
        self.master.db.upsert("allocations", {"allocation_id": alloc_id, "task_id": t.task_id,
                                              "slots": self.slots_per_trial, "resource_pool": self.pool,
                                              "state": "PENDING", "start_time": now()})
        self.master.register_allocation(alloc_id, self, t)
        self.master.rm.allocate(req)

    # ------------------------------------------------------------------ events from trials
    def validation_completed(self, t: Trial, length: int, metric: Any) -> None:
        with self.lock:
            if t.op is None or t.op.length != length:
                raise ValueError(f"trial {t.id} completed op length {length} but current op is {t.op}")
            op = t.op
            t.op_complete = True
            if isinstance(metric, (int, float)):
                better = self.best_metric is None or (metric < self.best_metric if self.smaller_is_better
                                                      else metric > self.best_metric)
                if better:
                    self.best_metric = float(metric)
            self._process(self.searcher.validation_completed(t.request_id, metric, op))
            self._persist()

    def progress(self, t: Trial, units: float) -> None:
        with self.lock:
            self.searcher.set_trial_progress(t.request_id, units)
            self.master.db.update("trials", "id", t.id, {"progress": units})
            self.master.db.update("experiments", "id", self.id, {"progress": self.searcher.progress()})

    def early_exit(self, t: Trial, reason: str) -> None:
        with self.lock:
            r = ExitedReason.INVALID_HP if "INVALID_HP" in reason else ExitedReason.USER_CANCELED \
                if "USER" in reason else ExitedReason.ERRORED
            t.exited_early = True
            self._process(self.searcher.trial_exited_early(t.request_id, r))
            self._persist()

    def allocation_exited(self, t: Trial, exit_code: int, reason: str = "") -> None:
        """The trial's processes are gone (clean exit, crash, preemption, kill)."""
        with self.lock:
            t.allocation_id = None
            t.allocation_state = None
            t.run_id += 1
            self.master.db.update("trials", "id", t.id, {"run_id": t.run_id})
            if t.killed or self.state in (STOPPING_CANCELED, STOPPING_ERROR):
                self._end_trial(t, CANCELED if self.state != STOPPING_ERROR else ERROR)
                if not t.closed:
                    self._process(self.searcher.trial_exited_early(t.request_id, ExitedReason.USER_CANCELED))
            elif exit_code != 0 and not t.exited_early:
                t.restarts += 1
                self.master.db.update("trials", "id", t.id, {"restarts": t.restarts})
                if t.restarts > int(self.config.get("max_restarts", 5)):
                    self._end_trial(t, ERROR)
                    self._process(self.searcher.trial_exited_early(t.request_id, ExitedReason.ERRORED))
                elif self.state == ACTIVE:
                    self._ensure_running(t)
            elif t.exited_early:
                self._end_trial(t, COMPLETED if t.closed else ERROR)
                if t.closed and not self.searcher.trial_is_closed(t.request_id):
                    self._process(self.searcher.trial_closed(t.request_id))
            else:
                if t.closed and t.op_complete:
                    self._trial_closed(t)
                elif not t.op_complete and self.state == ACTIVE:
                    self._ensure_running(t)  # preempted / stopped early: resume
            self._maybe_finish()
            self._persist()

    def _trial_closed(self, t: Trial) -> None:
        self._end_trial(t, COMPLETED)
        if not self.searcher.trial_is_closed(t.request_id):
            self._process(self.searcher.trial_closed(t.request_id))

    def _end_trial(self, t: Trial, state: str) -> None:
        if t.state in TERMINAL:
            return
        t.state = state
        self.master.db.update("trials", "id", t.id, {"state": state, "end_time": now()})
        self.master.checkpoint_gc_trial(self, t)

    # ------------------------------------------------------------------ user actions
    def _set_state(self, state: str) -> None:
        if state != self.state:
            logger.info(f"experiment {self.id}: {self.state} -> {state}")
        self.state = state
        self.master.db.update("experiments", "id", self.id, {"state": state})
        self.master.webhooks.experiment_state_changed(self, state)

    def pause(self) -> None:
        with self.lock:
            if self.state != ACTIVE:
                return
            self._set_state(PAUSED)
            for t in self.trials.values():
                if t.allocation_id is not None:
                    self.master.preempt_allocation(t.allocation_id)

    def activate(self) -> None:
        with self.lock:
            if self.state != PAUSED:
                return
            self._set_state(ACTIVE)
            for t in self.trials.values():
                self._ensure_running(t)

    def cancel(self, kill: bool = False) -> None:
        with self.lock:
            if self.state in TERMINAL:
                return
            self._set_state(STOPPING_CANCELED)
            for t in self.trials.values():
                if t.allocation_id is not None:
                    if kill:
                        t.killed = True
                        self.master.kill_allocation(t.allocation_id)
                    else:
                        self.master.preempt_allocation(t.allocation_id)
                elif t.state not in TERMINAL:
                    self._end_trial(t, CANCELED)
            self._maybe_finish()

    def continue_with(self, cfg: Dict[str, Any]) -> None:
        """ContinueExperiment (reference: ``api_experiment.go`` ContinueExperiment,
        ``e2e_tests/tests/cluster/test_exp_continue.py``): re-open a terminal single-trial
        experiment (COMPLETED, CANCELED or ERROR) with a merged config -- new constant
        hyperparameters, a longer ``searcher.max_length`` -- and resume its trial from its latest
        checkpoint under a fresh searcher whose operations are re-keyed to the existing trial."""
        with self.lock:
            if self.state not in TERMINAL:
                raise ValueError("only a terminal experiment can be continued")
            if len(self.trials) != 1 or cfg["searcher"]["name"] != "single":
                raise ValueError("only single-trial (searcher: single) experiments can be continued")
            (t,) = self.trials.values()
            self.config = cfg
            self.searcher = Searcher(self.seed, make_search_method(cfg["searcher"]), cfg["hyperparameters"])
            self.smaller_is_better = bool(cfg["searcher"].get("smaller_is_better", True))
            ops = self.searcher.initial_operations()
            for op in ops:
                if isinstance(op, Create):
                    t.hparams = op.hparams
                op.request_id = t.request_id
            ops = [op for op in ops if not isinstance(op, Create)]
            ops += self.searcher.trial_created(t.request_id)
            self.shutdown = False
            t.state, t.closed, t.op, t.op_complete = ACTIVE, False, None, True
            t.killed, t.exited_early, t.restarts = False, False, 0
            self.master.db.update("trials", "id", t.id, {"state": ACTIVE, "end_time": None, "restarts": 0,
                                                         "hparams": t.hparams})
            self.master.db.update("experiments", "id", self.id, {"config": cfg, "end_time": None})
            self._set_state(ACTIVE)
            self._process(ops)
            self._persist()

    def kill_trial(self, t: Trial) -> None:
        with self.lock:
            t.killed = True
            if t.allocation_id is not None:
                self.master.kill_allocation(t.allocation_id)
            else:
                self._end_trial(t, CANCELED)
                self._process(self.searcher.trial_exited_early(t.request_id, ExitedReason.USER_CANCELED))

    def _maybe_finish(self) -> None:
        active = [t for t in self.trials.values() if t.allocation_id is not None]
        if self.state == STOPPING_COMPLETED and not active:
            for t in self.trials.values():
                if t.state not in TERMINAL:
                    self._end_trial(t, COMPLETED)
            self._finish(COMPLETED)
        elif self.state == STOPPING_CANCELED and not active:
            for t in self.trials.values():
                if t.state not in TERMINAL:
                    self._end_trial(t, CANCELED)
            self._finish(CANCELED)
        elif self.state == STOPPING_ERROR and not active:
            for t in self.trials.values():
                if t.state not in TERMINAL:
                    self._end_trial(t, ERROR)
            self._finish(ERROR)

    def _finish(self, state: str) -> None:
        if self.state in TERMINAL:
            return
        self._set_state(state)
        self.master.db.update("experiments", "id", self.id, {"end_time": now(), "progress": 1.0 if state == COMPLETED else self.searcher.progress()})
        self.master.checkpoint_gc_experiment(self)
        self._persist()

    def _persist(self) -> None:
        trial_states = {rid: {"op": (t.op.to_dict() if t.op else None), "op_complete": t.op_complete,
                              "closed": t.closed, "restarts": t.restarts, "run_id": t.run_id,
                              "state": t.state, "id": t.id, "killed": t.killed,
                              "latest_checkpoint": t.latest_checkpoint,
                              "steps_completed": t.steps_completed, "exited_early": t.exited_early}
                        for rid, t in self.trials.items()}
        snap = {"searcher": self.searcher.snapshot(), "trials": trial_states,
                "best_metric": self.best_metric, "shutdown": self.shutdown}
        self.master.db.update("experiments", "id", self.id, {"searcher_snapshot": json.dumps(snap),
                                                             "progress": self.searcher.progress()})

    def restore(self, snap: Dict[str, Any]) -> None:
        """Rebuild in-memory state after a master restart (reference: restore.go)."""
        self.searcher.restore(snap["searcher"])
        self.best_metric = snap.get("best_metric")
        self.shutdown = snap.get("shutdown", False)
        for rid, st in snap["trials"].items():
            row = self.master.db.one("SELECT * FROM trials WHERE id=?", [st["id"]]) or {}
            t = Trial(self, st["id"], rid, dec(row.get("hparams"), {}), row.get("seed") or 0)
            t.op = ValidateAfter(**{k: v for k, v in st["op"].items() if k != "kind"}) if st["op"] else None
            t.op_complete = st["op_complete"]
            t.closed = st["closed"]
            t.restarts = st["restarts"]
            t.run_id = st["run_id"] + 1
            t.state = st["state"]
            t.killed = st.get("killed", False)
            t.latest_checkpoint = row.get("latest_checkpoint") or st.get("latest_checkpoint")
            t.steps_completed = row.get("steps_completed") or st.get("steps_completed", 0)
            t.exited_early = st.get("exited_early", False)
            self.trials[rid] = t
        if self.state == ACTIVE:
            for t in self.trials.values():
                self._ensure_running(t)
        self._maybe_finish()

    def to_dict(self) -> Dict[str, Any]:
        row = self.master.db.one("SELECT * FROM experiments WHERE id=?", [self.id]) or {}
        return experiment_row_to_api(row, self)


def experiment_row_to_api(row: Dict[str, Any], e: Optional[Experiment] = None) -> Dict[str, Any]:
    cfg = dec(row.get("config"), {}) or {}
    return {
        "id": row.get("id"), "name": cfg.get("name"), "description": cfg.get("description"),
        "state": e.state if e else row.get("state"), "progress": row.get("progress"),
        "start_time": row.get("start_time"), "end_time": row.get("end_time"),
        "archived": bool(row.get("archived")), "labels": cfg.get("labels", []),
        "config": cfg, "parent_id": row.get("parent_id"), "project_id": row.get("project_id"),
        "job_id": row.get("job_id"), "searcher_type": (cfg.get("searcher") or {}).get("name"),
        "resource_pool": (cfg.get("resources") or {}).get("resource_pool") or "default",
        "notes": row.get("notes"), "unmanaged": bool(row.get("unmanaged")),
        "num_trials": None,
    }
