"""Search methods (reference: `master/pkg/searcher/*.go`): single, random, grid, ASHA (promotion
and stop-once variants), adaptive ASHA (brackets in a tournament) and custom.

A search method reacts to trial events with *operations*:
  Create(request_id, hparams)    start a trial
  ValidateAfter(request_id, n)   train the trial to n units (ABSOLUTE) then validate
  Close(request_id)              the trial is done
  Shutdown()                     the search is over
State is JSON-serialisable (``snapshot``/``restore``) so the master can persist and resume it.
"""
import copy
import math
import uuid
from bisect import bisect_left, bisect_right
from typing import Any, Dict, List, Optional

import numpy as np

from determined_clone_amd.searcher import hparams as hp_mod

ASHA_EXITED_METRIC = float(np.finfo(np.float64).max)


# --------------------------------------------------------------------------- operations
class Operation:
    kind = ""

    def to_dict(self) -> Dict[str, Any]:
        d = dict(self.__dict__)
        d["kind"] = self.kind
        return d

    def __eq__(self, other: Any) -> bool:
        return type(self) is type(other) and self.__dict__ == other.__dict__

    def __repr__(self) -> str:
        return f"{self.kind}({self.__dict__})"


class Create(Operation):
    kind = "Create"

    def __init__(self, request_id: str, hparams: Dict[str, Any], checkpoint: Optional[str] = None) -> None:
        self.request_id = request_id
        self.hparams = hparams
        self.checkpoint = checkpoint


class ValidateAfter(Operation):
    kind = "ValidateAfter"

    def __init__(self, request_id: str, length: int) -> None:
        self.request_id = request_id
        self.length = int(length)


class Close(Operation):
    kind = "Close"

    def __init__(self, request_id: str) -> None:
        self.request_id = request_id


class Shutdown(Operation):
    kind = "Shutdown"

    def __init__(self, failure: bool = False, cancel: bool = False) -> None:
        self.failure = failure
        self.cancel = cancel


def op_from_dict(d: Dict[str, Any]) -> Operation:
    d = dict(d)
    kind = d.pop("kind")
    return {"Create": Create, "ValidateAfter": ValidateAfter, "Close": Close, "Shutdown": Shutdown}[kind](**d)


class Context:
    def __init__(self, rng: np.random.RandomState, hparams: Dict[str, Any]) -> None:
        self.rng = rng
        self.hparams = hparams

    def new_request_id(self) -> str:
        return str(uuid.UUID(bytes=self.rng.bytes(16), version=4))

    def create(self, params: Optional[Dict[str, Any]] = None) -> Create:
        if params is None:
            params = hp_mod.sample_all(self.hparams, self.rng)
        return Create(self.new_request_id(), params)


class ExitedReason:
    ERRORED = "ERRORED"
    USER_CANCELED = "USER_CANCELED"
    INVALID_HP = "INVALID_HP"
    INIT_INVALID_HP = "INIT_INVALID_HP"
    USER_REQUESTED_STOP = "USER_REQUESTED_STOP"  # model.UserRequestedStop (early exit from code)


# --------------------------------------------------------------------------- base
class SearchMethod:
    method_type = ""

    def initial_operations(self, ctx: Context) -> List[Operation]:
        raise NotImplementedError

    def trial_created(self, ctx: Context, rid: str) -> List[Operation]:
        return []

    def validation_completed(self, ctx: Context, rid: str, metric: Any, op: ValidateAfter) -> List[Operation]:
        return []

    def trial_closed(self, ctx: Context, rid: str) -> List[Operation]:
        return []

    def trial_exited_early(self, ctx: Context, rid: str, reason: str) -> List[Operation]:
        return [Shutdown(failure=True)]

    def progress(self, trial_progress: Dict[str, float], closed: Dict[str, bool]) -> float:
        raise NotImplementedError

    def snapshot(self) -> Dict[str, Any]:
        return copy.deepcopy(self.state)

    def restore(self, state: Dict[str, Any]) -> None:
        self.state = copy.deepcopy(state)


# --------------------------------------------------------------------------- random / single
class RandomSearch(SearchMethod):
    def __init__(self, max_trials: int, max_length: int, max_concurrent_trials: int = 16,
                 method_type: str = "random") -> None:
        self.max_trials = max_trials
        self.max_length = max_length
        self.max_concurrent_trials = max_concurrent_trials
        self.method_type = method_type
        self.state = {"created_trials": 0, "pending_trials": 0}

    def _new(self, ctx: Context) -> List[Operation]:
        c = ctx.create()
        self.state["created_trials"] += 1
        self.state["pending_trials"] += 1
        return [c, ValidateAfter(c.request_id, self.max_length), Close(c.request_id)]

    def initial_operations(self, ctx: Context) -> List[Operation]:
        n = self.max_trials
        if self.max_concurrent_trials > 0:
            n = min(n, self.max_concurrent_trials)
        ops: List[Operation] = []
        for _ in range(n):
            ops += self._new(ctx)
        return ops

    def trial_exited_early(self, ctx: Context, rid: str, reason: str) -> List[Operation]:
        self.state["pending_trials"] -= 1
        if self.method_type == "random" and reason in (ExitedReason.INVALID_HP, ExitedReason.INIT_INVALID_HP):
            self.state["created_trials"] -= 1  # replaced when its close arrives
        return []

    def trial_closed(self, ctx: Context, rid: str) -> List[Operation]:
        self.state["pending_trials"] -= 1
        if self.state["created_trials"] < self.max_trials:
            return self._new(ctx)
        return []

    def progress(self, trial_progress: Dict[str, float], closed: Dict[str, bool]) -> float:
        done = 0.0
        for k, v in trial_progress.items():
            done += self.max_length if closed.get(k) else v
        return done / float(self.max_length * self.max_trials)


def SingleSearch(max_length: int) -> RandomSearch:
    return RandomSearch(1, max_length, 1, method_type="single")


# --------------------------------------------------------------------------- grid
class GridSearch(SearchMethod):
    method_type = "grid"

    def __init__(self, max_length: int, max_concurrent_trials: int = 16) -> None:
        self.max_length = max_length
        self.max_concurrent_trials = max_concurrent_trials
        self.state = {"remaining": [], "pending_trials": 0, "trials": 0}

    def _pop(self, ctx: Context) -> List[Operation]:
        params = self.state["remaining"].pop()
        c = ctx.create(params)
        self.state["pending_trials"] += 1
        return [c, ValidateAfter(c.request_id, self.max_length), Close(c.request_id)]

    def initial_operations(self, ctx: Context) -> List[Operation]:
        g = hp_mod.grid(ctx.hparams)
        self.state["trials"] = len(g)
        self.state["remaining"] = g
        n = len(g)
        if self.max_concurrent_trials > 0:
            n = min(n, self.max_concurrent_trials)
        ops: List[Operation] = []
        for _ in range(n):
            ops += self._pop(ctx)
        return ops

    def trial_exited_early(self, ctx: Context, rid: str, reason: str) -> List[Operation]:
        return []

    def trial_closed(self, ctx: Context, rid: str) -> List[Operation]:
        self.state["pending_trials"] -= 1
        return self._pop(ctx) if self.state["remaining"] else []

    def progress(self, trial_progress: Dict[str, float], closed: Dict[str, bool]) -> float:
        done = sum(self.max_length for _ in closed) + sum(v for k, v in trial_progress.items() if not closed.get(k))
        return done / float(self.max_length * max(self.state["trials"], 1))


# --------------------------------------------------------------------------- ASHA
def _rung_units(max_length: int, num_rungs: int, divisor: float) -> List[int]:
    units, total = [], 0
    for i in range(num_rungs):
        rate = divisor ** (num_rungs - i - 1)
        total += max(int(max_length / rate), 1)
        units.append(total)
    return units


class AsyncHalvingSearch(SearchMethod):
    """Promotion-based asynchronous successive halving (`asha.go`)."""

    method_type = "asha"

    def __init__(self, num_rungs: int, max_length: int, max_trials: int, divisor: float = 4,
                 max_concurrent_trials: int = 0, smaller_is_better: bool = True) -> None:
        self.num_rungs = num_rungs
        self.max_length = max_length
        self.max_trials = max_trials
        self.divisor = float(divisor)
        self.max_concurrent_trials = max_concurrent_trials
        self.smaller_is_better = smaller_is_better
        self.state = {
            "rungs": [{"units_needed": u, "metrics": [], "outstanding_trials": 0}
                      for u in _rung_units(max_length, num_rungs, self.divisor)],
            "trial_rungs": {}, "early_exit_trials": {}, "closed_trials": {},
            "trials_completed": 0, "invalid_trials": 0, "pending_trials": 0,
        }

    # helpers
    def _rung(self, i: int) -> Dict[str, Any]:
        return self.state["rungs"][i]

    def _initial_n(self) -> int:
        if self.max_concurrent_trials > 0:
            return min(self.max_concurrent_trials, self.max_trials)
        return max(1, min(int(self.divisor ** (self.num_rungs - 1)), self.max_trials))

    def _create(self, ctx: Context) -> List[Operation]:
        c = ctx.create()
        self.state["trial_rungs"][c.request_id] = 0
        self.state["pending_trials"] += 1
        return [c, ValidateAfter(c.request_id, self._rung(0)["units_needed"])]

    def initial_operations(self, ctx: Context) -> List[Operation]:
        ops: List[Operation] = []
        for _ in range(self._initial_n()):
            ops += self._create(ctx)
        return ops

    def trial_created(self, ctx: Context, rid: str) -> List[Operation]:
        self._rung(0)["outstanding_trials"] += 1
        self.state["trial_rungs"][rid] = 0
        return []

    def trial_closed(self, ctx: Context, rid: str) -> List[Operation]:
        self.state["trials_completed"] += 1
        self.state["closed_trials"][rid] = True
        return []

    def validation_completed(self, ctx: Context, rid: str, metric: Any, op: ValidateAfter) -> List[Operation]:
        self.state["pending_trials"] -= 1
        if not isinstance(metric, (int, float)):
            raise TypeError(f"unexpected metric type for ASHA: {metric!r}")
        value = float(metric) if self.smaller_is_better else -float(metric)
        return self._promote(ctx, rid, value)

    @staticmethod
    def _promotions(rung: Dict[str, Any], rid: str, metric: float, divisor: float) -> List[str]:
        ms = rung["metrics"]
        old_np = int(len(ms) / divisor)
        new_np = int((len(ms) + 1) / divisor)
        keys = [m["metric"] for m in ms]
        idx = bisect_right(keys, metric)
        promote_now = idx < new_np
        ms.insert(idx, {"request_id": rid, "metric": metric, "promoted": promote_now})
        if promote_now:
            return [rid]
        if new_np != old_np and not ms[old_np]["promoted"]:
            ms[old_np]["promoted"] = True
            return [ms[old_np]["request_id"]]
        return []

    def _promote(self, ctx: Context, rid: str, metric: float) -> List[Operation]:
        st = self.state
        ri = st["trial_rungs"][rid]
        rung = self._rung(ri)
        rung["outstanding_trials"] -= 1
        added = False
        ops: List[Operation] = []
        if ri == self.num_rungs - 1:
            rung["metrics"].append({"request_id": rid, "metric": metric, "promoted": False})
            if not st["early_exit_trials"].get(rid):
                ops.append(Close(rid))
                st["closed_trials"][rid] = True
        else:
            nxt = self._rung(ri + 1)
            for pid in self._promotions(rung, rid, metric, self.divisor):
                st["trial_rungs"][pid] = ri + 1
                nxt["outstanding_trials"] += 1
                if not st["early_exit_trials"].get(pid):
                    ops.append(ValidateAfter(pid, max(nxt["units_needed"] - rung["units_needed"], 1)))
                    added = True
                    st["pending_trials"] += 1
                else:
                    return self._promote(ctx, pid, ASHA_EXITED_METRIC)
        all_trials = len(st["trial_rungs"]) - st["invalid_trials"]
        if not added and all_trials < self.max_trials:
            ops += self._create(ctx)
        if len(self._rung(0)["metrics"]) == self.max_trials:
            ops += self._close_out_rungs()
        return ops

    def _close_out_rungs(self) -> List[Operation]:
        ops: List[Operation] = []
        st = self.state
        for rung in st["rungs"]:
            if rung["outstanding_trials"] > 0:
                break
            for m in rung["metrics"]:
                r = m["request_id"]
                if not m["promoted"] and not st["closed_trials"].get(r) and not st["early_exit_trials"].get(r):
                    ops.append(Close(r))
                    st["closed_trials"][r] = True
        return ops

    def progress(self, trial_progress: Dict[str, float], closed: Dict[str, bool]) -> float:
        st = self.state
        if self.max_concurrent_trials > 0 and st["pending_trials"] > self.max_concurrent_trials:
            raise RuntimeError("pending trials is greater than max_concurrent_trials")
        n = len(self._rung(0)["metrics"])
        prog = n / (1.2 * self.max_trials)
        if n == self.max_trials:
            prog = max(prog, (st["trials_completed"] - st["invalid_trials"]) / float(self.max_trials))
        return prog

    def trial_exited_early(self, ctx: Context, rid: str, reason: str) -> List[Operation]:
        st = self.state
        st["pending_trials"] -= 1
        if reason in (ExitedReason.INVALID_HP, ExitedReason.INIT_INVALID_HP):
            st["early_exit_trials"][rid] = True
            st["closed_trials"][rid] = True
            st["invalid_trials"] += 1
            hi = st["trial_rungs"][rid]
            self._rung(hi)["outstanding_trials"] -= 1
            for i in range(hi + 1):
                ms = self._rung(i)["metrics"]
                for j, m in enumerate(ms):
                    if m["request_id"] == rid:
                        del ms[j]
                        break
            return [Close(rid)] + self._create(ctx)
        st["early_exit_trials"][rid] = True
        st["closed_trials"][rid] = True
        return self._promote(ctx, rid, ASHA_EXITED_METRIC)


class AsyncHalvingStoppingSearch(AsyncHalvingSearch):
    """ASHA with ``stop_once``: a trial is either continued or stopped at each rung, never resumed
    (`asha_stopping.go`)."""

    def validation_completed(self, ctx: Context, rid: str, metric: Any, op: ValidateAfter) -> List[Operation]:
        if not isinstance(metric, (int, float)):
            raise TypeError(f"unexpected metric type for ASHA: {metric!r}")
        value = float(metric) if self.smaller_is_better else -float(metric)
        return self._promote(ctx, rid, value)

    def _create(self, ctx: Context) -> List[Operation]:
        c = ctx.create()
        self.state["trial_rungs"][c.request_id] = 0
        return [c, ValidateAfter(c.request_id, self._rung(0)["units_needed"])]

    @staticmethod
    def _continue(rung: Dict[str, Any], rid: str, metric: float, divisor: float) -> bool:
        ms = rung["metrics"]
        num_promote = max(int((len(ms) + 1) / divisor), 1)
        keys = [m["metric"] for m in ms]
        idx = bisect_left(keys, metric)
        promote = idx < num_promote
        ms.insert(idx, {"request_id": rid, "metric": metric, "promoted": promote})
        return promote

    def _promote(self, ctx: Context, rid: str, metric: float) -> List[Operation]:
        st = self.state
        ri = st["trial_rungs"][rid]
        rung = self._rung(ri)
        rung["outstanding_trials"] -= 1
        added = False
        ops: List[Operation] = []
        if ri == self.num_rungs - 1:
            rung["metrics"].append({"request_id": rid, "metric": metric, "promoted": False})
            if not st["early_exit_trials"].get(rid):
                ops.append(Close(rid))
                st["closed_trials"][rid] = True
        else:
            nxt = self._rung(ri + 1)
            promote = self._continue(rung, rid, metric, self.divisor)
            if not st["early_exit_trials"].get(rid):
                if promote:
                    st["trial_rungs"][rid] = ri + 1
                    nxt["outstanding_trials"] += 1
                    ops.append(ValidateAfter(rid, max(nxt["units_needed"] - rung["units_needed"], 1)))
                    added = True
                else:
                    ops.append(Close(rid))
                    st["closed_trials"][rid] = True
        if not added and len(st["trial_rungs"]) - st["invalid_trials"] < self.max_trials:
            ops += self._create(ctx)
        return ops

    def progress(self, trial_progress: Dict[str, float], closed: Dict[str, bool]) -> float:
        st = self.state
        n = len(self._rung(0)["metrics"])
        prog = n / (1.2 * self.max_trials)
        if n == self.max_trials:
            prog = max(prog, (st["trials_completed"] - st["invalid_trials"]) / float(self.max_trials))
        return prog

    def trial_exited_early(self, ctx: Context, rid: str, reason: str) -> List[Operation]:
        st = self.state
        if reason in (ExitedReason.INVALID_HP, ExitedReason.INIT_INVALID_HP):
            st["early_exit_trials"][rid] = True
            st["closed_trials"][rid] = True
            st["invalid_trials"] += 1
            hi = st["trial_rungs"][rid]
            for i in range(hi + 1):
                ms = self._rung(i)["metrics"]
                for j, m in enumerate(ms):
                    if m["request_id"] == rid:
                        del ms[j]
                        break
            return [Close(rid)] + self._create(ctx)
        st["early_exit_trials"][rid] = True
        st["closed_trials"][rid] = True
        return self._promote(ctx, rid, ASHA_EXITED_METRIC)


# --------------------------------------------------------------------------- tournament / adaptive
class TournamentSearch(SearchMethod):
    def __init__(self, method_type: str, subs: List[SearchMethod]) -> None:
        self.method_type = method_type
        self.subs = subs
        self.state = {"trial_table": {}}

    def _mark(self, i: int, ops: List[Operation]) -> List[Operation]:
        for op in ops:
            if isinstance(op, Create):
                self.state["trial_table"][op.request_id] = i
        return ops

    def initial_operations(self, ctx: Context) -> List[Operation]:
        ops: List[Operation] = []
        for i, s in enumerate(self.subs):
            ops += self._mark(i, s.initial_operations(ctx))
        return ops

    def _route(self, rid: str) -> int:
        return self.state["trial_table"][rid]

    def trial_created(self, ctx: Context, rid: str) -> List[Operation]:
        i = self._route(rid)
        return self._mark(i, self.subs[i].trial_created(ctx, rid))

    def validation_completed(self, ctx: Context, rid: str, metric: Any, op: ValidateAfter) -> List[Operation]:
        i = self._route(rid)
        return self._mark(i, self.subs[i].validation_completed(ctx, rid, metric, op))

    def trial_closed(self, ctx: Context, rid: str) -> List[Operation]:
        i = self._route(rid)
        return self._mark(i, self.subs[i].trial_closed(ctx, rid))

    def trial_exited_early(self, ctx: Context, rid: str, reason: str) -> List[Operation]:
        i = self._route(rid)
        return self._mark(i, self.subs[i].trial_exited_early(ctx, rid, reason))

    def progress(self, trial_progress: Dict[str, float], closed: Dict[str, bool]) -> float:
        tot = 0.0
        for i, s in enumerate(self.subs):
            tp = {k: v for k, v in trial_progress.items() if self.state["trial_table"].get(k) == i}
            cl = {k: v for k, v in closed.items() if self.state["trial_table"].get(k) == i}
            tot += s.progress(tp, cl)
        return tot / len(self.subs)

    def snapshot(self) -> Dict[str, Any]:
        return {"trial_table": dict(self.state["trial_table"]), "subs": [s.snapshot() for s in self.subs]}

    def restore(self, state: Dict[str, Any]) -> None:
        self.state = {"trial_table": dict(state["trial_table"])}
        for s, st in zip(self.subs, state["subs"]):
            s.restore(st)


def bracket_max_trials(max_trials: int, divisor: float, brackets: List[int]) -> List[int]:
    weights = [divisor ** (r - 1) / r for r in brackets]
    total = sum(weights)
    out = [max(int(w / total * max_trials), 1) for w in weights]
    out[0] += max(max_trials - sum(out), 0)
    return out


def bracket_max_concurrent(max_concurrent: int, divisor: float, max_trials: List[int]) -> List[int]:
    nb = len(max_trials)
    if max_concurrent == 0:
        base, rem = max(max_trials[-1], int(divisor)), 0
    else:
        max_concurrent = max(max_concurrent, nb)
        base, rem = max_concurrent // nb, max_concurrent % nb
    out = [base] * nb
    for i in range(rem):
        out[i] += 1
    return out


def adaptive_bracket_rungs(mode: str, max_rungs: int) -> List[int]:
    if mode == "conservative":
        return list(range(1, max_rungs + 1))
    if mode == "standard":
        return list(range((max_rungs - 1) // 2 + 1, max_rungs + 1))
    if mode == "aggressive":
        return [max_rungs]
    raise ValueError(f"unexpected adaptive mode: {mode}")


def AdaptiveASHASearch(max_length: int, max_trials: int, mode: str = "standard", divisor: float = 4,
                       max_rungs: int = 5, max_concurrent_trials: int = 16,
                       bracket_rungs: Optional[List[int]] = None, stop_once: bool = False,
                       smaller_is_better: bool = True) -> TournamentSearch:
    brackets = list(bracket_rungs or [])
    if not brackets:
        mr = min(max_rungs, int(math.log(max_length) / math.log(divisor)) + 1,
                 int(math.log(max_trials) / math.log(divisor)) + 1)
        brackets = adaptive_bracket_rungs(mode, mr)
    brackets.sort(reverse=True)
    mts = bracket_max_trials(max_trials, divisor, brackets)
    mcs = bracket_max_concurrent(max_concurrent_trials, divisor, mts)
    cls = AsyncHalvingStoppingSearch if stop_once else AsyncHalvingSearch
    subs: List[SearchMethod] = [cls(r, max_length, mts[i], divisor, mcs[i], smaller_is_better)
                                for i, r in enumerate(brackets)]
    return TournamentSearch("adaptive_asha", subs)


# --------------------------------------------------------------------------- custom
class CustomSearch(SearchMethod):
    """Operations come from a user-side SearchMethod (searcher/custom.py) through the master's
    searcher-event queue; the master-side method only queues events and accepts posted ops."""

    method_type = "custom_search"

    def __init__(self) -> None:
        self.state = {"events": [], "next_event_id": 1, "progress": 0.0}

    def _event(self, kind: str, **payload: Any) -> None:
        self.state["events"].append({"id": self.state["next_event_id"], "type": kind, **payload})
        self.state["next_event_id"] += 1

    def initial_operations(self, ctx: Context) -> List[Operation]:
        self._event("initial_operations")
        return []

    def trial_created(self, ctx: Context, rid: str) -> List[Operation]:
        self._event("trial_created", request_id=rid)
        return []

    def validation_completed(self, ctx: Context, rid: str, metric: Any, op: ValidateAfter) -> List[Operation]:
        self._event("validation_completed", request_id=rid, metric=metric, validate_after_length=op.length)
        return []

    def trial_closed(self, ctx: Context, rid: str) -> List[Operation]:
        self._event("trial_closed", request_id=rid)
        return []

    def trial_exited_early(self, ctx: Context, rid: str, reason: str) -> List[Operation]:
        self._event("trial_exited_early", request_id=rid, exited_reason=reason)
        return []

    def trial_progress(self, rid: str, progress: float) -> None:
        self._event("trial_progress", request_id=rid, partial_units=progress)

    def progress(self, trial_progress: Dict[str, float], closed: Dict[str, bool]) -> float:
        return float(self.state["progress"])

    def events_after(self, last_id: int) -> List[Dict[str, Any]]:
        return [e for e in self.state["events"] if e["id"] > last_id]

    def ack_events(self, up_to: int) -> None:
        self.state["events"] = [e for e in self.state["events"] if e["id"] > up_to]


def make_search_method(searcher_cfg: Dict[str, Any]) -> SearchMethod:
    """expconf ``searcher`` section (completed by config.expconf) -> SearchMethod."""
    name = searcher_cfg["name"]
    ml = searcher_cfg.get("max_length")
    length = int(next(iter(ml.values()))) if isinstance(ml, dict) else (int(ml) if ml else 0)
    sib = bool(searcher_cfg.get("smaller_is_better", True))
    if name == "single":
        return SingleSearch(length)
    if name == "random":
        return RandomSearch(int(searcher_cfg["max_trials"]), length,
                            int(searcher_cfg.get("max_concurrent_trials") or 0))
    if name == "grid":
        return GridSearch(length, int(searcher_cfg.get("max_concurrent_trials") or 0))
    if name in ("async_halving", "asha"):
        cls = AsyncHalvingStoppingSearch if searcher_cfg.get("stop_once") else AsyncHalvingSearch
        return cls(int(searcher_cfg["num_rungs"]), length, int(searcher_cfg["max_trials"]),
                   float(searcher_cfg.get("divisor", 4)),
                   int(searcher_cfg.get("max_concurrent_trials") or 0), sib)
    if name == "adaptive_asha":
        return AdaptiveASHASearch(length, int(searcher_cfg["max_trials"]),
                                  searcher_cfg.get("mode", "standard"),
                                  float(searcher_cfg.get("divisor", 4)),
                                  int(searcher_cfg.get("max_rungs", 5)),
                                  int(searcher_cfg.get("max_concurrent_trials") or 0),
                                  searcher_cfg.get("bracket_rungs") or [],
                                  bool(searcher_cfg.get("stop_once", False)), sib)
    if name == "custom":
        return CustomSearch()
    raise ValueError(f"unknown searcher {name}")
