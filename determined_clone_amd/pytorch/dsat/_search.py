"""DeepSpeed autotuning search methods (reference: `harness/determined/pytorch/dsat/
_dsat_search_method.py`): find the (ZeRO stage, micro batch size) with the best measured
throughput / latency for a DeepSpeedTrial.

Every candidate is a short profiling trial: its hparams carry ``_use_dsat_mode`` plus an
``overwrite_deepspeed_args`` patch (stage, ``train_micro_batch_size_per_gpu``); the
DeepSpeedTrialController then trains ``end_profile_step`` batches, times the steps after
``start_profile_step`` and reports the metric (``throughput`` samples/s, ``latency`` ms/step,
``FLOPS_per_gpu`` when the model exposes ``flops_per_token``). An out-of-memory step ends the trial as
INVALID_HP, which the search treats as "micro batch too large".

* ``binary``: per stage, double the micro batch from 1 until OOM (or ``max_mbs``), then bisect
  between the largest success and the smallest failure.
* ``random``: random (stage, micro batch) pairs from the allowed space, never repeating a pair and
  never trying a micro batch at or above a known OOM for that stage; ``early_stopping`` ends the
  search after that many completed trials without a new best.
* ``_test``: micro batches 1, 2, ... ``max_trials`` over the stages in turn (for testing).

(``asha`` -- lineages of random DeepSpeed configurations, each binary-searching its micro batch, under
successive halving -- is :class:`._asha.ASHADSATSearchMethod`.)
Trials also carry an ``autotuning`` section in their overwrite, so the native engine measures the
profiled steps itself (``pytorch/deepspeed/_autotune.py``) for DeepSpeedTrials and Core API
scripts alike; a metric reported as the engine's dict is read by name.
"""
import json
import pathlib
import uuid
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from determined_clone_amd import searcher
from determined_clone_amd.pytorch.dsat import _defaults


class _Cand:
    def __init__(self, stage: int, mbs: int) -> None:
        self.stage, self.mbs = stage, mbs
        self.metric: Optional[float] = None
        self.oom = False
        self.done = False


class DSATSearchMethod(searcher.SearchMethod):
    def __init__(self, base_hparams: Dict[str, Any], search: str = "binary",
                 metric: str = "throughput", zero_stages: Tuple[int, ...] = (1, 2),
                 max_trials: int = 32, max_concurrent_trials: int = 4,
                 start_profile_step: int = 3, end_profile_step: int = 5, max_mbs: int = 1024,
                 seed: int = 42, early_stopping: Optional[int] = None) -> None:
        if search not in ("binary", "random", "_test"):
            raise ValueError(f"unknown dsat search {search!r}")
        self.early_stopping = early_stopping
        self._since_best = 0
        self._best_val: Optional[float] = None
        self.base = dict(base_hparams)
        self.search = search
        self.metric = metric
        self.smaller_is_better = metric in _defaults.SMALLER_IS_BETTER_METRICS
        self.stages = list(zero_stages)
        self.max_trials, self.max_concurrent = max_trials, max_concurrent_trials
        self.profile = [int(start_profile_step), int(end_profile_step)]
        self.max_mbs = max_mbs
        self.rng = np.random.RandomState(seed)
        self.cands: Dict[str, _Cand] = {}
        # binary-search bounds per stage: [largest ok, smallest oom]
        self.lo = {s: 0 for s in self.stages}
        self.hi = {s: max_mbs + 1 for s in self.stages}
        self.next_double = {s: 1 for s in self.stages}

    # ------------------------------------------------------------------ candidate generation
    def _tried(self, stage: int, mbs: int) -> bool:
        return any(c.stage == stage and c.mbs == mbs for c in self.cands.values())

    def _propose(self) -> Optional[Tuple[int, int]]:
        if self.search == "_test":
            m = len(self.cands) + 1
            return (self.stages[(m - 1) % len(self.stages)], m) if m <= self.max_mbs else None
        if self.search == "random":
            if self.early_stopping is not None and self._since_best >= self.early_stopping:
                return None
            for _ in range(64):
                s = int(self.rng.choice(self.stages))
                cap = min(self.hi[s] - 1, self.max_mbs)
                if cap < 1:
                    continue
                m = int(2 ** self.rng.uniform(0, np.log2(cap))) if cap > 1 else 1
                if not self._tried(s, m):
                    return s, m
            return None
        for s in self.stages:  # binary: stages in order, doubling then bisection
            running = any(c.stage == s and not c.done for c in self.cands.values())
            if running:
                continue
            if self.hi[s] > self.max_mbs and self.next_double[s] <= self.max_mbs:
                m = self.next_double[s]
                self.next_double[s] *= 2
                if not self._tried(s, m):
                    return s, m
                continue
            if self.hi[s] - self.lo[s] > 1:
                m = (self.lo[s] + self.hi[s]) // 2
                if not self._tried(s, m):
                    return s, m
        return None

    def _create(self) -> List[searcher.Operation]:
        ops: List[searcher.Operation] = []
        while len(self.cands) < self.max_trials and \
                sum(not c.done for c in self.cands.values()) < self.max_concurrent:
            p = self._propose()
            if p is None:
                break
            stage, mbs = p
            rid = uuid.uuid4()
            self.cands[str(rid)] = _Cand(stage, mbs)
            hp = dict(self.base)
            ow = dict(hp.get(_defaults.OVERWRITE_KEY) or {})
            ow["train_micro_batch_size_per_gpu"] = mbs
            ow.pop("train_batch_size", None)
            ow["zero_optimization"] = dict(ow.get("zero_optimization") or {}, stage=stage)
            ow["autotuning"] = {"enabled": True, "start_profile_step": self.profile[0],
                                "end_profile_step": self.profile[1]}
            hp[_defaults.OVERWRITE_KEY] = ow
            hp[_defaults.USE_DSAT_MODE_KEY] = True
            hp[_defaults.PROFILE_KEY] = list(self.profile)
            ops += [searcher.Create(rid, hp), searcher.ValidateAfter(rid, self.profile[1])]
        return ops

    # ------------------------------------------------------------------ SearchMethod
    def initial_operations(self, state: searcher.SearcherState) -> List[searcher.Operation]:
        return self._create()

    def on_trial_created(self, state, request_id):
        return []

    def on_validation_completed(self, state, request_id, metric: Any, train_length: int):
        c = self.cands[str(request_id)]
        c.metric = self._value(metric)
        c.done = True
        if c.metric is not None:
            better = self._best_val is None or (c.metric < self._best_val if self.smaller_is_better
                                                else c.metric > self._best_val)
            self._best_val = c.metric if better else self._best_val
            self._since_best = 0 if better else self._since_best + 1
        self.lo[c.stage] = max(self.lo[c.stage], c.mbs)
        return [searcher.Close(request_id)] + self._create() + self._maybe_shutdown()

    def on_trial_exited_early(self, state, request_id, exited_reason):
        c = self.cands.get(str(request_id))
        if c is not None:
            c.done = True
            c.oom = True
            self.hi[c.stage] = min(self.hi[c.stage], c.mbs)
        return self._create() + self._maybe_shutdown()

    def on_trial_closed(self, state, request_id):
        return self._maybe_shutdown()

    def _value(self, metric: Any) -> Optional[float]:
        if isinstance(metric, dict):  # the engine's autotuning measurements
            for name in (self.metric, "latency" if self.smaller_is_better else "throughput"):
                if metric.get(name) is not None:
                    return float(metric[name])
            return None
        return None if metric is None else float(metric)

    def _maybe_shutdown(self) -> List[searcher.Operation]:
        if self.cands and all(c.done for c in self.cands.values()) and self._propose_peek() is None:
            return [searcher.Shutdown()]
        return []

    def _propose_peek(self) -> Optional[Tuple[int, int]]:
        if len(self.cands) >= self.max_trials:
            return None
        saved = (dict(self.next_double), self.rng.get_state())
        p = self._propose()
        self.next_double, st = saved
        self.rng.set_state(st)
        return p

    def progress(self, state):
        return min(1.0, sum(c.done for c in self.cands.values()) / max(1, self.max_trials))

    # ------------------------------------------------------------------ results
    def best(self) -> Optional[Dict[str, Any]]:
        ok = [c for c in self.cands.values() if c.metric is not None]
        if not ok:
            return None
        pick = min if self.smaller_is_better else max
        b = pick(ok, key=lambda c: c.metric)
        return {"zero_stage": b.stage, "train_micro_batch_size_per_gpu": b.mbs, self.metric: b.metric}

    def results(self) -> List[Dict[str, Any]]:
        return [{"zero_stage": c.stage, "mbs": c.mbs, "metric": c.metric, "oom": c.oom}
                for c in self.cands.values()]

    def save_method_state(self, path: pathlib.Path) -> None:
        (path / "dsat_state.json").write_text(json.dumps({
            "cands": {k: vars(v) for k, v in self.cands.items()}, "lo": self.lo, "hi": self.hi,
            "next_double": self.next_double}))

    def load_method_state(self, path: pathlib.Path) -> None:
        d = json.loads((path / "dsat_state.json").read_text())
        self.cands = {}
        for k, v in d["cands"].items():
            c = _Cand(v["stage"], v["mbs"])
            c.metric, c.oom, c.done = v["metric"], v["oom"], v["done"]
            self.cands[k] = c
        self.lo = {int(k): v for k, v in d["lo"].items()}
        self.hi = {int(k): v for k, v in d["hi"].items()}
        self.next_double = {int(k): v for k, v in d["next_double"].items()}
