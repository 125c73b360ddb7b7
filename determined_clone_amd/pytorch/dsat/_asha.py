"""ASHA over DeepSpeed configurations (reference: `harness/determined/pytorch/dsat/
_dsat_search_method.py` ASHADSATSearchMethod; asynchronous successive halving, arxiv:1810.05934).

A *lineage* is one random DeepSpeed configuration -- ZeRO stage plus that stage's knobs (bucket
sizes, overlap / reduce-scatter / contiguous-gradient / partition switches) -- whose micro batch is
binary-searched between 1 and the largest size the model profile says fits. Every profiling trial
of a lineage is one unit of ASHA's resource: rung ``r`` lets a lineage run
``min_binary_search_trials * divisor ** (asha_early_stopping + r)`` trials in total, and only the
best ``1 / divisor`` of the lineages that finished rung ``r`` (ranked by their best measured metric
so far) are promoted to rung ``r + 1``. When no lineage can continue or be promoted, a new random
lineage starts.

The search begins with one model-profile trial (micro batch 1, ``autotuning.model_info``): its
parameter count, activation bytes per sample and device memory bound each ZeRO stage's micro-batch
range through :func:`._utils.approx_max_mbs_per_stage` (MI355X: 288 GB of HBM per GPU, so the ranges
are wide and the binary searches matter). If that trial fails, ranges fall back to ``max_mbs``.

Trials carry ``overwrite_deepspeed_args`` with the configuration and an ``autotuning`` section, so
both DeepSpeedTrials and Core API scripts (through ``dsat_reporting_context``) report the engine's
own measurements.
"""
import json
import pathlib
import random
import uuid
from typing import Any, Dict, List, Optional

from determined_clone_amd import searcher
from determined_clone_amd.pytorch.dsat import _defaults, _utils


class _Lineage:
    def __init__(self, lid: int, stage: int, zero_cfg: Dict[str, Any], lo: int, hi: int) -> None:
        self.lid, self.stage, self.zero_cfg = lid, stage, zero_cfg
        self.lo, self.hi = lo, hi          # micro batches still to search: [lo, hi]
        self.rung = 0
        self.results: List[Dict[str, Any]] = []  # {"mbs", "metric" (None = OOM)}
        self.running = False

    @property
    def exhausted(self) -> bool:
        return self.lo > self.hi

    def next_mbs(self) -> int:
        return (self.lo + self.hi) // 2

    def best(self, smaller_is_better: bool) -> Optional[Dict[str, Any]]:
        ok = [r for r in self.results if r["metric"] is not None]
        if not ok:
            return None
        return (min if smaller_is_better else max)(ok, key=lambda r: r["metric"])

    def to_dict(self) -> Dict[str, Any]:
        return dict(vars(self))


class ASHADSATSearchMethod(searcher.SearchMethod):
    def __init__(self, base_hparams: Dict[str, Any], metric: str = "throughput",
                 zero_stages=(1, 2, 3), max_trials: int = 32, max_concurrent_trials: int = 4,
                 start_profile_step: int = 3, end_profile_step: int = 5, max_mbs: int = 1024,
                 seed: int = 42, divisor: int = 2, min_binary_search_trials: int = 3,
                 max_rungs: int = 5, asha_early_stopping: int = 0, search_range_factor: float = 1.0,
                 slots_per_trial: int = 1, model_info: Optional[Dict[str, Any]] = None) -> None:
        self.base = dict(base_hparams)
        self.metric = metric
        self.smaller_is_better = _utils.smaller_is_better(metric)
        self.stages = [int(s) for s in zero_stages]
        self.max_trials, self.max_concurrent = int(max_trials), int(max_concurrent_trials)
        self.profile = [int(start_profile_step), int(end_profile_step)]
        self.max_mbs = int(max_mbs)
        self.rng = random.Random(seed)
        self.divisor = max(2, int(divisor))
        self.min_bs_trials = max(1, int(min_binary_search_trials))
        self.max_rungs = max(1, int(max_rungs))
        self.early = int(asha_early_stopping)
        self.range_factor = float(search_range_factor)
        self.dp = max(1, int(slots_per_trial))
        self.model_info = model_info
        self.stage_hi: Dict[int, int] = {}
        self.lineages: List[_Lineage] = []
        self.trials: Dict[str, Dict[str, Any]] = {}  # request id -> {"lid", "mbs"} | {"profile"}
        self.created = 0
        if model_info is not None:
            self._set_ranges(model_info)

    # ------------------------------------------------------------------ configuration
    def _set_ranges(self, info: Optional[Dict[str, Any]]) -> None:
        if info:
            caps = _utils.approx_max_mbs_per_stage(info, self.stages, self.dp, self.max_mbs)
        else:
            caps = {s: self.max_mbs for s in self.stages}
        self.stage_hi = {s: max(1, min(self.max_mbs, int(c * self.range_factor))) for s, c in caps.items()}

    def rung_budget(self, rung: int) -> int:
        return self.min_bs_trials * self.divisor ** (self.early + rung)

    def _hparams(self, overwrite: Dict[str, Any]) -> Dict[str, Any]:
        hp = dict(self.base)
        ow = _utils.merge_dicts(hp.get(_defaults.OVERWRITE_KEY) or {}, overwrite)
        ow.pop("train_batch_size", None)  # re-derived from the micro batch and the slots
        hp[_defaults.OVERWRITE_KEY] = ow
        hp[_defaults.USE_DSAT_MODE_KEY] = True
        hp[_defaults.PROFILE_KEY] = list(self.profile)
        return hp

    def _trial_ops(self, key: Dict[str, Any], overwrite: Dict[str, Any], length: int) -> List[searcher.Operation]:
        rid = uuid.uuid4()
        self.trials[str(rid)] = key
        self.created += 1
        return [searcher.Create(rid, self._hparams(overwrite)), searcher.ValidateAfter(rid, length)]

    def _lineage_ops(self, lin: _Lineage) -> List[searcher.Operation]:
        lin.running = True
        mbs = lin.next_mbs()
        ow = {"train_micro_batch_size_per_gpu": mbs, "zero_optimization": dict(lin.zero_cfg),
              "autotuning": {"enabled": True, "start_profile_step": self.profile[0],
                             "end_profile_step": self.profile[1]}}
        return self._trial_ops({"lid": lin.lid, "mbs": mbs}, ow, self.profile[1])

    def _new_lineage(self) -> _Lineage:
        stage = self.rng.choice(self.stages)
        lin = _Lineage(len(self.lineages), stage, _utils.get_random_zero_optim_config(stage, self.rng),
                       1, self.stage_hi.get(stage, self.max_mbs))
        self.lineages.append(lin)
        return lin

    # ------------------------------------------------------------------ ASHA bookkeeping
    def _finished_rung(self, lin: _Lineage, rung: int) -> bool:
        return lin.rung > rung or (lin.rung == rung and not lin.running and
                                   (lin.exhausted or len(lin.results) >= self.rung_budget(rung)))

    def _promotable(self) -> Optional[_Lineage]:
        for rung in reversed(range(self.max_rungs - 1)):
            done = [lin for lin in self.lineages if self._finished_rung(lin, rung)]
            k = len(done) // self.divisor
            if not k:
                continue
            ranked = [lin for lin in done if lin.best(self.smaller_is_better) is not None]
            ranked.sort(key=lambda lin: lin.best(self.smaller_is_better)["metric"],
                        reverse=not self.smaller_is_better)
            for lin in ranked[:k]:
                if lin.rung == rung and not lin.exhausted:
                    return lin
        return None

    def _next_work(self) -> Optional[_Lineage]:
        # 1. a lineage with budget left in its rung (highest rung first, then the longest search)
        open_ = [lin for lin in self.lineages if not lin.running and not lin.exhausted
                 and len(lin.results) < self.rung_budget(lin.rung)]
        if open_:
            return max(open_, key=lambda lin: (lin.rung, len(lin.results)))
        # 2. promote the best unpromoted lineage of the highest possible rung
        lin = self._promotable()
        if lin is not None:
            lin.rung += 1
            return lin
        # 3. a new random configuration
        return self._new_lineage() if self.stage_hi or not self.stages else None

    def _fill(self) -> List[searcher.Operation]:
        ops: List[searcher.Operation] = []
        while self.created < self.max_trials and self._running() < self.max_concurrent:
            lin = self._next_work()
            if lin is None:
                break
            ops += self._lineage_ops(lin)
        if self._running() == 0 and not ops:
            ops.append(searcher.Shutdown())
        return ops

    def _running(self) -> int:
        return sum(lin.running for lin in self.lineages) + sum(
            1 for k in self.trials.values() if k.get("profile") and not k.get("done"))

    def _value(self, metric: Any) -> Optional[float]:
        if isinstance(metric, dict):
            for name in (self.metric, "latency" if self.smaller_is_better else "throughput"):
                if metric.get(name) is not None:
                    return float(metric[name])
            return None
        return None if metric is None else float(metric)

    # ------------------------------------------------------------------ SearchMethod
    def initial_operations(self, state: searcher.SearcherState) -> List[searcher.Operation]:
        if self.model_info is None:
            ow = _utils.merge_dicts(_defaults.MODEL_INFO_PROFILE_DS_CONFIG, {})
            return self._trial_ops({"profile": True}, ow, 1)
        return self._fill()

    def on_trial_created(self, state, request_id):
        return []

    def on_validation_completed(self, state, request_id, metric: Any, train_length: int):
        key = self.trials[str(request_id)]
        ops: List[searcher.Operation] = [searcher.Close(request_id)]
        if key.get("profile"):
            key["done"] = True
            self.model_info = metric if isinstance(metric, dict) else {}
            self._set_ranges(self.model_info)
        else:
            lin = self.lineages[key["lid"]]
            lin.running = False
            lin.results.append({"mbs": key["mbs"], "metric": self._value(metric)})
            lin.lo = key["mbs"] + 1
        return ops + self._fill()

    def on_trial_exited_early(self, state, request_id, exited_reason):
        key = self.trials.get(str(request_id))
        if key is None:
            return self._fill()
        if key.get("profile"):
            key["done"] = True
            self.model_info = {}
            self._set_ranges(None)
        else:
            lin = self.lineages[key["lid"]]
            lin.running = False
            lin.results.append({"mbs": key["mbs"], "metric": None})
            lin.hi = key["mbs"] - 1  # out of memory (InvalidHP) or failed: search below
        return self._fill()

    def on_trial_closed(self, state, request_id):
        return []

    def progress(self, state) -> float:
        return min(1.0, self.created / max(1, self.max_trials))

    # ------------------------------------------------------------------ results
    def best(self) -> Optional[Dict[str, Any]]:
        cands = [(lin, lin.best(self.smaller_is_better)) for lin in self.lineages]
        cands = [(lin, b) for lin, b in cands if b is not None]
        if not cands:
            return None
        lin, b = (min if self.smaller_is_better else max)(cands, key=lambda c: c[1]["metric"])
        return {"zero_stage": lin.stage, "train_micro_batch_size_per_gpu": b["mbs"],
                "zero_optimization": dict(lin.zero_cfg), self.metric: b["metric"]}

    def results(self) -> List[Dict[str, Any]]:
        return [{"lineage": lin.lid, "zero_stage": lin.stage, "rung": lin.rung, "mbs": r["mbs"],
                 "metric": r["metric"], "oom": r["metric"] is None}
                for lin in self.lineages for r in lin.results]

    def save_method_state(self, path: pathlib.Path) -> None:
        (path / "dsat_asha_state.json").write_text(json.dumps({
            "lineages": [lin.to_dict() for lin in self.lineages], "trials": self.trials,
            "created": self.created, "model_info": self.model_info, "stage_hi": self.stage_hi,
            "rng": self.rng.getstate()}, default=list))

    def load_method_state(self, path: pathlib.Path) -> None:
        d = json.loads((path / "dsat_asha_state.json").read_text())
        self.lineages = []
        for v in d["lineages"]:
            lin = _Lineage(v["lid"], v["stage"], v["zero_cfg"], v["lo"], v["hi"])
            lin.rung, lin.results, lin.running = v["rung"], v["results"], v["running"]
            self.lineages.append(lin)
        self.trials, self.created = d["trials"], d["created"]
        self.model_info = d["model_info"]
        self.stage_hi = {int(k): v for k, v in d["stage_hi"].items()}
        st = d["rng"]
        self.rng.setstate((st[0], tuple(st[1]), st[2]))
