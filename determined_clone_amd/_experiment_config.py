"""``det.ExperimentConfig``: the merged expconf as a dict with typed accessors (reference:
`harness/determined/_experiment_config.py`). Missing sections fall back to the expconf defaults
(``config/expconf.py``) instead of raising, so a partially specified local config works too."""
from typing import Any, Dict, List, Optional, Tuple, Union


class ExperimentConfig(dict):
    def _section(self, key: str) -> Dict[str, Any]:
        v = self.get(key)
        return v if isinstance(v, dict) else {}

    def debug_enabled(self) -> bool:
        return bool(self.get("debug", False))

    def scheduling_unit(self) -> int:
        return int(self.get("scheduling_unit", 100))

    def native_parallel_enabled(self) -> bool:
        return bool(self._section("resources").get("native_parallel", False))

    def average_training_metrics_enabled(self) -> bool:
        return bool(self._section("optimizations").get("average_training_metrics", True))

    def slots_per_trial(self) -> int:
        return int(self._section("resources").get("slots_per_trial", 1))

    def experiment_seed(self) -> int:
        return int(self._section("reproducibility").get("experiment_seed", 0))

    def profiling_enabled(self) -> bool:
        return bool(self._section("profiling").get("enabled", False))

    def profiling_interval(self) -> Tuple[int, Optional[int]]:
        """(begin_on_batch, end_after_batch); (0, 0) when profiling is off."""
        p = self._section("profiling")
        if not p.get("enabled", False):
            return 0, 0
        end = p.get("end_after_batch")
        return int(p.get("begin_on_batch", 0)), (int(end) if end is not None else None)

    def profiling_sync_timings(self) -> bool:
        return bool(self._section("profiling").get("sync_timings", True))

    def get_records_per_epoch(self) -> Optional[int]:
        r = self.get("records_per_epoch")
        return None if r is None else int(r)

    def get_min_validation_period(self) -> Dict[str, Any]:
        return self._section("min_validation_period")

    def get_min_checkpoint_period(self) -> Dict[str, Any]:
        return self._section("min_checkpoint_period")

    def get_searcher_metric(self) -> str:
        m = self._section("searcher").get("metric")
        if not isinstance(m, str):
            raise ValueError(f"searcher.metric must be a string, got {m!r}")
        return m

    def get_optimizations_config(self) -> Dict[str, Any]:
        return self._section("optimizations")

    def get_checkpoint_storage(self) -> Dict[str, Any]:
        return self._section("checkpoint_storage")

    def get_entrypoint(self) -> Union[str, List[str]]:
        ep = self.get("entrypoint")
        if isinstance(ep, str) or (isinstance(ep, list) and all(isinstance(e, str) for e in ep)):
            return ep
        raise ValueError(f"invalid entrypoint in experiment config: {ep!r}")
