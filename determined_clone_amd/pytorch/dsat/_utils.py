"""DeepSpeed autotune helpers for user code and the search methods (reference:
`harness/determined/pytorch/dsat/_utils.py`).

* :func:`get_ds_config_from_hparams` -- the DeepSpeed config a trial should build its engine from:
  the json file named by ``hparams["deepspeed_config"]`` (relative to the model directory) with the
  search's ``overwrite_deepspeed_args`` merged over it.
* :func:`dsat_reporting_context` -- Core API scripts wrap their engine forward / backward / step in
  it. During a dsat trial the native engine's autotuning hook (``pytorch/deepspeed/_autotune.py``)
  writes its measurements to a json file and ends the run with ``SystemExit``; the context reports
  that file to the master (validation metrics + the searcher operation) and re-raises.
* the memory model (:func:`approx_max_mbs_per_stage`) that turns the model-profile trial's numbers
  into per-ZeRO-stage micro-batch ranges for MI355X's HBM.
"""
import contextlib
import copy
import json
import os
import pathlib
import random
from typing import Any, Dict, Generator, Iterable, Optional, Union

from determined_clone_amd.pytorch.dsat import _defaults


def merge_dicts(base: Dict[str, Any], overwrite: Dict[str, Any]) -> Dict[str, Any]:
    """Recursive merge: dict values merge key by key, anything else in ``overwrite`` replaces."""
    out = copy.deepcopy(base)
    for k, v in (overwrite or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = merge_dicts(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def smaller_is_better(metric: str) -> bool:
    if metric in _defaults.SMALLER_IS_BETTER_METRICS:
        return True
    if metric in _defaults.LARGER_IS_BETTER_METRICS:
        return False
    raise ValueError(f"unknown dsat metric {metric!r}; one of "
                     f"{_defaults.SMALLER_IS_BETTER_METRICS + _defaults.LARGER_IS_BETTER_METRICS}")


def get_ds_config_from_hparams(hparams: Dict[str, Any],
                               base_dir: Union[str, pathlib.Path] = ".") -> Dict[str, Any]:
    """The DeepSpeed config of this trial: ``hparams["deepspeed_config"]`` (a json path relative to
    ``base_dir``, or an inline dict) merged with ``hparams["overwrite_deepspeed_args"]``."""
    if _defaults.CONFIG_KEY not in hparams:
        raise KeyError(f"expected a {_defaults.CONFIG_KEY!r} hyperparameter naming the DeepSpeed "
                       f"json config; got {sorted(hparams)}")
    src = hparams[_defaults.CONFIG_KEY]
    if isinstance(src, dict):
        base = src
    else:
        with open(pathlib.Path(base_dir) / src) as f:
            base = json.load(f)
    return merge_dicts(base, hparams.get(_defaults.OVERWRITE_KEY) or {})


def get_batch_config_from_mbs_gas_and_slots(ds_config: Dict[str, Any], slots: int) -> Dict[str, int]:
    """A consistent (train_batch_size, micro batch, accumulation) triple for ``slots`` ranks."""
    mbs = int(ds_config["train_micro_batch_size_per_gpu"])
    gas = ds_config.get("gradient_accumulation_steps", _defaults.GAS_DEFAULT)
    gas = 1 if gas == "auto" else int(gas)
    return {"train_batch_size": mbs * gas * slots, "train_micro_batch_size_per_gpu": mbs,
            "gradient_accumulation_steps": gas}


def get_zero_stage_search_space(stage: int) -> Dict[str, list]:
    if stage not in _defaults.DEFAULT_ZERO_SEARCH_SPACE:
        raise ValueError(f"ZeRO stage must be one of {sorted(_defaults.DEFAULT_ZERO_SEARCH_SPACE)}")
    space: Dict[str, list] = {}
    for s in range(1, stage + 1):
        space.update(_defaults.DEFAULT_ZERO_SEARCH_SPACE[s])
    return space


def get_random_zero_optim_config(stage: int, rng: Optional[random.Random] = None) -> Dict[str, Any]:
    rng = rng or random
    cfg = {k: rng.choice(v) for k, v in sorted(get_zero_stage_search_space(stage).items())}
    cfg["stage"] = stage
    return cfg


# ------------------------------------------------------------------------------ memory model
def state_bytes_per_param(stage: int, dp: int) -> float:
    """Per-rank bytes of model + optimizer state per parameter in the native engine (bf16 weights
    and gradients, fp32 master weights and two Adam moments = 12 B in the fused optimizer):
    ZeRO-1 partitions the 12 B, ZeRO-2 also the gradients, ZeRO-3 everything."""
    dp = max(1, int(dp))
    return {0: 16.0, 1: 4.0 + 12.0 / dp, 2: 2.0 + 14.0 / dp, 3: 16.0 / dp}[int(stage)]


def approx_max_mbs_per_stage(model_info: Dict[str, Any], stages: Iterable[int], dp: int,
                             max_mbs: int, headroom: float = 0.9) -> Dict[int, int]:
    """Largest micro batch per ZeRO stage that the model-profile numbers say fits in device memory:
    (headroom * device bytes - state bytes) / activation bytes per sample."""
    mem = float(model_info.get("gpu_mem") or 0)
    params = float(model_info.get("num_params") or 0)
    act = float(model_info.get("activation_mem_per_gpu") or 0)
    out = {}
    for s in stages:
        free = headroom * mem - params * state_bytes_per_param(s, dp)
        if act <= 0 or mem <= 0:
            out[int(s)] = int(max_mbs)
        else:
            out[int(s)] = int(max(1, min(max_mbs, free // act)))
    return out


# ------------------------------------------------------------------------------ Core API reporting
def report_json_results(core_context: Any, op: Any, steps_completed: int,
                        path: Union[str, pathlib.Path]) -> Dict[str, Any]:
    """Report one autotuning result file: validation metrics + the searcher operation (chief)."""
    with open(path) as f:
        results = json.load(f)
    if core_context.distributed.rank == 0:
        core_context.train.report_validation_metrics(steps_completed=steps_completed, metrics=results)
        op.report_completed(results)
    return results


@contextlib.contextmanager
def dsat_reporting_context(core_context: Any, op: Any,
                           steps_completed: Optional[int] = None) -> Generator[None, None, None]:
    """Wrap the engine's forward / backward / step of a Core API training loop. When the engine
    ends a dsat profiling run (``SystemExit`` after writing its measurements), the measurements
    are reported for ``op`` and the exit continues."""
    steps = op.length if steps_completed is None else steps_completed
    try:
        yield
    except SystemExit:
        found = [p for p in (_defaults.MODEL_INFO_PROFILING_PATH, _defaults.AUTOTUNING_RESULTS_PATH)
                 if os.path.exists(p)]
        if len(found) == 1:
            report_json_results(core_context, op, steps, found[0])
        raise
