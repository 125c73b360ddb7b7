"""Hyperparameter sampling and grids (reference: `master/pkg/searcher/hyperparameters.go`,
`grid.go`). Iteration order over hyperparameter names is sorted, so a given seed always produces the
same samples."""
import itertools
import math
from typing import Any, Dict, List, Tuple

import numpy as np


def _is_hp(d: Any) -> bool:
    return isinstance(d, dict) and "type" in d


def sample_one(hp: Any, rng: np.random.RandomState) -> Any:
    if not isinstance(hp, dict):
        return hp
    if not _is_hp(hp):  # nested group
        return {k: sample_one(hp[k], rng) for k in sorted(hp)}
    t = hp["type"]
    if t == "const":
        return hp["val"]
    if t == "int":
        return int(hp["minval"] + rng.randint(0, hp["maxval"] - hp["minval"] + 1))
    if t == "double":
        return float(rng.uniform(hp["minval"], hp["maxval"]))
    if t == "log":
        return float(math.pow(hp.get("base", 10.0), rng.uniform(hp["minval"], hp["maxval"])))
    if t == "categorical":
        vals = hp["vals"]
        return vals[int(rng.randint(0, len(vals)))]
    raise ValueError(f"unknown hyperparameter type {t}")


def sample_all(hps: Dict[str, Any], rng: np.random.RandomState) -> Dict[str, Any]:
    return {name: sample_one(hps[name], rng) for name in sorted(hps)}


def _axes(route: Tuple[str, ...], hp: Any) -> List[List[Tuple[Tuple[str, ...], Any]]]:
    if not isinstance(hp, dict):
        return [[(route, hp)]]
    if not _is_hp(hp):
        axes = []
        for k in sorted(hp):
            axes += _axes(route + (k,), hp[k])
        return axes
    t = hp["type"]
    if t == "const":
        return [[(route, hp["val"])]]
    if t == "categorical":
        return [[(route, v) for v in hp["vals"]]]
    count = int(hp["count"])
    lo, hi = hp["minval"], hp["maxval"]
    if t == "int":
        count = min(count, hi - lo + 1)
        if count == 1:
            return [[(route, int(round((lo + hi) / 2.0)))]]
        return [[(route, int(round(lo + i * (hi - lo) / (count - 1)))) for i in range(count)]]
    if t == "double":
        if count == 1:
            return [[(route, (lo + hi) / 2.0)]]
        return [[(route, lo + i * (hi - lo) / (count - 1)) for i in range(count)]]
    if t == "log":
        base = hp.get("base", 10.0)
        if count == 1:
            return [[(route, math.pow(base, (lo + hi) / 2.0))]]
        return [[(route, math.pow(base, lo + i * (hi - lo) / (count - 1))) for i in range(count)]]
    raise ValueError(f"unknown hyperparameter type {t}")


def grid(hps: Dict[str, Any]) -> List[Dict[str, Any]]:
    """Cartesian product of every axis (nested groups contribute one axis per leaf)."""
    axes = []
    for name in sorted(hps):
        axes += _axes((name,), hps[name])
    out = []
    for combo in itertools.product(*axes) if axes else [()]:
        sample: Dict[str, Any] = {}
        for route, val in combo:
            d = sample
            for r in route[:-1]:
                d = d.setdefault(r, {})
            d[route[-1]] = val
        out.append(sample)
    return out
