"""Searcher simulation / HP-search preview (reference: `master/pkg/searcher/simulate.go`,
`PreviewHPSearch` API). Runs a search method against synthetic validation metrics and reports, per
trial, the sequence of training lengths it would be asked for."""
import random
from typing import Any, Callable, Dict, List, Optional

from determined_clone_amd.searcher._searcher import Searcher
from determined_clone_amd.searcher.methods import (Close, Create, SearchMethod, Shutdown,
                                                   ValidateAfter)


def constant_validation(rng: random.Random, trial_id: int, idx: int) -> float:
    return 1.0


def random_validation(rng: random.Random, trial_id: int, idx: int) -> float:
    return rng.random()


def trial_id_metric(rng: random.Random, trial_id: int, idx: int) -> float:
    return float(trial_id)


def simulate(method: SearchMethod, hparams: Dict[str, Any], seed: int = 0,
             metric_fn: Callable[[random.Random, int, int], float] = random_validation,
             max_events: int = 100000) -> Dict[str, Any]:
    s = Searcher(seed, method, hparams)
    rng = random.Random(seed)
    pending: List[Any] = list(s.initial_operations())
    trial_ids: Dict[str, int] = {}
    lengths: Dict[str, List[int]] = {}
    queue: Dict[str, List[ValidateAfter]] = {}
    closed: Dict[str, bool] = {}
    shutdown = False
    events = 0

    def handle(ops: List[Any]) -> None:
        nonlocal shutdown
        for op in ops:
            if isinstance(op, Create):
                trial_ids[op.request_id] = len(trial_ids)
                lengths[op.request_id] = []
                queue[op.request_id] = []
                handle(s.trial_created(op.request_id))
            elif isinstance(op, ValidateAfter):
                queue[op.request_id].append(op)
            elif isinstance(op, Close):
                closed[op.request_id] = True
            elif isinstance(op, Shutdown):
                shutdown = True

    handle(pending)
    while not shutdown and events < max_events:
        ready = [r for r in trial_ids if queue[r]]
        if not ready:
            to_close = [r for r in trial_ids if closed.get(r) and not s.trial_is_closed(r)]
            if not to_close:
                break
            for r in to_close:
                handle(s.trial_closed(r))
            continue
        r = rng.choice(ready)
        op = queue[r].pop(0)
        lengths[r].append(op.length)
        metric = metric_fn(rng, trial_ids[r], len(lengths[r]) - 1)
        handle(s.validation_completed(r, metric, op))
        events += 1
        for rr in [x for x in trial_ids if closed.get(x) and not queue[x] and not s.trial_is_closed(x)]:
            handle(s.trial_closed(rr))
    summary: Dict[str, int] = {}
    for r, ls in lengths.items():
        key = str(ls)
        summary[key] = summary.get(key, 0) + 1
    return {"trials": len(trial_ids), "results": summary,
            "total_units": sum(sum(_incremental(ls)) for ls in lengths.values()),
            "lengths": {trial_ids[r]: ls for r, ls in lengths.items()}}


def _incremental(ls: List[int]) -> List[int]:
    # ValidateAfter lengths for ASHA promotions are increments; single/random/grid are absolute.
    return ls
