"""Custom searcher run locally against a master (reference: examples/features/custom_search_method).
A simple successive-halving search implemented as a user-side SearchMethod."""
import sys
import uuid
from typing import Any, Dict, List

import numpy as np

from determined_clone_amd import searcher


class SimpleHalving(searcher.SearchMethod):
    def __init__(self, n: int = 8, rungs=(10, 30, 90), seed: int = 0) -> None:
        self.rng = np.random.RandomState(seed)
        self.n, self.rungs = n, list(rungs)
        self.results: Dict[int, Dict[str, float]] = {i: {} for i in range(len(self.rungs))}
        self.rung_of: Dict[str, int] = {}

    def initial_operations(self, state: searcher.SearcherState) -> List[searcher.Operation]:
        ops: List[searcher.Operation] = []
        for _ in range(self.n):
            rid = uuid.uuid4()
            self.rung_of[str(rid)] = 0
            ops += [searcher.Create(rid, {"global_batch_size": 4, "lr": float(10 ** self.rng.uniform(-3, -1))}),
                    searcher.ValidateAfter(rid, self.rungs[0])]
        return ops

    def on_trial_created(self, state, request_id):
        return []

    def on_validation_completed(self, state, request_id, metric: Any, train_length: int):
        r = self.rung_of[str(request_id)]
        self.results[r][str(request_id)] = float(metric)
        expected = max(1, self.n // (2 ** r))
        if len(self.results[r]) < expected:
            return []
        ranked = sorted(self.results[r], key=self.results[r].get)
        keep = ranked[: max(1, expected // 2)] if r + 1 < len(self.rungs) else []
        ops: List[searcher.Operation] = []
        for rid in ranked:
            u = uuid.UUID(rid)
            if rid in keep:
                self.rung_of[rid] = r + 1
                ops.append(searcher.ValidateAfter(u, self.rungs[r + 1]))
            else:
                ops.append(searcher.Close(u))
        return ops

    def on_trial_closed(self, state, request_id):
        return [searcher.Shutdown()] if len(state.trials_closed) == self.n else []

    def progress(self, state):
        return len(state.trials_closed) / self.n

    def on_trial_exited_early(self, state, request_id, exited_reason):
        return [searcher.Close(request_id)]


if __name__ == "__main__":
    import yaml

    cfg = yaml.safe_load(open(sys.argv[1]))
    runner = searcher.LocalSearchRunner(SimpleHalving(), searcher_dir="searcher_state")
    print("experiment", runner.run(cfg, model_dir=sys.argv[2]))
