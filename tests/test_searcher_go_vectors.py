"""The reference's Go searcher test vectors, ported verbatim with a port of its value-simulation
harness (master/pkg/searcher/util_test.go:156-300 checkValueSimulation: Create requests get the
predefined trials in order, every ValidateAfter is checked against the trial's expected length,
early-exit trials exit at their last op, the method's state is snapshotted and restored after
every validation, and every trial must have run exactly its expected ops).

Sources: asha_test.go:12-229 (records / batches / epochs unit vectors and TestASHASearchMethod),
adaptive_asha_test.go:14-30 (bracket allocation)."""
import numpy as np
import pytest

from determined_clone_amd import searcher as S
from determined_clone_amd.searcher import methods as M


def _ops(spec):
    """toOps("1000B 3000B") -> [1000, 3000] (units are length-agnostic in our searcher)."""
    return [int(tok[:-1]) for tok in spec.split()]


class Trial:
    def __init__(self, ops, metric, early_exit=False):
        self.ops = _ops(ops)
        self.metrics = [metric] * len(self.ops)
        self.early_exit = len(self.ops) - 1 if early_exit else None


def const(ops, metric):
    return Trial(ops, metric)


def early(ops, metric):
    return Trial(ops, metric, early_exit=True)


def _save_and_reload(method):
    state = method.snapshot()
    method.restore(state)


def check_value_simulation(method, trials, hparams=None):
    ctx = M.Context(np.random.RandomState(0), hparams or {})
    next_trial = 0
    trial_of, op_idx, exited = {}, {}, set()
    pending = list(method.initial_operations(ctx))
    while pending:
        op = pending.pop(0)
        if isinstance(op, M.Create):
            assert next_trial < len(trials), "search method created too many trials"
            trial_of[op.request_id] = next_trial
            op_idx[op.request_id] = 0
            ops = method.trial_created(ctx, op.request_id)
            next_trial += 1
        elif isinstance(op, M.ValidateAfter):
            rid = op.request_id
            if rid in exited:
                continue
            t = trials[trial_of[rid]]
            i = op_idx[rid]
            assert i < len(t.ops), f"trial {trial_of[rid] + 1}: ran out of expected ops"
            assert op.length == t.ops[i], f"trial {trial_of[rid] + 1}: wanted {t.ops[i]} got {op.length}"
            if t.early_exit is not None and i == t.early_exit:
                exited.add(rid)
                ops = method.trial_exited_early(ctx, rid, M.ExitedReason.USER_REQUESTED_STOP)
            else:
                ops = method.validation_completed(ctx, rid, t.metrics[i], op)
            op_idx[rid] += 1
            _save_and_reload(method)
        elif isinstance(op, M.Close):
            rid = op.request_id
            t = trials[trial_of[rid]]
            assert op_idx[rid] == len(t.ops), f"trial {trial_of[rid] + 1} closed with ops left"
            ops = method.trial_closed(ctx, rid)
        elif isinstance(op, M.Shutdown):
            ops = []
        else:
            raise AssertionError(f"unexpected searcher operation {op!r}")
        pending.extend(ops)
    for rid, ti in trial_of.items():
        assert op_idx[rid] == len(trials[ti].ops), f"incomplete trial {ti + 1}"
    assert next_trial == len(trials), f"created {next_trial} trials, expected {len(trials)}"


def _asha(smaller=True, num_rungs=3, max_length=9000, max_trials=12, divisor=3):
    return S.AsyncHalvingSearch(num_rungs=num_rungs, max_length=max_length, max_trials=max_trials,
                                divisor=divisor, smaller_is_better=smaller)


def _simulate_lengths(method):
    res = S.simulate(method, {}, seed=0, metric_fn=S.constant_validation)
    return sorted(res["lengths"].values(), key=lambda l: (len(l), l))


@pytest.mark.parametrize("max_length,expected", [
    # TestASHASearcherRecords / Batches / Epochs (asha_test.go:12-70)
    (576000, [[64000]] * 8 + [[64000, 192000]] * 3 + [[64000, 192000, 576000]]),
    (9000, [[1000]] * 8 + [[1000, 3000]] * 3 + [[1000, 3000, 9000]]),
    (12, [[1]] * 8 + [[1, 4]] * 3 + [[1, 4, 12]]),
])
def test_asha_unit_vectors(max_length, expected):
    assert _simulate_lengths(_asha(max_length=max_length)) == expected


ASHA_METHOD_CASES = {
    # TestASHASearchMethod (asha_test.go:72-229)
    "smaller is better": (True, [
        const("1000B 3000B 9000B", 0.01), const("1000B 3000B", 0.02), const("1000B 3000B", 0.03),
        const("1000B 3000B", 0.04), const("1000B", 0.05), const("1000B", 0.06), const("1000B", 0.07),
        const("1000B", 0.08), const("1000B", 0.09), const("1000B", 0.10), const("1000B", 0.11),
        const("1000B", 0.12)]),
    "early exit -- smaller is better": (True, [
        const("1000B 3000B 9000B", 0.01), const("1000B 3000B", 0.02), early("1000B 3000B", 0.03),
        const("1000B 3000B", 0.04), const("1000B", 0.05), const("1000B", 0.06), const("1000B", 0.07),
        const("1000B", 0.08), const("1000B", 0.09), const("1000B", 0.10), const("1000B", 0.11),
        const("1000B", 0.12)]),
    "smaller is not better": (False, [
        const("1000B 3000B 9000B", 0.12), const("1000B 3000B", 0.11), const("1000B 3000B", 0.10),
        const("1000B 3000B", 0.09), const("1000B", 0.08), const("1000B", 0.07), const("1000B", 0.06),
        const("1000B", 0.05), const("1000B", 0.04), const("1000B", 0.03), const("1000B", 0.02),
        const("1000B", 0.01)]),
    "early exit -- smaller is not better": (False, [
        const("1000B 3000B 9000B", 0.12), const("1000B 3000B", 0.11), early("1000B 3000B", 0.10),
        const("1000B 3000B", 0.09), const("1000B", 0.08), const("1000B", 0.07), const("1000B", 0.06),
        const("1000B", 0.05), const("1000B", 0.04), const("1000B", 0.03), const("1000B", 0.02),
        const("1000B", 0.01)]),
    "async promotions": (True, [
        const("1000B 3000B", 0.10), const("1000B", 0.11), early("1000B", 0.12),
        const("1000B 3000B 9000B", 0.01), const("1000B 3000B", 0.02), const("1000B 3000B", 0.03),
        const("1000B 3000B", 0.04), const("1000B", 0.05), const("1000B", 0.06), const("1000B", 0.07),
        const("1000B", 0.08), const("1000B", 0.09)]),
}


@pytest.mark.parametrize("name", sorted(ASHA_METHOD_CASES))
def test_asha_search_method_value_simulation(name):
    smaller, trials = ASHA_METHOD_CASES[name]
    check_value_simulation(_asha(smaller=smaller), trials)


def test_asha_single_rung_bracket():
    trials = [const("9000B", 0.05), const("9000B", 0.06), const("9000B", 0.07), const("9000B", 0.08)]
    check_value_simulation(_asha(num_rungs=1, max_trials=4), trials)


def test_bracket_max_trials_go_vectors():
    # adaptive_asha_test.go:14-19
    assert M.bracket_max_trials(20, 3.0, [3, 2, 1]) == [12, 5, 3]
    assert M.bracket_max_trials(50, 3.0, [4, 3]) == [35, 15]
    assert M.bracket_max_trials(50, 4.0, [3, 2]) == [37, 13]
    assert M.bracket_max_trials(100, 4.0, [4, 3, 2]) == [70, 22, 8]


def test_bracket_max_concurrent_trials_go_vectors():
    # adaptive_asha_test.go:21-26
    assert M.bracket_max_concurrent(0, 3.0, [9, 3, 1]) == [3, 3, 3]
    assert M.bracket_max_concurrent(11, 3.0, [9, 3, 1]) == [4, 4, 3]
    assert M.bracket_max_concurrent(0, 4.0, [40, 10]) == [10, 10]
