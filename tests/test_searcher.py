"""Search-method behaviour, mirroring the reference's Go searcher tests (asha_test.go,
adaptive_asha_test.go, grid_test.go, random_test.go) with our simulator."""
import pytest

from determined_clone_amd import searcher as S


def _sorted_lengths(res):
    return sorted(res["lengths"].values(), key=lambda l: (len(l), l))


def test_asha_batches_constant_metric():
    m = S.AsyncHalvingSearch(num_rungs=3, max_length=9000, max_trials=12, divisor=3)
    res = S.simulate(m, {"x": {"type": "double", "minval": 0, "maxval": 1}}, seed=0,
                     metric_fn=S.constant_validation)
    got = _sorted_lengths(res)
    expected = [[1000]] * 8 + [[1000, 3000]] * 3 + [[1000, 3000, 9000]]
    assert got == expected


def test_asha_stopping_variant_terminates():
    m = S.AsyncHalvingStoppingSearch(num_rungs=3, max_length=900, max_trials=12, divisor=3)
    res = S.simulate(m, {}, seed=1, metric_fn=S.random_validation)
    assert res["trials"] == 12
    assert max(len(l) for l in res["lengths"].values()) <= 3


def test_random_and_single():
    res = S.simulate(S.RandomSearch(5, 100, 2), {"lr": {"type": "log", "minval": -3, "maxval": -1}}, seed=3)
    assert res["trials"] == 5 and all(l == [100] for l in res["lengths"].values())
    res = S.simulate(S.SingleSearch(7), {}, seed=3)
    assert res["trials"] == 1 and list(res["lengths"].values()) == [[7]]


def test_grid_cartesian_product_with_nested():
    hps = {"a": {"type": "int", "minval": 1, "maxval": 3, "count": 3},
           "b": {"type": "categorical", "vals": ["x", "y"]},
           "n": {"c": {"type": "double", "minval": 0.0, "maxval": 1.0, "count": 2}, "d": 5}}
    g = S.hparams.grid(hps)
    assert len(g) == 3 * 2 * 2
    assert {"a": 1, "b": "x", "n": {"c": 0.0, "d": 5}} in g
    res = S.simulate(S.GridSearch(10, 4), hps, seed=0)
    assert res["trials"] == 12


def test_grid_int_count_clamped_and_log():
    g = S.hparams.grid({"i": {"type": "int", "minval": 0, "maxval": 1, "count": 10},
                        "l": {"type": "log", "minval": 0, "maxval": 2, "base": 10, "count": 3}})
    assert sorted({x["i"] for x in g}) == [0, 1]
    assert sorted({round(x["l"], 6) for x in g}) == [1.0, 10.0, 100.0]


def test_adaptive_asha_brackets():
    m = S.AdaptiveASHASearch(max_length=1000, max_trials=64, mode="standard", divisor=4, max_rungs=5,
                             max_concurrent_trials=16)
    # standard mode: max_rungs=min(5, int(log4 1000)+1=5, int(log4 64)+1=4)=4 -> brackets 2..4
    assert [s.num_rungs for s in m.subs] == [4, 3, 2]
    assert sum(s.max_trials for s in m.subs) == 64
    res = S.simulate(m, {"x": {"type": "double", "minval": 0, "maxval": 1}}, seed=0)
    assert res["trials"] == 64


def test_bracket_allocation_helpers():
    # weights divisor^(r-1)/r = 16/3 : 2 : 1 of 100 trials (the Go vectors themselves are in
    # test_searcher_go_vectors.py)
    assert S.methods.bracket_max_trials(100, 4, [3, 2, 1]) == [64, 24, 12]
    assert S.methods.bracket_max_concurrent(16, 4, [10, 10, 10]) == [6, 5, 5]
    assert S.methods.adaptive_bracket_rungs("conservative", 3) == [1, 2, 3]
    assert S.methods.adaptive_bracket_rungs("aggressive", 3) == [3]


def test_invalid_hp_replaced_in_asha():
    hps = {"x": {"type": "double", "minval": 0, "maxval": 1}}
    s = S.Searcher(0, S.AsyncHalvingSearch(2, 100, 4, 2, 4), hps)
    ops = s.initial_operations()
    creates = [o for o in ops if isinstance(o, S.Create)]
    assert len(creates) == 4
    for c in creates:
        s.trial_created(c.request_id)
    out = s.trial_exited_early(creates[0].request_id, S.ExitedReason.INVALID_HP)
    assert any(isinstance(o, S.Create) for o in out)
    assert any(isinstance(o, S.Close) and o.request_id == creates[0].request_id for o in out)


def test_searcher_snapshot_restore_roundtrip():
    hps = {"x": {"type": "double", "minval": 0, "maxval": 1}}
    s1 = S.Searcher(7, S.AsyncHalvingSearch(3, 90, 9, 3), hps)
    ops = s1.initial_operations()
    for o in ops:
        if isinstance(o, S.Create):
            s1.trial_created(o.request_id)
    blob = s1.snapshot()
    s2 = S.Searcher(7, S.AsyncHalvingSearch(3, 90, 9, 3), hps)
    s2.restore(blob)
    va = [o for o in ops if isinstance(o, S.ValidateAfter)][0]
    a = s1.validation_completed(va.request_id, 0.5, va)
    b = s2.validation_completed(va.request_id, 0.5, va)
    assert [x.to_dict() for x in a] == [x.to_dict() for x in b]


def test_sampling_deterministic():
    import numpy as np

    hps = {"a": {"type": "int", "minval": 1, "maxval": 10}, "b": {"type": "categorical", "vals": [1, 2, 3]},
           "c": {"type": "const", "val": "z"}}
    x = S.hparams.sample_all(hps, np.random.RandomState(5))
    y = S.hparams.sample_all(hps, np.random.RandomState(5))
    assert x == y and x["c"] == "z" and 1 <= x["a"] <= 10
