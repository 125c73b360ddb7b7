"""PyTorchTrial controller behaviour (local-training mode, CPU)."""
import os

import pytest
import torch

from determined_clone_amd import core, pytorch
from tests.fixtures.onevar import OneVarTrial


def _fit(tmp_path, hparams=None, **fit_kw):
    storage = str(tmp_path / "ckpts")
    with pytorch.init(hparams=hparams or {"batch_size": 4}) as ctx:
        ctx._core.checkpoint._storage_manager = __import__(
            "determined_clone_amd.common.storage", fromlist=["x"]).SharedFSStorageManager(storage)
        trial = OneVarTrial(ctx)
        trainer = pytorch.Trainer(trial, ctx)
        ctrl = trainer.fit(**fit_kw)
        return trial, ctrl, storage


def _closed_form(n_steps, lr=OneVarTrial.LR, w=0.0):
    for _ in range(n_steps):
        w = w + 2 * lr * (1 - w)
    return w


def test_weight_updates_match_closed_form(tmp_path):
    trial, ctrl, _ = _fit(tmp_path, max_length=pytorch.Batch(10), reporting_period=pytorch.Batch(5))
    assert ctrl.state.batches_trained == 10
    w = float(trial.model.weight.detach())
    assert abs(w - _closed_form(10)) < 1e-6
    # two REPORT workloads of 5 batches each
    assert len(trial.recorder.train) == 2
    # metrics averaged over the workload: w_after == w_exp every batch
    for m in trial.recorder.train:
        assert abs(m["w_after"] - m["w_exp"]) < 1e-6
    # label_sum reducer: 5 batches * batch_size 4 labels of 1
    assert trial.recorder.train[0]["label_sum"] == pytest.approx(20.0)


def test_validation_and_checkpoint_periods(tmp_path):
    trial, ctrl, storage = _fit(tmp_path, max_length=pytorch.Batch(12),
                                validation_period=pytorch.Batch(4),
                                checkpoint_period=pytorch.Batch(6), checkpoint_policy="none")
    assert len(trial.recorder.val) == 3  # at 4, 8, 12
    assert abs(trial.recorder.val[-1]["weight"] - _closed_form(12)) < 1e-6
    # checkpoints at 6 and 12 (+ none extra since 12 is current)
    assert len(trial.recorder.uuids) == 2
    for u in trial.recorder.uuids:
        d = os.path.join(storage, u)
        assert os.path.exists(os.path.join(d, "state_dict.pth"))
        assert os.path.exists(os.path.join(d, "load_data.json"))
        assert os.path.exists(os.path.join(d, "metadata.json"))


def test_epoch_units(tmp_path):
    # 64 records / batch 4 = 16 batches per epoch
    trial, ctrl, _ = _fit(tmp_path, max_length=pytorch.Epoch(2))
    assert ctrl.state.batches_trained == 32
    assert ctrl.state.epochs_trained == 2
    assert trial.recorder.epochs_ended == [0, 1]


def test_resume_from_checkpoint_matches_uninterrupted(tmp_path):
    trial, ctrl, storage = _fit(tmp_path, max_length=pytorch.Batch(6),
                                checkpoint_period=pytorch.Batch(6))
    uuid = trial.recorder.uuids[-1]
    # continue for 4 more batches from the checkpoint
    with pytorch.init(hparams={"batch_size": 4}) as ctx:
        from determined_clone_amd.common.storage import SharedFSStorageManager

        ctx._core.checkpoint._storage_manager = SharedFSStorageManager(storage)
        t2 = OneVarTrial(ctx)
        ctrl2 = pytorch.Trainer(t2, ctx).fit(max_length=pytorch.Batch(10), latest_checkpoint=uuid)
    assert ctrl2.state.batches_trained == 10
    assert abs(float(t2.model.weight.detach()) - _closed_form(10)) < 1e-6
    assert t2.recorder.epochs_ended == []  # callback state restored, no epoch ended yet


def test_test_mode_runs_one_batch(tmp_path):
    trial, ctrl, _ = _fit(tmp_path, max_length=pytorch.Batch(100), test_mode=True)
    assert ctrl.state.batches_trained == 1


def test_aggregation_frequency(tmp_path):
    with pytorch.init(hparams={"batch_size": 4}, aggregation_frequency=2) as ctx:
        trial = OneVarTrial(ctx)
        pytorch.Trainer(trial, ctx).fit(max_length=pytorch.Batch(8))
    # gradients of 2 batches are averaged and applied once: 4 optimizer steps
    assert abs(float(trial.model.weight.detach()) - _closed_form(4)) < 1e-6


def test_fused_optimizer_cpu_path_matches(tmp_path):
    trial, ctrl, _ = _fit(tmp_path, hparams={"batch_size": 4, "fused": True}, max_length=pytorch.Batch(10))
    assert abs(float(trial.model.weight.detach()) - _closed_form(10)) < 1e-6


def test_trainunit_semantics():
    assert pytorch.Batch(5).should_stop(10)
    assert not pytorch.Batch(5).should_stop(7)
    assert pytorch.Batch([3, 7]).should_stop(7)
    assert pytorch.Batch(0).should_stop(1)
    assert pytorch.TrainUnit._from_searcher_unit(100, core.Unit.RECORDS, 32).value == 3


def test_hip_graph_option_falls_back_to_eager_on_cpu(tmp_path, caplog):
    """optimizations.hip_graph is accepted by expconf; off-GPU the controller logs why it is
    disabled and trains eagerly (the GPU replay path is tests/test_graph_gpu.py)."""
    from determined_clone_amd.config import expconf

    cfg = expconf.complete({"entrypoint": "x:y", "searcher": {"name": "single", "metric": "m",
                                                              "max_length": {"batches": 1}},
                            "optimizations": {"hip_graph": True, "hip_graph_warmup_steps": 2}})
    assert cfg["optimizations"]["hip_graph"] is True
    storage = str(tmp_path / "ckpts")
    with pytorch.init(hparams={"batch_size": 4}, exp_conf={"optimizations": {"hip_graph": True}}) as ctx:
        ctx._core.checkpoint._storage_manager = __import__(
            "determined_clone_amd.common.storage", fromlist=["x"]).SharedFSStorageManager(storage)
        trial = OneVarTrial(ctx)
        with caplog.at_level("WARNING"):
            ctrl = pytorch.Trainer(trial, ctx).fit(max_length=pytorch.Batch(4))
    assert "hip_graph disabled: not on a GPU" in caplog.text
    assert getattr(ctrl, "_graphed", None) is None
