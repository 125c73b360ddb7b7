"""Experimental APIs (reference: `harness/determined/experimental/__init__.py`): the Python client
SDK lives in :mod:`.client`."""
from determined_clone_amd.experimental import client
from determined_clone_amd.experimental.client import (Checkpoint, CheckpointState, Determined,
                                                      DownloadMode, Experiment, ExperimentState,
                                                      Model, ModelVersion, OrderBy, Project, Trial,
                                                      TrialMetrics, TrialState, User, Workspace)


def test_one_batch(trial_class, config=None):
    """Smoke-test a trial class locally: one training batch + validation in test mode, with the
    config's hyperparameters (reference: `harness/determined/experimental/_native.py`
    test_one_batch). PyTorchTrial subclasses only -- the trial API this framework implements."""
    import logging

    from determined_clone_amd import pytorch

    log = logging.getLogger("determined_clone_amd")
    config = {**(config or {}), "scheduling_unit": 1}
    if not (isinstance(trial_class, type) and issubclass(trial_class, pytorch.PyTorchTrial)):
        raise TypeError(f"test_one_batch supports PyTorchTrial subclasses, got {trial_class!r}")
    hparams = {k: (v.get("val") if isinstance(v, dict) and "val" in v else v)
               for k, v in (config.get("hyperparameters") or {}).items()}
    log.info("Running a minimal test experiment locally")
    with pytorch.init(hparams=hparams, exp_conf=config) as ctx:
        trainer = pytorch.Trainer(trial_class(ctx), ctx)
        trainer.fit(max_length=pytorch.Batch(1), test_mode=True, checkpoint_policy="none")
    log.info("The test experiment passed.")
