"""Run a class-based trial (``module:Class`` entrypoint) on the cluster
(reference: `harness/determined/exec/harness.py` + `_execution.py`).

Training periods come from the experiment config: ``min_validation_period`` and
``min_checkpoint_period`` (batches/records/epochs), ``scheduling_unit`` as the metrics reporting
period, ``checkpoint_policy``, ``perform_initial_validation``."""
import importlib
import logging
import os
import sys

from determined_clone_amd import _info


def _unit(length, gbs, records_per_epoch):
    from determined_clone_amd import pytorch

    (k, n), = length.items()
    if n <= 0:
        return None
    if k == "batches":
        return pytorch.Batch(n)
    if k == "records":
        return pytorch.Batch(max(n // gbs, 1)) if gbs else None
    return pytorch.Epoch(n)


def load_trial_class(spec: str):
    ctx = os.environ.get("DET_CONTEXT_DIR")
    if ctx and ctx not in sys.path:
        sys.path.insert(0, ctx)
    mod, _, qual = spec.partition(":")
    obj = importlib.import_module(mod)
    for part in qual.split("."):
        obj = getattr(obj, part)
    return obj


def _trace(what: str) -> None:
    from determined_clone_amd.util import startup_mark

    startup_mark(what)


def main(spec: str) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    _trace("harness main")
    prof = None
    if os.environ.get("DET_STARTUP_PROFILE") == "1":
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    from determined_clone_amd import pytorch

    info = _info.get_cluster_info()
    cfg = info.trial._config
    _trace("framework imported")
    trial_cls = load_trial_class(spec)
    _trace("trial class loaded")
    if getattr(trial_cls, "_is_deepspeed_trial", False):
        from determined_clone_amd.pytorch import deepspeed as ds

        return ds.run_deepspeed_trial(trial_cls, info)
    gbs = info.trial.hparams.get("global_batch_size")
    rpe = int(cfg.get("records_per_epoch") or 0)
    opts = cfg.get("optimizations") or {}
    with pytorch.init(aggregation_frequency=int(opts.get("aggregation_frequency", 1))) as ctx:
        _trace("pytorch.init")
        if prof is not None:
            import io
            import pstats

            prof.disable()
            buf = io.StringIO()
            pstats.Stats(prof, stream=buf).sort_stats("cumulative").print_stats(25)
            logging.getLogger("determined_clone_amd.startup").info(buf.getvalue())
        trial = trial_cls(ctx)
        _trace("trial constructed")
        trainer = pytorch.Trainer(trial, ctx)
        if (cfg.get("profiling") or {}).get("enabled"):
            p = cfg["profiling"]
            trainer.configure_profiler(True, p.get("sync_timings", True), p.get("begin_on_batch", 0),
                                       p.get("end_after_batch"))
        trainer.fit(
            checkpoint_period=_unit(cfg["min_checkpoint_period"], gbs, rpe),
            validation_period=_unit(cfg["min_validation_period"], gbs, rpe),
            reporting_period=pytorch.Batch(int(cfg.get("scheduling_unit") or 100)),
            checkpoint_policy=cfg.get("checkpoint_policy", "best"),
            latest_checkpoint=info.latest_checkpoint,
            step_zero_validation=bool(cfg.get("perform_initial_validation")),
        )
        _trace("fit done")
    _trace("context closed")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
