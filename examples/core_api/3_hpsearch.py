"""Core API stage 3: hyperparameter search -- train to each searcher operation's length and report
the searcher metric (reference: core_api/3_hpsearch.py)."""
import logging
import time

import determined_clone_amd as det
from determined_clone_amd import core


def main(core_context: core.Context, increment_by: float) -> None:
    x, batch = 0.0, 0
    for op in core_context.searcher.operations():
        while batch < op.length:
            x += increment_by
            batch += 1
            time.sleep(0.01)
            if batch % 10 == 0:
                core_context.train.report_training_metrics(steps_completed=batch, metrics={"x": x})
                op.report_progress(batch)
        core_context.train.report_validation_metrics(steps_completed=batch, metrics={"x": x})
        op.report_completed(x)


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format=det.LOG_FORMAT)
    info = det.get_cluster_info()
    hparams = info.trial.hparams if info else {"increment_by": 1.0}
    with core.init() as core_context:
        main(core_context, increment_by=float(hparams["increment_by"]))
