"""Core API stage 1: report training / validation metrics (reference: core_api/1_metrics.py)."""
import logging
import time

import determined_clone_amd as det
from determined_clone_amd import core


def main(core_context: core.Context, increment_by: int) -> None:
    x = 0
    steps_completed = 0
    for batch in range(100):
        x += increment_by
        steps_completed = batch + 1
        time.sleep(0.01)
        if steps_completed % 10 == 0:
            core_context.train.report_training_metrics(steps_completed=steps_completed, metrics={"x": x})
    core_context.train.report_validation_metrics(steps_completed=steps_completed, metrics={"x": x})


if __name__ == "__main__":
    logging.basicConfig(level=logging.DEBUG, format=det.LOG_FORMAT)
    with core.init() as core_context:
        main(core_context=core_context, increment_by=1)
