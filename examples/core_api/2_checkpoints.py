"""Core API stage 2: checkpoints + pause/resume via preemption (reference: core_api/2_checkpoints.py)."""
import json
import logging
import pathlib
import time

import determined_clone_amd as det
from determined_clone_amd import core


def save_state(x: int, steps_completed: int, trial_id: int, checkpoint_directory: pathlib.Path) -> None:
    (checkpoint_directory / "state").write_text(json.dumps({"x": x, "steps_completed": steps_completed,
                                                            "trial_id": trial_id}))


def load_state(trial_id: int, checkpoint_directory: pathlib.Path):
    st = json.loads((checkpoint_directory / "state").read_text())
    if st["trial_id"] != trial_id:  # a new trial continuing from another trial's checkpoint
        return st["x"], 0
    return st["x"], st["steps_completed"]


def main(core_context: core.Context, latest_checkpoint, trial_id: int, increment_by: int) -> None:
    x, starting_batch = 0, 0
    if latest_checkpoint is not None:
        with core_context.checkpoint.restore_path(latest_checkpoint) as path:
            x, starting_batch = load_state(trial_id, path)
    steps_completed = starting_batch
    for batch in range(starting_batch, 100):
        x += increment_by
        steps_completed = batch + 1
        time.sleep(0.01)
        if steps_completed % 10 == 0:
            core_context.train.report_training_metrics(steps_completed=steps_completed, metrics={"x": x})
            with core_context.checkpoint.store_path({"steps_completed": steps_completed}) as (path, uuid):
                save_state(x, steps_completed, trial_id, path)
            if core_context.preempt.should_preempt():
                return
    core_context.train.report_validation_metrics(steps_completed=steps_completed, metrics={"x": x})


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format=det.LOG_FORMAT)
    info = det.get_cluster_info()
    latest = info.latest_checkpoint if info else None
    trial_id = info.trial.trial_id if info else -1
    with core.init() as core_context:
        main(core_context, latest, trial_id, increment_by=1)
