"""Unmanaged experiment with checkpoints and resume: the external experiment/trial ids make a
second run of this script attach to the same trial and continue from its latest checkpoint
(reference: examples/features/unmanaged/2_checkpoints.py)."""
import random
from typing import Any, Tuple

from determined_clone_amd.experimental import core_v2


def main(steps: int = 100, client: Any = None,
         external_id: str = "test-unmanaged-2-checkpoints") -> Tuple[int, int]:
    """Returns (trial id, first step of this run)."""
    core_v2.init(
        defaults=core_v2.DefaultConfig(name="unmanaged-2-checkpoints"),
        unmanaged=core_v2.UnmanagedConfig(external_experiment_id=external_id,
                                          external_trial_id=external_id),
        client=client,
    )
    initial_i = 0
    latest = core_v2.info.latest_checkpoint
    if latest is not None:
        with core_v2.checkpoint.restore_path(latest) as path:
            i_str, _ = (path / "state").read_text().split(",")
            initial_i = int(i_str) + 1
    print("initial step:", initial_i, flush=True)
    for i in range(initial_i, initial_i + steps):
        core_v2.train.report_training_metrics(steps_completed=i, metrics={"loss": random.random()})
        if (i + 1) % 10 == 0:
            loss = random.random()
            core_v2.train.report_validation_metrics(steps_completed=i, metrics={"loss": loss})
            with core_v2.checkpoint.store_path({"steps_completed": i}) as (path, _uuid):
                (path / "state").write_text(f"{i},{loss}")
    trial_id = core_v2.info.trial.trial_id
    core_v2.close()
    return trial_id, initial_i


if __name__ == "__main__":
    main()
