"""Unmanaged experiment, singleton style: an ordinary script (not launched by the master) reports
training/validation metrics as a trial of a new experiment (reference:
examples/features/unmanaged/1_singleton.py). Set ``DET_MASTER`` and run ``python 1_singleton.py``."""
import random
from typing import Any

from determined_clone_amd.experimental import core_v2


def main(steps: int = 100, client: Any = None) -> int:
    core_v2.init(defaults=core_v2.DefaultConfig(name="unmanaged-1-singleton"), client=client)
    trial_id = core_v2.info.trial.trial_id
    for i in range(steps):
        core_v2.train.report_training_metrics(steps_completed=i, metrics={"loss": random.random()})
        if (i + 1) % 10 == 0:
            core_v2.train.report_validation_metrics(steps_completed=i,
                                                    metrics={"loss": random.random()})
    core_v2.close()
    return trial_id


if __name__ == "__main__":
    main()
