"""Core API stage 4: distributed -- every rank works, the chief reports; gather/broadcast through
the DistributedContext (reference: core_api/4_distributed.py). Launch with
``python -m determined_clone_amd.launch.torch_distributed -- python3 4_distributed.py``."""
import logging
import time

import determined_clone_amd as det
from determined_clone_amd import core


def main(core_context: core.Context, increment_by: float) -> None:
    dist = core_context.distributed
    x, batch = 0.0, 0
    for op in core_context.searcher.operations():
        while batch < op.length:
            x += increment_by * (dist.rank + 1)
            batch += 1
            time.sleep(0.01)
            if batch % 10 == 0:
                all_x = dist.gather(x)
                if dist.rank == 0:
                    core_context.train.report_training_metrics(steps_completed=batch,
                                                               metrics={"x": sum(all_x)})
                    op.report_progress(batch)
        all_x = dist.gather(x)
        if dist.rank == 0:
            core_context.train.report_validation_metrics(steps_completed=batch, metrics={"x": sum(all_x)})
            op.report_completed(sum(all_x))


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format=det.LOG_FORMAT)
    distributed = core.DistributedContext.from_torch_distributed() if __import__("os").environ.get("WORLD_SIZE") else None
    info = det.get_cluster_info()
    hparams = info.trial.hparams if info else {"increment_by": 1.0}
    with core.init(distributed=distributed) as core_context:
        main(core_context, increment_by=float(hparams["increment_by"]))
