"""Unmanaged distributed training: every rank joins one torch.distributed group (RCCL on
MI355X, gloo on CPU), the chief owns the trial, all ranks share the DistributedContext
(reference: examples/features/unmanaged/3_torch_distributed.py). Launch with
``python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 3_torch_distributed.py``."""
import os
from typing import Any, Optional

import torch
import torch.distributed as dist

from determined_clone_amd import core
from determined_clone_amd.experimental import core_v2


def main(steps: int = 50, client: Any = None) -> Optional[int]:
    backend = "nccl" if torch.cuda.is_available() else "gloo"
    if not dist.is_initialized():
        dist.init_process_group(backend)
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    distributed = core.DistributedContext.from_torch_distributed()
    core_v2.init(defaults=core_v2.DefaultConfig(name="unmanaged-3-torch-distributed"),
                 distributed=distributed, client=client)
    dev = torch.device("cuda") if backend == "nccl" else torch.device("cpu")
    w = torch.zeros(8, device=dev)
    for i in range(steps):
        # a stand-in for a gradient all-reduce: every rank contributes rank+1
        g = torch.full((8,), float(distributed.rank + 1), device=dev)
        dist.all_reduce(g)
        w -= 0.01 * g / distributed.size
        if (i + 1) % 10 == 0:
            losses = distributed.gather(float(w.abs().mean()))
            if distributed.rank == 0:
                core_v2.train.report_training_metrics(steps_completed=i,
                                                      metrics={"loss": sum(losses) / len(losses)})
    trial_id = core_v2.info.trial.trial_id if distributed.rank == 0 else None
    core_v2.close()
    return trial_id


if __name__ == "__main__":
    main()
