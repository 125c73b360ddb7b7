"""Which tensor collectives a process group runs natively.

The production path (RCCL over xGMI, backend ``"nccl"``) uses the in-place tensor collectives:
``reduce_scatter_tensor`` into the rank's own slice of a flat gradient bucket,
``all_gather_into_tensor`` of parameter shards straight into the flat parameter buffer, and
``ReduceOp.AVG`` (the 1/world scaling folded into the collective). torch's gloo backend runs the
same three on HOST tensors (verified for in-place aliasing: the reduce-scatter output may be a view
into its input), so the CPU multi-rank tests execute exactly the code the 8-GPU run executes.
Only gloo with DEVICE tensors (two ranks sharing one GPU in the GPU test tier) falls back to
``all_reduce`` + slice / list ``all_gather``.
"""
from typing import Any

import torch
import torch.distributed as dist


def tensor_collectives(group: Any, device: torch.device) -> bool:
    """True when ``reduce_scatter_tensor`` / ``all_gather_into_tensor`` / ``ReduceOp.AVG`` run
    natively on ``group`` for tensors on ``device``."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    backend = dist.get_backend(group)
    if backend == "nccl":
        return True
    if backend == "gloo":
        return torch.device(device).type == "cpu" and hasattr(dist, "reduce_scatter_tensor") \
            and hasattr(dist, "all_gather_into_tensor")
    return False
