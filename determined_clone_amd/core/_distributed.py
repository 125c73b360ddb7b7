"""DistributedContext: rank topology + small object collectives for the Core API.

Reference: `harness/determined/core/_distributed.py` (ZMQ-based gather/allgather/broadcast between
the chief and workers, `from_horovod` / `from_deepspeed` / `from_torch_distributed`).

MI355X design: there is no separate ZMQ side channel. Object collectives ride on the same
``torch.distributed`` world the training uses, but on a dedicated gloo (CPU) process group so
that control-plane messages (metrics, searcher ops, preemption decisions) never serialise through
RCCL or touch HBM. One process per GPU; local == node-local ranks.
"""
import datetime
import logging
import os
from typing import Any, List, Optional

logger = logging.getLogger("determined_clone_amd.core")


class DistributedContext:
    """Topology and object collectives for one task (all ranks of all nodes)."""

    def __init__(self, *, rank: int, size: int, local_rank: int, local_size: int,
                 cross_rank: int, cross_size: int, chief_ip: Optional[str] = None,
                 pub_port: int = 12360, pull_port: int = 12376, port_offset: int = 0,
                 force_tcp: bool = False, _group: Any = None) -> None:
        self.rank = rank
        self.size = size
        self.local_rank = local_rank
        self.local_size = local_size
        self.cross_rank = cross_rank
        self.cross_size = cross_size
        self._chief_ip = chief_ip
        self._group = _group  # torch.distributed ProcessGroup (gloo) or None
        self._local_group = None
        self._closed = False
        self._owns_pg = False
        if size > 1 and _group is None:
            self._group = _new_object_group()
        if size > 1 and local_size < size:
            self._local_group = _node_local_group(cross_rank, local_size, cross_size)

    # ------------------------------------------------------------------ constructors
    @classmethod
    def from_torch_distributed(cls, chief_ip: Optional[str] = None) -> "DistributedContext":
        """Read topology from torchrun-style env vars (``RANK``, ``LOCAL_RANK``,
        ``WORLD_SIZE``, ``LOCAL_WORLD_SIZE``, ``GROUP_RANK``); ``torch.distributed`` must be
        initialised (or is initialised here with the gloo/nccl backend)."""
        import torch.distributed as dist

        rank = int(os.environ["RANK"])
        size = int(os.environ["WORLD_SIZE"])
        local_rank = int(os.environ.get("LOCAL_RANK", rank))
        local_size = int(os.environ.get("LOCAL_WORLD_SIZE", size))
        cross_rank = int(os.environ.get("GROUP_RANK", rank // max(local_size, 1)))
        cross_size = size // max(local_size, 1)
        owns = False
        if not dist.is_initialized():
            import torch

            backend = "nccl" if torch.cuda.is_available() else "gloo"
            if backend == "nccl":
                torch.cuda.set_device(local_rank)
            dist.init_process_group(backend=backend)
            owns = True
        ctx = cls(rank=rank, size=size, local_rank=local_rank, local_size=local_size,
                  cross_rank=cross_rank, cross_size=cross_size,
                  chief_ip=chief_ip or os.environ.get("MASTER_ADDR"))
        ctx._owns_pg = owns
        return ctx

    @classmethod
    def from_deepspeed(cls, chief_ip: Optional[str] = None) -> "DistributedContext":
        # The DeepSpeedTrial path in this framework is native ZeRO on torch.distributed.
        return cls.from_torch_distributed(chief_ip)

    @classmethod
    def from_horovod(cls, hvd: Any = None, chief_ip: Optional[str] = None) -> "DistributedContext":
        raise NotImplementedError(
            "Horovod is not part of the MI355X stack; use determined_clone_amd.launch.torch_distributed")

    # ------------------------------------------------------------------ topology
    def get_rank(self) -> int:
        return self.rank

    def get_local_rank(self) -> int:
        return self.local_rank

    def get_size(self) -> int:
        return self.size

    def get_local_size(self) -> int:
        return self.local_size

    def get_cross_rank(self) -> int:
        return self.cross_rank

    def get_cross_size(self) -> int:
        return self.cross_size

    def get_num_agents(self) -> int:
        return self.cross_size

    def close(self) -> None:
        """Release the gloo object-collective groups this context created (a worker that exits
        with a live gloo SUBGROUP can abort in the group's destructor -- "terminate called without
        an active exception" -- while a peer is still tearing down). The default process group is
        left up, also when ``from_torch_distributed`` initialised it (the reference's close()
        never tears torch.distributed down either): user code may still run collectives after the
        Core API context exits, and the process's exit releases it
        (``tests/test_distributed.py::test_default_group_survives_core_context_close`` exits
        straight after close() on 2 gloo ranks)."""
        if self._closed:
            return
        self._closed = True
        if self.size <= 1:
            return
        import torch.distributed as dist

        if not (dist.is_available() and dist.is_initialized()):
            return
        for g in (self._local_group, self._group):
            if g is not None:
                try:
                    dist.destroy_process_group(g)
                except Exception:  # noqa: BLE001 - teardown is best effort
                    pass
        self._local_group = self._group = None
        # The default process group stays up even when from_torch_distributed() created it (as the
        # reference's close() never tears torch.distributed down): user code may still run
        # collectives after the Core API context exits (a final barrier, DDP / engine teardown).
        # The process's exit releases it.

    # ------------------------------------------------------------------ collectives
    def _objs(self, obj: Any, group: Any) -> List[Any]:
        import torch.distributed as dist

        n = dist.get_world_size(group)
        out: List[Any] = [None] * n
        dist.all_gather_object(out, obj, group=group)
        return out

    def allgather(self, stuff: Any) -> List[Any]:
        if self.size == 1:
            return [stuff]
        return self._objs(stuff, self._group)

    def gather(self, stuff: Any) -> Optional[List[Any]]:
        """Chief gets the list of every rank's object; other ranks get None."""
        if self.size == 1:
            return [stuff]
        import torch.distributed as dist

        out: Optional[List[Any]] = [None] * self.size if self.rank == 0 else None
        dist.gather_object(stuff, out, dst=0, group=self._group)
        return out

    def broadcast(self, stuff: Any) -> Any:
        if self.size == 1:
            return stuff
        import torch.distributed as dist

        box = [stuff if self.rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=self._group)
        return box[0]

    def allgather_local(self, stuff: Any) -> List[Any]:
        if self.local_size == 1:
            return [stuff]
        if self._local_group is None:
            return self.allgather(stuff)
        return self._objs(stuff, self._local_group)

    def gather_local(self, stuff: Any) -> Optional[List[Any]]:
        allv = self.allgather_local(stuff)
        return allv if self.local_rank == 0 else None

    def broadcast_local(self, stuff: Any = None) -> Any:
        allv = self.allgather_local(stuff)
        return allv[0]

    def barrier(self) -> None:
        if self.size > 1:
            import torch.distributed as dist

            dist.barrier(group=self._group)


def _new_object_group() -> Any:
    import torch.distributed as dist

    if not dist.is_initialized():
        raise RuntimeError("torch.distributed must be initialised for a multi-rank DistributedContext")
    if dist.get_backend() == "gloo":
        return None  # the default group already is CPU/gloo
    return dist.new_group(backend="gloo", timeout=datetime.timedelta(minutes=30))


def _node_local_group(cross_rank: int, local_size: int, cross_size: int) -> Any:
    import torch.distributed as dist

    mine = None
    for node in range(cross_size):
        ranks = list(range(node * local_size, (node + 1) * local_size))
        g = dist.new_group(ranks=ranks, backend="gloo")
        if node == cross_rank:
            mine = g
    return mine


class DummyDistributedContext(DistributedContext):
    """Single-process context used off-cluster and for 1-slot trials."""

    def __init__(self) -> None:
        super().__init__(rank=0, size=1, local_rank=0, local_size=1, cross_rank=0, cross_size=1)
