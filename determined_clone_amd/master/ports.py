"""Per-agent port registry (reference: `master/internal/portregistry/port_registry.go`).

A multi-container task rendezvouses (``torch.distributed.run`` c10d store, DeepSpeed launcher) on
a TCP port of its chief container's host. Two such tasks whose chief lands on the same agent --
e.g. two 2-node jobs sharing a node -- must not pick the same port, so the master hands out the
lowest free port of ``[base, base + span)`` per agent when the allocation starts and takes it back
when the allocation ends."""
import threading
from typing import Dict, Set, Tuple


class PortRegistry:
    def __init__(self, base: int = 29400, span: int = 600) -> None:
        self.base, self.span = base, span
        self._used: Dict[str, Set[int]] = {}
        self._owner: Dict[str, Tuple[str, int]] = {}
        self._lock = threading.Lock()

    def acquire(self, agent_id: str, alloc_id: str) -> int:
        with self._lock:
            if alloc_id in self._owner:
                return self._owner[alloc_id][1]
            used = self._used.setdefault(agent_id, set())
            for p in range(self.base, self.base + self.span):
                if p not in used:
                    used.add(p)
                    self._owner[alloc_id] = (agent_id, p)
                    return p
        raise RuntimeError(f"no free rendezvous port on agent {agent_id} in "
                           f"[{self.base}, {self.base + self.span})")

    def release(self, alloc_id: str) -> None:
        with self._lock:
            owner = self._owner.pop(alloc_id, None)
            if owner is not None:
                self._used.get(owner[0], set()).discard(owner[1])

    def in_use(self, agent_id: str) -> Set[int]:
        with self._lock:
            return set(self._used.get(agent_id, set()))
