"""PreemptContext (reference: `harness/determined/core/_preempt.py`).

The chief runs a watcher thread that long-polls the master's preemption signal for its allocation;
``should_preempt()`` is answered from the watcher's cached flag (never blocks a training step on
HTTP) and broadcast to workers in ``WorkersAskChief`` mode so every rank exits at the same step.
"""
import enum
import logging
import threading
from typing import Any, Optional

logger = logging.getLogger("determined_clone_amd.core")


class PreemptMode(enum.Enum):
    WorkersAskChief = "WORKERS_ASK_CHIEF"
    ChiefOnly = "CHIEF_ONLY"
    WorkersAskMaster = "WORKERS_ASK_MASTER"


class _PreemptionWatcher(threading.Thread):
    def __init__(self, session: Any, allocation_id: str, longpoll_s: int = 60) -> None:
        super().__init__(daemon=True, name="preemption-watcher")
        self._session = session
        self._allocation_id = allocation_id
        self._longpoll = longpoll_s
        self._should_preempt = False
        self._stop = threading.Event()

    def _get(self, timeout: int) -> bool:
        r = self._session.get(f"/api/v1/allocations/{self._allocation_id}/signals/preemption",
                              params={"timeout_seconds": timeout}, timeout=timeout + 30)
        return bool((r or {}).get("preempt"))

    def run(self) -> None:
        while not self._stop.is_set() and not self._should_preempt:
            try:
                if self._get(self._longpoll):
                    self._should_preempt = True
            except Exception as e:  # master restarts / transient errors: keep watching
                logger.debug(f"preemption watcher: {e}")
                self._stop.wait(1.0)

    def should_preempt(self) -> bool:
        return self._should_preempt

    def close(self) -> None:
        self._stop.set()


class PreemptContext:
    def __init__(self, session: Any, allocation_id: str, dist: Any,
                 preempt_mode: PreemptMode = PreemptMode.WorkersAskChief) -> None:
        self._session = session
        self._allocation_id = allocation_id
        self._dist = dist
        self._preempt_mode = PreemptMode(preempt_mode)
        self._watcher: Optional[_PreemptionWatcher] = None
        self._started = False
        self._ack_sent = False

    def start(self) -> "PreemptContext":
        if self._dist.rank == 0 or self._preempt_mode == PreemptMode.WorkersAskMaster:
            self._watcher = _PreemptionWatcher(self._session, self._allocation_id)
            self._watcher.start()
        self._started = True
        return self

    def close(self) -> None:
        if self._watcher is not None:
            self._watcher.close()

    def __enter__(self) -> "PreemptContext":
        return self.start()

    def __exit__(self, *_: Any) -> None:
        self.close()

    def should_preempt(self, auto_ack: bool = True) -> bool:
        if not self._started:
            raise RuntimeError("PreemptContext.should_preempt() called before start()")
        if self._watcher is not None:
            out = self._watcher.should_preempt()
            if auto_ack and out and not self._ack_sent:
                self.acknowledge_preemption_signal()
                self._ack_sent = True
            if self._preempt_mode == PreemptMode.WorkersAskChief:
                self._dist.broadcast(out)
            return out
        if self._preempt_mode == PreemptMode.ChiefOnly:
            raise RuntimeError("preempt_mode=ChiefOnly but should_preempt() called on a worker")
        return bool(self._dist.broadcast(None))

    def acknowledge_preemption_signal(self) -> None:
        self._session.post(f"/api/v1/allocations/{self._allocation_id}/signals/ack_preemption")


class DummyPreemptContext(PreemptContext):
    """Off-cluster: never preempts; ``_force()`` lets tests/users trigger it (e.g. on SIGTERM)."""

    def __init__(self, dist: Any, preempt_mode: PreemptMode = PreemptMode.WorkersAskChief) -> None:
        super().__init__(None, "", dist, preempt_mode)
        self._forced = False

    def _force(self) -> None:
        self._forced = True

    def start(self) -> "PreemptContext":
        self._started = True
        return self

    def close(self) -> None:
        pass

    def should_preempt(self, auto_ack: bool = True) -> bool:
        if not self._started:
            raise RuntimeError("PreemptContext.should_preempt() called before start()")
        out = self._forced
        if self._preempt_mode == PreemptMode.WorkersAskChief and self._dist.size > 1:
            out = bool(self._dist.broadcast(out))
        return out

    def acknowledge_preemption_signal(self) -> None:
        pass
