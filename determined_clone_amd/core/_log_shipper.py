"""Ship an unmanaged trial's stdout/stderr to the master's task logs (reference:
``harness/determined/core/_log_shipper.py``, ``_UnmanagedTrialLogShipper``).

Managed trials get their output collected by the agent; a process running off-cluster has no
agent, so the Core API tees ``sys.stdout`` / ``sys.stderr`` and a background thread posts the
buffered lines to ``POST /api/v1/task/logs`` about once a second (and once more on close)."""
import sys
import threading
import time
from typing import Any, List, Optional, TextIO


class _Tee:
    def __init__(self, inner: TextIO, shipper: "_UnmanagedTrialLogShipper", stdtype: str) -> None:
        self._inner = inner
        self._shipper = shipper
        self._stdtype = stdtype
        self._partial = ""

    def write(self, s: str) -> int:
        n = self._inner.write(s)
        text = self._partial + s
        *lines, self._partial = text.split("\n")
        for line in lines:
            self._shipper._add(line, self._stdtype)
        return n

    def flush(self) -> None:
        self._inner.flush()

    def __getattr__(self, name: str) -> Any:
        return getattr(self._inner, name)


class _UnmanagedTrialLogShipper:
    def __init__(self, *, session: Any, trial_id: int, task_id: str, distributed: Any = None,
                 period_s: float = 1.0) -> None:
        self._session = session
        self._trial_id = trial_id
        self._task_id = task_id
        self._rank = getattr(distributed, "rank", 0) if distributed is not None else 0
        self._period = period_s
        self._buf: List[dict] = []
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._saved: Optional[tuple] = None

    def _add(self, line: str, stdtype: str) -> None:
        with self._lock:
            self._buf.append({"task_id": self._task_id, "rank_id": self._rank, "log": line + "\n",
                              "timestamp": time.time(), "stdtype": stdtype, "source": "unmanaged",
                              "level": "ERROR" if stdtype == "stderr" else "INFO"})

    def _flush(self) -> None:
        with self._lock:
            batch, self._buf = self._buf, []
        if batch:
            try:
                self._session.post("/api/v1/task/logs", {"logs": batch})
            except Exception:  # the master being unreachable must not kill training
                pass

    def start(self) -> "_UnmanagedTrialLogShipper":
        self._saved = (sys.stdout, sys.stderr)
        sys.stdout = _Tee(sys.stdout, self, "stdout")  # type: ignore[assignment]
        sys.stderr = _Tee(sys.stderr, self, "stderr")  # type: ignore[assignment]

        def loop() -> None:
            while not self._stop.wait(self._period):
                self._flush()

        self._thread = threading.Thread(target=loop, daemon=True, name="log-shipper")
        self._thread.start()
        return self

    def close(self, *exc: Any) -> None:
        self._stop.set()
        if self._saved is not None:
            for tee in (sys.stdout, sys.stderr):
                if isinstance(tee, _Tee) and tee._partial:
                    self._add(tee._partial, tee._stdtype)
                    tee._partial = ""
            sys.stdout, sys.stderr = self._saved
            self._saved = None
        if self._thread is not None:
            self._thread.join(timeout=5)
        self._flush()
