"""Heartbeat for unmanaged/detached trials (reference: `harness/determined/core/_heartbeat.py`):
reports RUNNING periodically and the final state (COMPLETED / ERROR) on exit."""
import threading
from typing import Any, Optional


class _Heartbeat:
    def __init__(self, *, session: Any, trial_id: int, period_s: float = 30.0) -> None:
        self._session = session
        self._trial_id = trial_id
        self._period = period_s
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def _post(self, state: str) -> None:
        try:
            self._session.post(f"/api/v1/trials/{self._trial_id}/heartbeat", {"state": state})
        except Exception:
            pass

    def start(self) -> "_Heartbeat":
        def loop() -> None:
            while not self._stop.wait(self._period):
                self._post("RUNNING")

        self._post("RUNNING")
        self._thread = threading.Thread(target=loop, daemon=True, name="heartbeat")
        self._thread.start()
        return self

    def close(self, exc_type: Any = None, exc_val: Any = None, exc_tb: Any = None) -> None:
        self._stop.set()
        self._post("ERROR" if exc_type is not None else "COMPLETED")
