"""Wait for a freshly deployed master to answer (reference: `deploy/healthcheck.py`)."""
import time
from typing import Callable, Optional

import requests


def wait_for_master(master_url: str, timeout: float = 300.0, interval: float = 2.0,
                    log: Optional[Callable[[str], None]] = None,
                    session: Optional[requests.Session] = None) -> dict:
    """Poll ``GET /api/v1/master`` until it answers 200; returns its info or raises TimeoutError."""
    http = session or requests.Session()
    deadline = time.time() + timeout
    url = master_url.rstrip("/") + "/api/v1/master"
    last = ""
    while True:
        try:
            r = http.get(url, timeout=min(10.0, max(1.0, interval * 2)))
            if r.status_code == 200:
                return r.json()
            last = f"HTTP {r.status_code}"
        except requests.RequestException as e:
            last = type(e).__name__
        if time.time() >= deadline:
            raise TimeoutError(f"master at {master_url} not healthy after {timeout:.0f}s ({last})")
        if log:
            log(f"waiting for master at {master_url} ({last})")
        time.sleep(interval)


def wait_for_agents(master_url: str, token: str, n: int, timeout: float = 600.0,
                    interval: float = 5.0, session: Optional[requests.Session] = None) -> int:
    """Poll ``GET /api/v1/agents`` until ``n`` agents are registered; returns the count."""
    http = session or requests.Session()
    deadline = time.time() + timeout
    while True:
        r = http.get(master_url.rstrip("/") + "/api/v1/agents", timeout=10,
                     headers={"Authorization": f"Bearer {token}"})
        got = len(r.json().get("agents", [])) if r.status_code == 200 else 0
        if got >= n:
            return got
        if time.time() >= deadline:
            raise TimeoutError(f"{got}/{n} agents registered after {timeout:.0f}s")
        time.sleep(interval)
