"""Prometheus endpoints of the master (reference: `master/internal/prom/det_state_metrics.go` and
the master's ``/debug/prom/metrics``).

* ``GET /prom/det-state-metrics`` -- cluster state as info-style gauges meant to be JOINED with
  device exporters: every running allocation's GPUs (``det_gpu_uuid_allocation`` carries the
  ``gpu_uuid`` label an amd-smi / ROCm exporter reports), allocation -> task / experiment / trial,
  per-agent slot counts, queue and experiment counts.
* ``GET /debug/prom/metrics`` -- the master process: API requests by handler / method / status
  and their latency, plus the client library's process collectors.

Both are unauthenticated, like the reference's (scrape them from inside the cluster network)."""
import time
from typing import Any, Tuple

from prometheus_client import CONTENT_TYPE_LATEST, CollectorRegistry, Counter, Gauge, Histogram
from prometheus_client import REGISTRY, generate_latest

API_REQUESTS = Counter("det_api_requests", "REST API requests handled by the master",
                       ["handler", "method", "code"])
API_SECONDS = Histogram("det_api_request_seconds", "REST API request latency", ["handler"],
                        buckets=(0.001, 0.005, 0.02, 0.1, 0.5, 2.0, 10.0, 60.0))


def observe(handler: str, method: str, code: int, started: float) -> None:
    API_REQUESTS.labels(handler, method, str(code)).inc()
    API_SECONDS.labels(handler).observe(time.time() - started)


def state_metrics(master: Any) -> Tuple[str, bytes]:
    reg = CollectorRegistry()
    slots = Gauge("det_agent_slots", "slots per agent by state", ["agent_id", "resource_pool", "state"], registry=reg)
    alloc = Gauge("det_allocation_info", "running allocations (value 1)",
                  ["allocation_id", "task_id", "task_type", "experiment_id", "trial_id"], registry=reg)
    gpu = Gauge("det_gpu_uuid_allocation", "GPU held by an allocation (value 1)",
                ["gpu_uuid", "agent_id", "slot_id", "allocation_id", "task_id"], registry=reg)
    queue = Gauge("det_queue_jobs", "allocation requests by state", ["resource_pool", "state"], registry=reg)
    exps = Gauge("det_experiments", "experiments by state", ["state"], registry=reg)
    rm = master.rm
    for a in list(rm.agents.values()):
        used = sum(1 for o in a.slot_owner if o)
        disabled = sum(1 for e in a.slot_enabled if not e)
        slots.labels(a.id, a.pool, "used").set(used)
        slots.labels(a.id, a.pool, "disabled").set(disabled)
        slots.labels(a.id, a.pool, "free").set(len(a.slots) - used - disabled)
    for al in list(master.allocations.values()):
        if al.exited or al.state == "PENDING":
            continue
        eid = str(al.exp.id) if getattr(al, "exp", None) is not None else ""
        tid = str(getattr(al.trial, "id", "") or "") if getattr(al, "trial", None) is not None else ""
        alloc.labels(al.id, al.task_id, al.kind, eid, tid).set(1)
        for p in al.placements:
            agent = rm.agents.get(p.get("agent_id"))
            for sid in p.get("slots") or []:
                dev = agent.slots[sid] if agent is not None and 0 <= sid < len(agent.slots) else {}
                gpu.labels(str(dev.get("uuid", "")), str(p.get("agent_id")), str(sid), al.id, al.task_id).set(1)
    for row in rm.queue():
        queue.labels(row["resource_pool"], row["state"]).inc()
    for row in master.db.all("SELECT state, COUNT(*) AS n FROM experiments GROUP BY state"):
        exps.labels(str(row["state"])).set(row["n"])
    return CONTENT_TYPE_LATEST, generate_latest(reg)


def process_metrics() -> Tuple[str, bytes]:
    return CONTENT_TYPE_LATEST, generate_latest(REGISTRY)
