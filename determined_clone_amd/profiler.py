"""Trial profiler: system metrics + training-loop timings shipped to the master.

Reference: ``harness/determined/profiler.py`` (``ProfilerAgent`` :238-556, the collector / batcher
/ sender threads :602-924) and its call sites in ``pytorch/_pytorch_trial.py`` (:200-209, 883-932).

Behaviour kept from the reference:

* profiling runs only between ``begin_on_batch`` and ``end_after_batch`` (and at most
  ``MAX_COLLECTION_SECONDS`` after it began);
* system metrics are sampled on the local chief of every node (``local_rank == 0``): CPU %, free
  host memory (GB), network send / receive (Gbit/s), disk read / write (bytes/s) and IOPS, and per
  GPU utilisation (%) and free memory (GB) -- on MI355X from the amdgpu sysfs files through
  ``gpu.get_gpu_stats`` (no pynvml, no rocm-smi, no HIP initialisation);
* timings (``record_timing``) and misc metrics (``record_metric``, e.g. ``samples_per_second``)
  are recorded on the global chief while training; ``accumulate=True`` timings are summed per batch;
* everything is grouped into per-series batches ``{values, batches, timestamps, labels}`` (labels:
  trialId, name, agentId, gpuUuid, metricType) and POSTed to ``/api/v1/trials/profiler/metrics``
  off the training thread;
* a restarted trial that already has profiler data does not profile again.

Design differences: one sampler thread and one shipping thread (the reference uses three threads
and message objects); the sender is a plain callable so tests and the Core API can substitute it.
"""
import contextlib
import datetime
import logging
import queue
import threading
import time
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple

try:
    import psutil
except ImportError:  # pragma: no cover
    psutil = None

logger = logging.getLogger("determined_clone_amd.profiler")

MAX_COLLECTION_SECONDS = 300
SYSTEM = "PROFILER_METRIC_TYPE_SYSTEM"
TIMING = "PROFILER_METRIC_TYPE_TIMING"
MISC = "PROFILER_METRIC_TYPE_MISC"

GIGA = 1_000_000_000


class SysMetricName:
    GPU_UTIL_METRIC = "gpu_util"
    GPU_FREE_MEMORY_METRIC = "gpu_free_memory"
    NET_THRU_SENT_METRIC = "net_throughput_sent"
    NET_THRU_RECV_METRIC = "net_throughput_recv"
    DISK_IOPS_METRIC = "disk_iops"
    DISK_THRU_READ_METRIC = "disk_throughput_read"
    DISK_THRU_WRITE_METRIC = "disk_throughput_write"
    FREE_MEM_METRIC = "free_memory"
    SIMPLE_CPU_UTIL_METRIC = "cpu_util_simple"


SendBatchFn = Callable[[List[Dict[str, Any]]], None]
CheckExistsFn = Callable[[], bool]


def _iso(ts: float) -> str:
    return datetime.datetime.fromtimestamp(ts, datetime.timezone.utc).isoformat()


class MetricBatch:
    """Measurements grouped by series (metric type, name, gpu uuid) until consumed."""

    def __init__(self, trial_id: int, agent_id: str) -> None:
        self.trial_id = trial_id
        self.agent_id = agent_id
        self._series: Dict[Tuple[str, str, str], List[Tuple[float, int, float]]] = {}

    def append(self, metric_type: str, name: str, ts: float, batch_idx: int, value: float,
               gpu_uuid: str = "") -> None:
        self._series.setdefault((metric_type, name, gpu_uuid), []).append((ts, batch_idx, float(value)))

    def isempty(self) -> bool:
        return not any(self._series.values())

    def consume(self) -> List[Dict[str, Any]]:
        out = []
        for (mtype, name, uuid), pts in self._series.items():
            if not pts:
                continue
            out.append({
                "values": [p[2] for p in pts],
                "batches": [p[1] for p in pts],
                "timestamps": [_iso(p[0]) for p in pts],
                "labels": {"trialId": self.trial_id, "name": name, "agentId": self.agent_id,
                           "gpuUuid": uuid, "metricType": mtype},
            })
        self._series = {}
        return out


class _Rate:
    """Counter -> per-second rate since the previous reading (first reading discarded)."""

    def __init__(self, multiplier: float = 1.0) -> None:
        self.multiplier = multiplier
        self.t: Optional[float] = None
        self.v = 0.0

    def add(self, value: float, now: float) -> Optional[float]:
        rate = None
        if self.t is not None and now > self.t:
            rate = (value - self.v) / (now - self.t) * self.multiplier
        self.t, self.v = now, value
        return rate


class SystemSampler:
    """One reading of every system metric per call (rates relative to the previous call)."""

    def __init__(self) -> None:
        self.net_sent = _Rate(8 / GIGA)
        self.net_recv = _Rate(8 / GIGA)
        self.disk_read = _Rate()
        self.disk_write = _Rate()
        self.iops = _Rate()
        if psutil is not None:
            psutil.cpu_percent(interval=None)

    def sample(self, batch: MetricBatch, batch_idx: int) -> None:
        from determined_clone_amd import gpu

        now = time.time()
        if psutil is not None:
            batch.append(SYSTEM, SysMetricName.SIMPLE_CPU_UTIL_METRIC, now, batch_idx,
                         psutil.cpu_percent(interval=None))
            batch.append(SYSTEM, SysMetricName.FREE_MEM_METRIC, now, batch_idx,
                         psutil.virtual_memory().available / GIGA)
            net = psutil.net_io_counters()
            for rate, val, name in ((self.net_sent, net.bytes_sent, SysMetricName.NET_THRU_SENT_METRIC),
                                    (self.net_recv, net.bytes_recv, SysMetricName.NET_THRU_RECV_METRIC)):
                r = rate.add(float(val), now)
                if r is not None:
                    batch.append(SYSTEM, name, now, batch_idx, r)
            disk = psutil.disk_io_counters()
            if disk is not None:
                for rate, val, name in (
                        (self.disk_read, disk.read_bytes, SysMetricName.DISK_THRU_READ_METRIC),
                        (self.disk_write, disk.write_bytes, SysMetricName.DISK_THRU_WRITE_METRIC),
                        (self.iops, disk.read_count + disk.write_count, SysMetricName.DISK_IOPS_METRIC)):
                    r = rate.add(float(val), now)
                    if r is not None:
                        batch.append(SYSTEM, name, now, batch_idx, r)
        try:
            for g in gpu.get_gpu_stats():
                batch.append(SYSTEM, SysMetricName.GPU_UTIL_METRIC, now, batch_idx, g.util_percent, g.uuid)
                batch.append(SYSTEM, SysMetricName.GPU_FREE_MEMORY_METRIC, now, batch_idx,
                             g.free_memory_gb, g.uuid)
        except Exception as e:  # noqa: BLE001 - a sysfs hiccup must not stop the sampler
            logger.debug(f"gpu stats: {e}")


def sample_system() -> Dict[str, Any]:
    """One flat reading of the system metrics (for ad-hoc use and the tests)."""
    b = MetricBatch(0, "")
    SystemSampler().sample(b, 0)
    out: Dict[str, Any] = {"time": time.time(), "gpus": []}
    for s in b.consume():
        lab = s["labels"]
        if lab["gpuUuid"]:
            continue
        out[lab["name"]] = s["values"][-1]
    from determined_clone_amd import gpu

    out["gpus"] = [{"uuid": g.uuid, "gpu_util": g.util_percent, "gpu_free_memory": g.free_memory_gb}
                   for g in gpu.get_gpu_stats()]
    return out


class ProfilerAgent:
    """Collects system metrics and timings between ``begin_on_batch`` and ``end_after_batch`` and
    ships them with ``send_batch_fn`` (a callable taking a list of series batches). With
    ``profiling_is_enabled=False`` every method is a no-op and no thread is started."""

    MEASUREMENT_INTERVAL = 0.1
    FLUSH_INTERVAL = 10.0

    def __init__(self, trial_id: int = 0, agent_id: str = "", profiling_is_enabled: bool = True,
                 global_rank: int = 0, local_rank: int = 0, begin_on_batch: int = 0,
                 sync_timings: bool = True, end_after_batch: Optional[int] = None,
                 send_batch_fn: Optional[SendBatchFn] = None,
                 check_data_exists_fn: Optional[CheckExistsFn] = None,
                 measurement_interval: Optional[float] = None,
                 flush_interval: Optional[float] = None,
                 max_collection_seconds: float = MAX_COLLECTION_SECONDS) -> None:
        self.trial_id = trial_id
        self.agent_id = agent_id
        self.enabled_in_config = profiling_is_enabled
        self.global_rank = global_rank
        self.local_rank = local_rank
        self.begin_on_batch = begin_on_batch
        self.end_after_batch = end_after_batch
        self.sync_timings = sync_timings
        self.send_batch_fn = send_batch_fn
        self.measurement_interval = measurement_interval or self.MEASUREMENT_INTERVAL
        self.flush_interval = flush_interval or self.FLUSH_INTERVAL
        self.max_collection_seconds = max_collection_seconds
        self.current_batch_idx = 0
        self.training = False
        self.has_started = False
        self.has_finished = False
        self.disabled_due_to_preexisting_metrics = False
        self.sync_device: Optional[Callable[[], None]] = None
        self.shipped: List[Dict[str, Any]] = []  # everything sent (kept for local inspection)
        self._lock = threading.Lock()
        self._timings = MetricBatch(trial_id, agent_id)
        self._accum: Dict[str, Tuple[float, int, float]] = {}
        self._stop = threading.Event()
        self._active_evt = threading.Event()
        self._send_q: "queue.Queue[Optional[List[Dict[str, Any]]]]" = queue.Queue()
        self._threads: List[threading.Thread] = []
        self._started_at = 0.0
        if self.enabled_in_config and check_data_exists_fn is not None:
            try:
                self.disabled_due_to_preexisting_metrics = bool(check_data_exists_fn())
            except Exception as e:  # noqa: BLE001
                logger.warning(f"profiler: could not check for existing data: {e}")
            if self.disabled_due_to_preexisting_metrics and global_rank == 0:
                logger.warning("ProfilerAgent is disabled because profiling data for this trial already "
                               "exists. No additional profiling data is generated after a restart.")

    # ------------------------------------------------------------------ construction helpers
    @staticmethod
    def from_config(profiling: Dict[str, Any], trial_id: int, agent_id: str, global_rank: int,
                    local_rank: int, session: Any = None) -> "ProfilerAgent":
        """The agent a managed trial builds from the expconf ``profiling`` section; ``session``
        (common.api.Session) ships to the master."""
        send = check = None
        if session is not None:
            def send(batches: List[Dict[str, Any]]) -> None:
                session.post("/api/v1/trials/profiler/metrics", {"batches": batches})

            def check() -> bool:
                r = session.get(f"/api/v1/trials/{trial_id}/profiler/available_series")
                return bool(r.get("labels"))
        return ProfilerAgent(trial_id=trial_id, agent_id=agent_id,
                             profiling_is_enabled=bool(profiling.get("enabled", False)),
                             global_rank=global_rank, local_rank=local_rank,
                             begin_on_batch=int(profiling.get("begin_on_batch") or 0),
                             end_after_batch=profiling.get("end_after_batch"),
                             sync_timings=bool(profiling.get("sync_timings", True)),
                             send_batch_fn=send, check_data_exists_fn=check)

    def _set_sync_device(self, fn: Callable[[], None]) -> None:
        self.sync_device = fn

    # ------------------------------------------------------------------ state
    @property
    def is_enabled(self) -> bool:
        if not self.enabled_in_config or self.disabled_due_to_preexisting_metrics:
            return False
        return self.sysmetrics_is_enabled or self.global_rank == 0

    @property
    def sysmetrics_is_enabled(self) -> bool:
        return (self.enabled_in_config and not self.disabled_due_to_preexisting_metrics
                and self.local_rank == 0)

    @property
    def timings_is_enabled(self) -> bool:
        return (self.enabled_in_config and not self.disabled_due_to_preexisting_metrics
                and self.training and self.global_rank == 0)

    @property
    def is_active(self) -> bool:
        return self.is_enabled and self.has_started and not self.has_finished

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        if not self.is_enabled or self._threads:
            return
        t = threading.Thread(target=self._ship_loop, daemon=True, name="det-profiler-sender")
        t.start()
        self._threads.append(t)
        if self.sysmetrics_is_enabled:
            s = threading.Thread(target=self._sample_loop, daemon=True, name="det-profiler-sysmetrics")
            s.start()
            self._threads.append(s)
        if self.current_batch_idx >= self.begin_on_batch:
            self._begin_collection()

    def end(self) -> None:
        if not self.is_enabled:
            return
        self._end_collection()

    def __enter__(self) -> "ProfilerAgent":
        self.start()
        return self

    def __exit__(self, *a: Any) -> None:
        self.end()

    def set_training(self, training: bool) -> None:
        if not self.is_enabled:
            return
        if not training:
            self._finalize_batch()
        self.training = training

    def update_batch_idx(self, new_batch_idx: int) -> None:
        if not self.is_enabled:
            return
        if new_batch_idx < self.current_batch_idx:
            raise ValueError("Batch index should never decrease over time")
        if self.timings_is_enabled:
            self._finalize_batch()
        self.current_batch_idx = new_batch_idx
        if not self.has_started and new_batch_idx >= self.begin_on_batch and self._threads:
            self._begin_collection()
        if self.is_active and self.end_after_batch is not None and new_batch_idx > self.end_after_batch:
            self._end_collection()

    # ------------------------------------------------------------------ recording
    def record_metric(self, metric_name: str, value: float) -> None:
        if not (self.is_active and self.timings_is_enabled):
            return
        with self._lock:
            self._timings.append(MISC, metric_name, time.time(), self.current_batch_idx, value)

    @contextlib.contextmanager
    def record_timing(self, metric_name: str, accumulate: bool = False,
                      requires_sync: bool = True) -> Iterator[None]:
        if (not self.is_active or not self.timings_is_enabled
                or (requires_sync and not self.sync_timings)):
            yield
            return
        t0 = time.time()
        yield
        if self.sync_timings and self.sync_device is not None:
            self.sync_device()
        dt = time.time() - t0
        with self._lock:
            if accumulate:
                prev = self._accum.get(metric_name)
                self._accum[metric_name] = (t0, self.current_batch_idx, dt + (prev[2] if prev else 0.0))
            else:
                self._timings.append(TIMING, metric_name, t0, self.current_batch_idx, dt)

    def _finalize_batch(self) -> None:
        with self._lock:
            for name, (ts, b, v) in self._accum.items():
                self._timings.append(TIMING, name, ts, b, v)
            self._accum = {}

    # ------------------------------------------------------------------ threads
    def _begin_collection(self) -> None:
        self.has_started = True
        self._started_at = time.time()
        self._active_evt.set()

    def _end_collection(self) -> None:
        with self._lock:
            if self.has_finished:
                return
            self.has_finished = True
        self._finalize_batch()
        self._stop.set()
        self._active_evt.set()  # wake a sampler still waiting for begin_on_batch
        for t in self._threads:
            if t.name == "det-profiler-sysmetrics":
                t.join(timeout=10)
        with self._lock:
            pending = self._timings.consume()
        if pending:
            self._send_q.put(pending)
        self._send_q.put(None)
        for t in self._threads:
            if t.name == "det-profiler-sender":
                t.join(timeout=30)

    def _sample_loop(self) -> None:
        self._active_evt.wait()
        if self._stop.is_set():
            return
        sampler = SystemSampler()
        batch = MetricBatch(self.trial_id, self.agent_id)
        last_flush = time.time()
        nxt = time.time()
        while not self._stop.wait(max(0.0, nxt - time.time())):
            nxt += self.measurement_interval
            sampler.sample(batch, self.current_batch_idx)
            if time.time() - last_flush >= self.flush_interval:
                self._send_q.put(batch.consume())
                last_flush = time.time()
            if time.time() - self._started_at > self.max_collection_seconds:
                threading.Thread(target=self._end_collection, daemon=True).start()
                break
        rest = batch.consume()
        if rest:
            self._send_q.put(rest)

    def _ship_loop(self) -> None:
        last = time.time()
        while True:
            try:
                item = self._send_q.get(timeout=max(0.05, self.flush_interval - (time.time() - last)))
            except queue.Empty:
                item = []
            if item is None:
                return
            if time.time() - last >= self.flush_interval:
                with self._lock:
                    item = item + self._timings.consume()
                last = time.time()
            if item:
                self._send(item)

    def _send(self, batches: List[Dict[str, Any]]) -> None:
        self.shipped.extend(batches)
        if self.send_batch_fn is None:
            return
        for attempt in range(2):
            try:
                self.send_batch_fn(batches)
                return
            except Exception as e:  # noqa: BLE001 - profiling never fails the trial
                if attempt == 1:
                    logger.warning(f"profiler: dropping {len(batches)} series batch(es): {e}")
                else:
                    time.sleep(1.0)


class DummyProfilerAgent(ProfilerAgent):
    """The disabled agent (every method a no-op)."""

    def __init__(self) -> None:
        super().__init__(profiling_is_enabled=False)
