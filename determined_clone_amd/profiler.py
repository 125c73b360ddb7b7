"""System + timing profiler (reference: `harness/determined/profiler.py`).

A background sampler thread records CPU / host-memory / network / disk (psutil) and, for AMD GPUs,
utilisation and VRAM from the amdgpu sysfs files (``gpu_busy_percent``, ``mem_info_vram_used``)
— no nvidia-smi / pynvml. Samples are batched and shipped to the master (or kept locally)."""
import contextlib
import glob
import os
import threading
import time
from typing import Any, Callable, Dict, Iterator, List, Optional

try:
    import psutil
except ImportError:  # pragma: no cover
    psutil = None


def amd_gpu_stats() -> List[Dict[str, float]]:
    out = []
    for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
        busy = os.path.join(dev, "gpu_busy_percent")
        used = os.path.join(dev, "mem_info_vram_used")
        total = os.path.join(dev, "mem_info_vram_total")
        if not os.path.exists(busy):
            continue
        try:
            rec = {"gpu_util": float(open(busy).read().strip())}
            if os.path.exists(used) and os.path.exists(total):
                u, t = float(open(used).read()), float(open(total).read())
                rec["gpu_free_memory"] = (t - u) / 2**30
                rec["gpu_memory_util"] = u / t if t else 0.0
            out.append(rec)
        except (OSError, ValueError):
            continue
    return out


def sample_system() -> Dict[str, Any]:
    s: Dict[str, Any] = {"time": time.time()}
    if psutil is not None:
        s["cpu_util_simple"] = psutil.cpu_percent(interval=None)
        vm = psutil.virtual_memory()
        s["free_memory"] = vm.available / 2**30
        net = psutil.net_io_counters()
        s["net_throughput_sent"] = float(net.bytes_sent)
        s["net_throughput_recv"] = float(net.bytes_recv)
        disk = psutil.disk_io_counters()
        if disk is not None:
            s["disk_iops"] = float(disk.read_count + disk.write_count)
            s["disk_throughput_read"] = float(disk.read_bytes)
            s["disk_throughput_write"] = float(disk.write_bytes)
    s["gpus"] = amd_gpu_stats()
    return s


class ProfilerAgent:
    def __init__(self, begin_on_batch: int = 0, end_after_batch: Optional[int] = None,
                 sync_timings: bool = True, interval_s: float = 1.0,
                 ship: Optional[Callable[[List[Dict[str, Any]]], None]] = None) -> None:
        self.begin_on_batch = begin_on_batch
        self.end_after_batch = end_after_batch
        self.sync_timings = sync_timings
        self.interval_s = interval_s
        self.ship = ship
        self.samples: List[Dict[str, Any]] = []
        self.timings: Dict[str, List[float]] = {}
        self._batch_idx = 0
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._sync_device: Optional[Callable[[], None]] = None

    def _active(self) -> bool:
        return self._batch_idx >= self.begin_on_batch and (
            self.end_after_batch is None or self._batch_idx <= self.end_after_batch)

    def update_batch_idx(self, idx: int) -> None:
        self._batch_idx = idx

    def _set_sync_device(self, fn: Callable[[], None]) -> None:
        self._sync_device = fn

    @contextlib.contextmanager
    def record_timing(self, name: str, requires_sync: bool = True, accumulate: bool = False) -> Iterator[None]:
        if not self._active():
            yield
            return
        if requires_sync and self.sync_timings and self._sync_device:
            self._sync_device()
        t0 = time.time()
        yield
        if requires_sync and self.sync_timings and self._sync_device:
            self._sync_device()
        self.timings.setdefault(name, []).append(time.time() - t0)

    def record_metric(self, name: str, value: float) -> None:
        if self._active():
            self.timings.setdefault(name, []).append(float(value))

    def _loop(self) -> None:
        batch: List[Dict[str, Any]] = []
        while not self._stop.wait(self.interval_s):
            if not self._active():
                continue
            batch.append(sample_system())
            if len(batch) >= 10:
                self._flush(batch)
                batch = []
        if batch:
            self._flush(batch)

    def _flush(self, batch: List[Dict[str, Any]]) -> None:
        self.samples.extend(batch)
        if self.ship is not None:
            try:
                self.ship(batch)
            except Exception:
                pass

    def __enter__(self) -> "ProfilerAgent":
        if psutil is not None:
            psutil.cpu_percent(interval=None)
        self._thread = threading.Thread(target=self._loop, daemon=True, name="det-profiler")
        self._thread.start()
        return self

    def __exit__(self, *a: Any) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)


class DummyProfilerAgent(ProfilerAgent):
    def __enter__(self) -> "ProfilerAgent":
        return self

    def __exit__(self, *a: Any) -> None:
        pass
