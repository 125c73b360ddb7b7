"""TensorBoard support without a TensorFlow dependency.

Reference: `harness/determined/tensorboard/*` (TensorboardManager that syncs event files to
checkpoint storage, metric writers for TF/PyTorch). TensorBoard/TF are not installed here, so the
event-file format is written natively: TFRecord framing (length, masked CRC32C) around hand-encoded
``Event``/``Summary`` protobuf messages (scalars). Files are readable by stock TensorBoard.
"""
import os
import pathlib
import shutil
import socket
import struct
import threading
import time
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple

# ----------------------------------------------------------------------------- CRC32C
_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    tbl = _CRC_TABLE
    for b in data:
        c = tbl[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ----------------------------------------------------------------------------- protobuf encoding
def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wire: int) -> bytes:
    return _varint((num << 3) | wire)


def _bytes_field(num: int, payload: bytes) -> bytes:
    return _field(num, 2) + _varint(len(payload)) + payload


def encode_scalar_event(tag: str, value: float, step: int, wall_time: Optional[float] = None) -> bytes:
    val = _bytes_field(1, tag.encode()) + _field(2, 5) + struct.pack("<f", float(value))
    summary = _bytes_field(1, val)
    ev = _field(1, 1) + struct.pack("<d", wall_time or time.time())
    ev += _field(2, 0) + _varint(int(step))
    ev += _bytes_field(5, summary)
    return ev


def encode_image_event(tag: str, png: bytes, height: int, width: int, step: int,
                       channels: int = 3, wall_time: Optional[float] = None) -> bytes:
    """Event with one Summary.Value.image (PNG-encoded) -- what TensorBoard's image dashboard
    reads (field numbers of tensorflow/core/framework/summary.proto)."""
    img = (_field(1, 0) + _varint(int(height)) + _field(2, 0) + _varint(int(width))
           + _field(3, 0) + _varint(int(channels)) + _bytes_field(4, png))
    val = _bytes_field(1, tag.encode()) + _bytes_field(4, img)
    ev = _field(1, 1) + struct.pack("<d", wall_time or time.time())
    ev += _field(2, 0) + _varint(int(step))
    ev += _bytes_field(5, _bytes_field(1, val))
    return ev


def encode_file_version_event() -> bytes:
    return _field(1, 1) + struct.pack("<d", time.time()) + _bytes_field(3, b"brain.Event:2")


def frame(record: bytes) -> bytes:
    header = struct.pack("<Q", len(record))
    return header + struct.pack("<I", _masked_crc(header)) + record + struct.pack("<I", _masked_crc(record))


def read_records(path: str):
    """Iterate raw records of an event file (used by tests and the tensorboard fetcher)."""
    with open(path, "rb") as f:
        while True:
            header = f.read(12)
            if len(header) < 12:
                return
            (n,) = struct.unpack("<Q", header[:8])
            data = f.read(n)
            f.read(4)
            yield data


class EventFileWriter:
    def __init__(self, logdir: str, suffix: str = "") -> None:
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}{suffix}"
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "ab")
        self._lock = threading.Lock()
        self._write(encode_file_version_event())

    def _write(self, rec: bytes) -> None:
        with self._lock:
            self._f.write(frame(rec))

    def add_scalar(self, tag: str, value: float, step: int) -> None:
        self._write(encode_scalar_event(tag, value, step))

    def add_image(self, tag: str, image: Any, step: int) -> None:
        """``image``: HxWx3 uint8 array-like (or a PIL image); stored PNG-encoded."""
        import io

        from PIL import Image

        im = image if hasattr(image, "save") else Image.fromarray(image)
        buf = io.BytesIO()
        im.save(buf, format="PNG")
        self._write(encode_image_event(tag, buf.getvalue(), im.height, im.width, step,
                                       len(im.getbands())))

    def flush(self) -> None:
        with self._lock:
            self._f.flush()

    def close(self) -> None:
        with self._lock:
            self._f.close()


class MetricWriter:
    """Writes reported training/validation metrics as scalars (reference: metric_writers)."""

    def __init__(self, logdir: str) -> None:
        self._w = EventFileWriter(logdir)

    def on_metrics(self, group: str, steps_completed: int, metrics: Dict[str, Any]) -> None:
        from determined_clone_amd.util import is_numerical_scalar, to_python

        prefix = "Determined/" if group == "training" else f"Determined/{group}_"
        for k, v in metrics.items():
            if is_numerical_scalar(v):
                self._w.add_scalar(prefix + k, float(to_python(v)), steps_completed)
        self._w.flush()

    def close(self) -> None:
        self._w.close()


class TensorboardManager:
    """Owns the local tensorboard directory of a trial and syncs it into storage."""

    def __init__(self, base_path: pathlib.Path, sync_path: Optional[pathlib.Path],
                 storage: Any = None, storage_prefix: Optional[str] = None) -> None:
        self.base_path = pathlib.Path(base_path)
        self.sync_path = sync_path
        # object storage (s3 / gcs / azure): files go up through the storage manager instead
        self.storage, self.storage_prefix = storage, storage_prefix
        self._uploaded: Dict[str, float] = {}
        self.base_path.mkdir(parents=True, exist_ok=True)
        self._writer: Optional[MetricWriter] = None

    def metric_writer(self) -> MetricWriter:
        if self._writer is None:
            self._writer = MetricWriter(str(self.base_path))
        return self._writer

    def start(self) -> None:
        pass

    def sync(self, selector: Optional[Callable[[str], bool]] = None, mangler: Any = None) -> None:
        if self.sync_path is None:
            if self.storage is not None and self.storage_prefix:
                # upload only files that changed since the last sync
                changed = [str(p.relative_to(self.base_path)) for p in self.base_path.rglob("*")
                           if p.is_file() and (selector is None or selector(str(p)))
                           and self._uploaded.get(str(p)) != p.stat().st_mtime]
                if changed:
                    self.storage.upload(str(self.base_path), self.storage_prefix, changed)
                    for rel in changed:
                        q = self.base_path / rel
                        self._uploaded[str(q)] = q.stat().st_mtime
            return
        self.sync_path.mkdir(parents=True, exist_ok=True)
        for p in self.base_path.rglob("*"):
            if p.is_file() and (selector is None or selector(str(p))):
                dst = self.sync_path / p.relative_to(self.base_path)
                dst.parent.mkdir(parents=True, exist_ok=True)
                shutil.copy2(p, dst)

    def close(self) -> None:
        if self._writer is not None:
            self._writer.close()
        self.sync()


def build(cluster_id: str, experiment_id: str, trial_id: str, storage_config: Dict[str, Any],
          rank: int = 0) -> Optional[TensorboardManager]:
    # per cluster + trial: a host that ran another cluster's "experiment 1 / trial 1" must not
    # upload that run's event files into this trial's TensorBoard directory
    base = pathlib.Path(os.environ.get("DET_TENSORBOARD_DIR",
                                       f"/tmp/tensorboard-{cluster_id[:8]}-{experiment_id}-{trial_id}"))
    rel = f"tensorboard/{cluster_id}/experiment/{experiment_id}/trial/{trial_id}"
    sync = None
    storage = None
    if storage_config.get("type") in ("shared_fs", "directory"):
        root = storage_config.get("host_path") or storage_config.get("container_path")
        if storage_config.get("storage_path"):
            root = os.path.join(root, storage_config["storage_path"])
        sync = pathlib.Path(root) / rel
    elif storage_config.get("type"):
        from determined_clone_amd.common import storage as storage_mod

        storage = storage_mod.build(storage_config)
    if rank != 0:
        return None
    return TensorboardManager(base, sync, storage, rel if storage is not None else None)


def get_metric_writer(logdir: str) -> MetricWriter:
    return MetricWriter(logdir)


# ------------------------------------------------------------------ reading (no TF/TB dependency)
def _read_varint(buf: bytes, i: int) -> Tuple[int, int]:
    shift = result = 0
    while True:
        b = buf[i]
        i += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, i
        shift += 7


def _fields(buf: bytes) -> Iterator[Tuple[int, int, Any]]:
    """(field number, wire type, value) of a protobuf message; length-delimited values are bytes."""
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        num, wire = key >> 3, key & 7
        if wire == 0:
            v, i = _read_varint(buf, i)
        elif wire == 1:
            v = buf[i:i + 8]
            i += 8
        elif wire == 2:
            n, i = _read_varint(buf, i)
            v = buf[i:i + n]
            i += n
        elif wire == 5:
            v = buf[i:i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wire}")
        yield num, wire, v


def decode_scalar_event(record: bytes) -> List[Tuple[str, int, float, float]]:
    """Event{wall_time=1, step=2, summary=5{value=1{tag=1, simple_value=2}}} -> [(tag, step,
    wall_time, value)]."""
    wall, step, out = 0.0, 0, []
    summaries = []
    for num, wire, v in _fields(record):
        if num == 1 and wire == 1:
            (wall,) = struct.unpack("<d", v)
        elif num == 2 and wire == 0:
            step = v
        elif num == 5 and wire == 2:
            summaries.append(v)
    for s in summaries:
        for num, wire, v in _fields(s):
            if num != 1 or wire != 2:
                continue
            tag, val = None, None
            for n2, w2, v2 in _fields(v):
                if n2 == 1 and w2 == 2:
                    tag = v2.decode("utf-8", "replace")
                elif n2 == 2 and w2 == 5:
                    (val,) = struct.unpack("<f", v2)
            if tag is not None and val is not None:
                out.append((tag, int(step), float(wall), float(val)))
    return out


def read_scalars(logdir: str) -> Dict[str, Dict[str, List[Tuple[int, float, float]]]]:
    """{run (relative dir): {tag: [(step, wall_time, value)]}} for every event file under logdir."""
    runs: Dict[str, Dict[str, List[Tuple[int, float, float]]]] = {}
    for root, _dirs, files in os.walk(logdir):
        for fn in sorted(files):
            if "tfevents" not in fn:
                continue
            run = os.path.relpath(root, logdir)
            tags = runs.setdefault(run, {})
            for rec in read_records(os.path.join(root, fn)):
                for tag, step, wall, val in decode_scalar_event(rec):
                    tags.setdefault(tag, []).append((step, wall, val))
    for tags in runs.values():
        for series in tags.values():
            series.sort()
    return runs


def decode_image_event(record: bytes) -> List[Tuple[str, int, float, Dict[str, Any]]]:
    """Event -> [(tag, step, wall_time, {"height", "width", "png"})] for its Summary.Value.image
    entries (summary.proto: Value.image = 4; Image{height=1, width=2, colorspace=3,
    encoded_image_string=4})."""
    wall, step, summaries, out = 0.0, 0, [], []
    for num, wire, v in _fields(record):
        if num == 1 and wire == 1:
            (wall,) = struct.unpack("<d", v)
        elif num == 2 and wire == 0:
            step = v
        elif num == 5 and wire == 2:
            summaries.append(v)
    for s in summaries:
        for num, wire, v in _fields(s):
            if num != 1 or wire != 2:
                continue
            tag, img = None, None
            for n2, w2, v2 in _fields(v):
                if n2 == 1 and w2 == 2:
                    tag = v2.decode("utf-8", "replace")
                elif n2 == 4 and w2 == 2:
                    img = {"height": 0, "width": 0, "png": b""}
                    for n3, w3, v3 in _fields(v2):
                        if n3 == 1 and w3 == 0:
                            img["height"] = v3
                        elif n3 == 2 and w3 == 0:
                            img["width"] = v3
                        elif n3 == 4 and w3 == 2:
                            img["png"] = bytes(v3)
            if tag is not None and img is not None:
                out.append((tag, int(step), float(wall), img))
    return out


def read_images(logdir: str) -> Dict[str, Dict[str, List[Tuple[int, float, Dict[str, Any]]]]]:
    """{run: {tag: [(step, wall_time, {"height", "width", "png"})]}} for every event file."""
    runs: Dict[str, Dict[str, List[Tuple[int, float, Dict[str, Any]]]]] = {}
    for root, _dirs, files in os.walk(logdir):
        for fn in sorted(files):
            if "tfevents" not in fn:
                continue
            run = os.path.relpath(root, logdir)
            for rec in read_records(os.path.join(root, fn)):
                for tag, step, wall, img in decode_image_event(rec):
                    runs.setdefault(run, {}).setdefault(tag, []).append((step, wall, img))
    for tags in runs.values():
        for series in tags.values():
            series.sort(key=lambda t: (t[0], t[1]))
    return runs
