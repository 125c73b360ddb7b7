"""TensorBoard fetchers: sync trial event files from checkpoint storage into the TensorBoard
task's local directory (reference: ``harness/determined/tensorboard/fetchers/{__init__,base,s3,
gcs,azure,shared,directory}.py`` and ``exec/tensorboard.py:100-190``).

Every fetcher lists the storage paths it was given (``tensorboard/<cluster>/experiment/<id>``
relative to the storage root) and copies files that are new or changed since the last pass into
``<local_dir>/<path>``. Object stores (s3 / gcs / azure) go through the SDK-free REST clients of
``common/storage/_cloud.py``; a change is a new key or a new size (event files are append-only).
Shared-filesystem storage is copied by modification time.
"""
import os
import pathlib
import shutil
import threading
from typing import Any, Dict, List, Optional, Tuple, Type


class Fetcher:
    """Base: ``fetch_new()`` copies what changed and returns how many files it fetched."""

    def __init__(self, storage_config: Dict[str, Any], storage_paths: List[str], local_dir: str) -> None:
        self.storage_config = storage_config
        self.storage_paths = [p.strip("/") for p in storage_paths]
        self.local_dir = local_dir
        self._records: Dict[str, Any] = {}
        self._lock = threading.Lock()

    def _list(self, storage_path: str) -> List[Tuple[str, Any]]:
        """(relative file path under the storage root, change token) under ``storage_path``."""
        raise NotImplementedError

    def _fetch(self, rel: str, dst: str) -> None:
        raise NotImplementedError

    def fetch_new(self) -> int:
        n = 0
        with self._lock:
            for sp in self.storage_paths:
                for rel, token in self._list(sp):
                    if self._records.get(rel) == token:
                        continue
                    dst = os.path.join(self.local_dir, rel)
                    os.makedirs(os.path.dirname(dst), exist_ok=True)
                    tmp = dst + ".part"
                    self._fetch(rel, tmp)
                    os.replace(tmp, dst)
                    self._records[rel] = token
                    n += 1
        return n


class SharedFSFetcher(Fetcher):
    """``type: shared_fs`` (host_path [+ storage_path]) -- copy by mtime/size."""

    def _root(self) -> pathlib.Path:
        c = self.storage_config
        root = c.get("host_path") or c.get("container_path") or ""
        sp = c.get("storage_path")
        if sp:
            root = sp if os.path.isabs(sp) else os.path.join(root, sp)
        return pathlib.Path(root)

    def _list(self, storage_path: str) -> List[Tuple[str, Any]]:
        root = self._root()
        base = root / storage_path
        out = []
        if base.is_dir():
            for p in sorted(base.rglob("*")):
                if p.is_file():
                    st = p.stat()
                    out.append((str(p.relative_to(root)), (st.st_mtime_ns, st.st_size)))
        return out

    def _fetch(self, rel: str, dst: str) -> None:
        shutil.copyfile(self._root() / rel, dst)


class DirectoryFetcher(SharedFSFetcher):
    """``type: directory`` (container_path)."""

    def _root(self) -> pathlib.Path:
        return pathlib.Path(self.storage_config["container_path"])


class ObjectStoreFetcher(Fetcher):
    """``type: s3 | gcs | azure``: list keys under ``[<prefix>/]<path>/`` and download changed ones."""

    def __init__(self, storage_config: Dict[str, Any], storage_paths: List[str], local_dir: str,
                 manager: Any = None) -> None:
        super().__init__(storage_config, storage_paths, local_dir)
        if manager is None:
            from determined_clone_amd.common import storage

            manager = storage.build(storage_config)
        self.manager = manager

    def _list(self, storage_path: str) -> List[Tuple[str, Any]]:
        base = self.manager._key(storage_path) + "/"
        root = self.manager._key("")
        cut = len(root) + 1 if root else 0
        return [(k[cut:], size) for k, size in self.manager.store.list(base) if k.startswith(base)]

    def _fetch(self, rel: str, dst: str) -> None:
        self.manager.store.get(self.manager._key(rel), dst)


S3Fetcher = GCSFetcher = AzureFetcher = ObjectStoreFetcher

_FETCHERS: Dict[str, Type[Fetcher]] = {
    "s3": ObjectStoreFetcher,
    "gcs": ObjectStoreFetcher,
    "azure": ObjectStoreFetcher,
    "shared_fs": SharedFSFetcher,
    "directory": DirectoryFetcher,
}


def build(storage_config: Dict[str, Any], paths: List[str], local_dir: str,
          manager: Optional[Any] = None) -> Fetcher:
    t = storage_config.get("type")
    if t not in _FETCHERS:
        raise ValueError(f"checkpoint_storage type '{t}' is not supported")
    if manager is not None and _FETCHERS[t] is ObjectStoreFetcher:
        return ObjectStoreFetcher(storage_config, paths, local_dir, manager=manager)
    return _FETCHERS[t](storage_config, paths, local_dir)
