"""Checkpoint storage managers (reference: `harness/determined/common/storage/*`).

``shared_fs`` and ``directory`` write straight into the target directory (no staging copy — on a
single MI355X node the checkpoint directory IS the storage). Cloud backends (s3/gcs/azure) speak
their REST protocols directly (``_cloud.py``: SigV4, Azure SharedKey/SAS, GCS JSON API) -- no
vendor SDK is needed.
"""
import contextlib
import os
import pathlib
import shutil
import tempfile
from typing import Any, Callable, Dict, Iterator, List, Optional, Union

Selector = Optional[Callable[[str], bool]]


class StorageManager:
    """Base class. ``storage_id`` is the checkpoint UUID (a directory name)."""

    def __init__(self, base_path: str) -> None:
        self._base_path = str(base_path)

    # --- interface
    def upload(self, src: Union[str, os.PathLike], dst: str, paths: Optional[List[str]] = None) -> None:
        raise NotImplementedError

    def download(self, src: str, dst: Union[str, os.PathLike], selector: Selector = None) -> None:
        raise NotImplementedError

    def delete(self, storage_id: str, globs: Optional[List[str]] = None) -> Dict[str, int]:
        raise NotImplementedError

    def list_files(self, storage_id: str) -> Dict[str, int]:
        raise NotImplementedError

    def store_path_is_direct_access(self) -> bool:
        """True when ``store_path`` yields the storage location itself (files written there ARE
        the checkpoint; sharded writers share it). Object stores stage locally and upload."""
        return False

    def pre_store_path(self, dst: str) -> pathlib.Path:
        """A fresh local staging directory for one writer of checkpoint ``dst``."""
        return pathlib.Path(tempfile.mkdtemp(prefix=f"dca-ckpt-{dst[:8]}-"))

    def post_store_path(self, path: Union[str, os.PathLike]) -> None:
        """Remove a staging directory from :meth:`pre_store_path` (after its upload)."""
        shutil.rmtree(path, ignore_errors=True)

    @contextlib.contextmanager
    def store_path(self, dst: str) -> Iterator[pathlib.Path]:
        tmp = tempfile.mkdtemp(prefix="dca-ckpt-")
        try:
            yield pathlib.Path(tmp)
            self.upload(tmp, dst)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)

    @contextlib.contextmanager
    def restore_path(self, src: str, selector: Selector = None) -> Iterator[pathlib.Path]:
        tmp = tempfile.mkdtemp(prefix="dca-restore-")
        try:
            self.download(src, tmp, selector)
            yield pathlib.Path(tmp)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)


def _walk(root: str) -> Dict[str, int]:
    out: Dict[str, int] = {}
    for dirpath, dirnames, filenames in os.walk(root):
        rel = os.path.relpath(dirpath, root)
        if rel != ".":
            out[rel + "/"] = 0
        for f in filenames:
            p = os.path.join(dirpath, f)
            out[os.path.normpath(os.path.join(rel, f))] = os.path.getsize(p)
    return out


class SharedFSStorageManager(StorageManager):
    """Checkpoints are directories under ``base_path``."""

    def __init__(self, base_path: str) -> None:
        super().__init__(base_path)
        os.makedirs(self._base_path, exist_ok=True)

    def store_path_is_direct_access(self) -> bool:
        return True

    def pre_store_path(self, dst: str) -> pathlib.Path:
        p = self.path(dst)
        p.mkdir(parents=True, exist_ok=True)
        return p

    def post_store_path(self, path: Union[str, os.PathLike]) -> None:
        pass  # the checkpoint directory itself

    def path(self, storage_id: str) -> pathlib.Path:
        return pathlib.Path(self._base_path) / storage_id

    def upload(self, src, dst, paths=None) -> None:
        target = self.path(dst)
        target.mkdir(parents=True, exist_ok=True)
        src = pathlib.Path(src)
        files = paths if paths is not None else [str(p.relative_to(src)) for p in src.rglob("*")]
        for rel in files:
            s = src / rel
            d = target / rel
            if s.is_dir():
                d.mkdir(parents=True, exist_ok=True)
            elif s.exists():
                d.parent.mkdir(parents=True, exist_ok=True)
                shutil.copy2(s, d)

    def download(self, src, dst, selector=None) -> None:
        root = self.path(src)
        if not root.exists():
            from determined_clone_amd.errors import CheckpointNotFoundException

            raise CheckpointNotFoundException(f"checkpoint {src} not found in {self._base_path}")
        dst = pathlib.Path(dst)
        for p in root.rglob("*"):
            rel = str(p.relative_to(root))
            if selector is not None and not selector(rel + ("/" if p.is_dir() else "")):
                continue
            d = dst / rel
            if p.is_dir():
                d.mkdir(parents=True, exist_ok=True)
            else:
                d.parent.mkdir(parents=True, exist_ok=True)
                shutil.copy2(p, d)

    @contextlib.contextmanager
    def store_path(self, dst: str) -> Iterator[pathlib.Path]:
        p = self.path(dst)
        p.mkdir(parents=True, exist_ok=True)
        yield p

    @contextlib.contextmanager
    def restore_path(self, src: str, selector: Selector = None) -> Iterator[pathlib.Path]:
        p = self.path(src)
        if not p.exists():
            from determined_clone_amd.errors import CheckpointNotFoundException

            raise CheckpointNotFoundException(f"checkpoint {src} not found in {self._base_path}")
        yield p

    def delete(self, storage_id: str, globs: Optional[List[str]] = None) -> Dict[str, int]:
        root = self.path(storage_id)
        if not root.exists():
            return {}
        if not globs or globs == ["**/*"]:
            shutil.rmtree(root, ignore_errors=True)
            return {}
        for g in globs:
            for p in sorted(root.glob(g), reverse=True):
                if p.is_dir():
                    shutil.rmtree(p, ignore_errors=True)
                elif p.exists():
                    p.unlink()
        return _walk(str(root))

    def list_files(self, storage_id: str) -> Dict[str, int]:
        root = self.path(storage_id)
        return _walk(str(root)) if root.exists() else {}


class DirectoryStorageManager(SharedFSStorageManager):
    """``type: directory`` — a path already mounted in the task (container_path)."""


from determined_clone_amd.common.storage._cloud import (AzureBlobStore, GCSStore,  # noqa: E402
                                                        ObjectStorageManager, S3Store)


class S3StorageManager(ObjectStorageManager):
    """``type: s3`` (AWS or any S3-compatible endpoint), SigV4 over HTTP."""

    def __init__(self, bucket: str, access_key: Optional[str] = None, secret_key: Optional[str] = None,
                 endpoint_url: Optional[str] = None, prefix: Optional[str] = None,
                 region: Optional[str] = None) -> None:
        super().__init__(S3Store(bucket, access_key, secret_key, endpoint_url, region), prefix)


class GCSStorageManager(ObjectStorageManager):
    """``type: gcs``, GCS JSON API with an OAuth bearer token."""

    def __init__(self, bucket: str, prefix: Optional[str] = None, endpoint_url: Optional[str] = None) -> None:
        super().__init__(GCSStore(bucket, endpoint_url), prefix)


class AzureStorageManager(ObjectStorageManager):
    """``type: azure``, Blob REST with SharedKey or SAS."""

    def __init__(self, container: str, connection_string: Optional[str] = None,
                 account_url: Optional[str] = None, credential: Optional[str] = None,
                 prefix: Optional[str] = None) -> None:
        super().__init__(AzureBlobStore(container, connection_string, account_url, credential), prefix)


def build(cfg: Dict[str, Any], container_path: Optional[str] = None) -> StorageManager:
    t = cfg.get("type")
    if t == "shared_fs":
        base = cfg.get("host_path")
        if cfg.get("storage_path"):
            sp = cfg["storage_path"]
            base = sp if os.path.isabs(sp) else os.path.join(base, sp)
        if container_path:
            base = container_path
        return SharedFSStorageManager(base)
    if t == "directory":
        return DirectoryStorageManager(cfg["container_path"])
    if t == "s3":
        return S3StorageManager(cfg["bucket"], **{k: cfg.get(k) for k in ("access_key", "secret_key", "endpoint_url", "prefix")})
    if t == "gcs":
        return GCSStorageManager(cfg["bucket"], prefix=cfg.get("prefix"), endpoint_url=cfg.get("endpoint_url"))
    if t == "azure":
        return AzureStorageManager(cfg["container"], connection_string=cfg.get("connection_string"),
                                   account_url=cfg.get("account_url"), credential=cfg.get("credential"),
                                   prefix=cfg.get("prefix"))
    raise ValueError(f"unknown checkpoint storage type: {t}")


def from_string(s: str) -> StorageManager:
    if s.startswith("s3://"):
        bucket, _, prefix = s[5:].partition("/")
        return S3StorageManager(bucket, prefix=prefix)
    if s.startswith("gs://"):
        bucket, _, prefix = s[5:].partition("/")
        return GCSStorageManager(bucket, prefix=prefix)
    return SharedFSStorageManager(s)
