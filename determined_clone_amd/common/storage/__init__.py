"""Checkpoint storage managers (reference: `harness/determined/common/storage/*`).

``shared_fs`` and ``directory`` write straight into the target directory (no staging copy — on a
single MI355X node the checkpoint directory IS the storage). Cloud backends (s3/gcs/azure) are
implemented against their SDKs and raise a clear error when the SDK is not importable.
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


class _CloudStorageManager(StorageManager):
    sdk = ""

    def __init__(self, base_path: str, **kw: Any) -> None:
        super().__init__(base_path)
        self._kw = kw
        self._client = self._make_client()

    def _make_client(self) -> Any:
        raise RuntimeError(f"{type(self).__name__} needs the '{self.sdk}' package, which is not "
                           "installed in this environment")


class S3StorageManager(_CloudStorageManager):
    sdk = "boto3"

    def _make_client(self) -> Any:
        try:
            import boto3  # type: ignore
        except ImportError:
            return super()._make_client()
        return boto3.client("s3", endpoint_url=self._kw.get("endpoint_url"),
                            aws_access_key_id=self._kw.get("access_key"),
                            aws_secret_access_key=self._kw.get("secret_key"))

    def _key(self, *parts: str) -> str:
        prefix = (self._kw.get("prefix") or "").strip("/")
        return "/".join(p for p in [prefix, *parts] if p)

    def upload(self, src, dst, paths=None) -> None:
        src = pathlib.Path(src)
        files = paths if paths is not None else [str(p.relative_to(src)) for p in src.rglob("*") if p.is_file()]
        for rel in files:
            if (src / rel).is_file():
                self._client.upload_file(str(src / rel), self._base_path, self._key(dst, rel))

    def download(self, src, dst, selector=None) -> None:
        pag = self._client.get_paginator("list_objects_v2")
        for page in pag.paginate(Bucket=self._base_path, Prefix=self._key(src) + "/"):
            for obj in page.get("Contents", []):
                rel = obj["Key"][len(self._key(src)) + 1:]
                if selector is not None and not selector(rel):
                    continue
                d = pathlib.Path(dst) / rel
                d.parent.mkdir(parents=True, exist_ok=True)
                self._client.download_file(self._base_path, obj["Key"], str(d))

    def delete(self, storage_id, globs=None) -> Dict[str, int]:
        pag = self._client.get_paginator("list_objects_v2")
        for page in pag.paginate(Bucket=self._base_path, Prefix=self._key(storage_id) + "/"):
            keys = [{"Key": o["Key"]} for o in page.get("Contents", [])]
            if keys:
                self._client.delete_objects(Bucket=self._base_path, Delete={"Objects": keys})
        return {}

    def list_files(self, storage_id: str) -> Dict[str, int]:
        out: Dict[str, int] = {}
        pag = self._client.get_paginator("list_objects_v2")
        for page in pag.paginate(Bucket=self._base_path, Prefix=self._key(storage_id) + "/"):
            for o in page.get("Contents", []):
                out[o["Key"][len(self._key(storage_id)) + 1:]] = o["Size"]
        return out


class GCSStorageManager(_CloudStorageManager):
    sdk = "google-cloud-storage"


class AzureStorageManager(_CloudStorageManager):
    sdk = "azure-storage-blob"


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
        return GCSStorageManager(cfg["bucket"], prefix=cfg.get("prefix"))
    if t == "azure":
        return AzureStorageManager(cfg["container"], connection_string=cfg.get("connection_string"))
    raise ValueError(f"unknown checkpoint storage type: {t}")


def from_string(s: str) -> StorageManager:
    if s.startswith("s3://"):
        bucket, _, prefix = s[5:].partition("/")
        return S3StorageManager(bucket, prefix=prefix)
    if s.startswith("gs://"):
        bucket, _, prefix = s[5:].partition("/")
        return GCSStorageManager(bucket, prefix=prefix)
    return SharedFSStorageManager(s)
