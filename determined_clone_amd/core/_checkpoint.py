"""CheckpointContext (reference: `harness/determined/core/_checkpoint.py`).

A checkpoint is a directory identified by a UUID (``storage_id``) in the configured storage, with a
``metadata.json`` beside the user's files; the chief registers it with the master (``resources`` =
file -> size map, ``metadata`` incl. ``steps_completed``). ``shard=True`` lets every rank write its
own files into the same checkpoint (ZeRO optimizer shards, per-rank RNG), merged by the chief.
"""
import contextlib
import enum
import hashlib
import json
import logging
import os
import pathlib
import uuid
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple

from determined_clone_amd.common import storage

logger = logging.getLogger("determined_clone_amd.core")


class DownloadMode(enum.Enum):
    LocalWorkersShareDownload = "LOCAL_WORKERS_SHARE_DOWNLOAD"
    NoSharedDownload = "NO_SHARED_DOWNLOAD"


def _merge_md(merged: Dict[str, Any], md: Dict[str, Any], rank: int, owners: Dict[str, Any],
              conflicts: Dict[str, List[int]], prefix: str) -> None:
    for k, v in md.items():
        full = f"{prefix}{k}"
        if k not in merged:
            if isinstance(v, dict):
                merged[k], owners[k] = {}, {}
                _merge_md(merged[k], v, rank, owners[k], conflicts, full + ".")
            else:
                merged[k], owners[k] = v, [rank]
            continue
        cur = merged[k]
        if isinstance(cur, dict) and isinstance(v, dict):
            _merge_md(cur, v, rank, owners[k], conflicts, full + ".")
        elif isinstance(cur, dict) or isinstance(v, dict) or cur != v:
            prev = owners[k] if isinstance(owners[k], list) else []
            conflicts[full] = sorted(set(conflicts.get(full, prev) + [rank]))
        else:
            owners[k].append(rank)


def merge_metadata(all_metadata: List[Dict[str, Any]]) -> Tuple[Dict[str, Any], Dict[str, List[int]]]:
    """Merge every rank's metadata (reference core/_checkpoint.py:84-124): dictionaries under one
    key merge recursively, equal repeated values are fine, anything else is a conflict. Returns
    ``(merged, {dotted key: ranks that reported it})``."""
    merged: Dict[str, Any] = {}
    owners: Dict[str, Any] = {}
    conflicts: Dict[str, List[int]] = {}
    for rank, md in enumerate(all_metadata):
        _merge_md(merged, md or {}, rank, owners, conflicts, "")
    return merged, conflicts


def merge_resources(all_resources: List[Dict[str, int]]) -> Tuple[Dict[str, int], Dict[str, List[int]]]:
    """Merge every rank's ``{path: size}`` (directories end in ``/``; reference :127-167). Two
    ranks may both create a directory; a FILE name that more than one rank writes (or that one
    rank writes as a file and another as a directory) is a conflict: ``{name: ranks}``."""
    files = set()
    uploaders: Dict[str, List[int]] = {}
    merged: Dict[str, int] = {}
    for rank, rscs in enumerate(all_resources):
        for name, size in rscs.items():
            if name.endswith("/") or name.endswith(os.sep):
                uploaders.setdefault(name.rstrip("/").rstrip(os.sep), []).append(rank)
            else:
                files.add(name)
                uploaders.setdefault(name, []).append(rank)
            merged[name] = size
    conflicts = {n: uploaders[n] for n in sorted(files) if len(uploaders[n]) > 1}
    return merged, conflicts


class CheckpointContext:
    def __init__(self, dist: Any, storage_manager: storage.StorageManager, session: Any = None,
                 task_id: Optional[str] = None, allocation_id: Optional[str] = None,
                 tbd_sync_mode: Any = None, tensorboard_manager: Any = None,
                 storage_backend_id: Optional[int] = None) -> None:
        self._dist = dist
        self._storage_manager = storage_manager
        self._session = session
        self._task_id = task_id
        self._allocation_id = allocation_id
        self._tensorboard_manager = tensorboard_manager

    # ------------------------------------------------------------------ writing
    def upload(self, ckpt_dir: Optional[os.PathLike], metadata: Optional[Dict[str, Any]] = None, *,
               shard: bool = False, selector: Optional[Callable[[str], bool]] = None,
               _storage_id: Optional[str] = None) -> str:
        if not shard:
            if self._dist.rank != 0:
                raise RuntimeError("upload(shard=False) may only be called on the chief")
            if ckpt_dir is None:
                raise ValueError("ckpt_dir required when shard=False")
            storage_id = str(uuid.uuid4())
            self._storage_manager.upload(ckpt_dir, storage_id, self._selected(ckpt_dir, selector))
            resources = self._storage_manager.list_files(storage_id) if isinstance(
                self._storage_manager, storage.SharedFSStorageManager) else _local_resources(ckpt_dir)
            md = dict(metadata or {})
            self._write_metadata(storage_id, md)
            self._report_checkpoint(storage_id, resources, md)
            return storage_id
        storage_id = _storage_id or self._dist.broadcast(str(uuid.uuid4()) if self._dist.rank == 0 else None)
        if selector is not None and ckpt_dir is None:
            raise RuntimeError("ckpt_dir has to be provided if selector is not None")
        # A rank uploads when it has a selector (each rank contributes ITS selected files, even
        # from a directory shared with other ranks; byte-identical duplicates are deduplicated by
        # _resolve_conflicts), or when it is the lowest rank naming a shared directory without a
        # selector (reference core/_checkpoint.py:305-318).
        uid = None
        if ckpt_dir is not None:
            st = os.stat(ckpt_dir)
            uid = (os.uname().nodename, st.st_dev, st.st_ino)
        uids = self._dist.allgather(uid)
        if not any(u is not None for u in uids):
            raise RuntimeError("cannot call .upload(ckpt_dir=None, shard=True) from all ranks; "
                               "at least one rank must have a valid ckpt_dir")
        want_upload = selector is not None or (uid is not None and uids.index(uid) == self._dist.rank)
        res = {}
        if want_upload:
            res = _local_resources(ckpt_dir)
            if selector is not None:
                res = {k: v for k, v in res.items() if selector(k.rstrip("/"))}
        merged_res, conflicts = merge_resources(self._dist.allgather(res))
        res = self._resolve_conflicts(res, conflicts, ckpt_dir)
        md = self._merge_metadata(metadata)
        if want_upload and res:
            self._storage_manager.upload(ckpt_dir, storage_id, [k for k in res if not k.endswith("/")])
        self._dist.allgather(None)  # every shard is in storage before the chief reports
        if self._dist.rank == 0:
            self._write_metadata(storage_id, md)
            self._report_checkpoint(storage_id, merged_res, md)
        return storage_id

    @contextlib.contextmanager
    def store_path(self, metadata: Optional[Dict[str, Any]] = None, *,
                   shard: bool = False) -> Iterator[Tuple[pathlib.Path, str]]:
        """Yields ``(path, storage_id)``; files written under ``path`` become the checkpoint.

        ``shard=False``: chief only. ``shard=True`` (reference core/_checkpoint.py:526-590): every
        rank must enter; ranks' metadata are merged and a conflicting key raises. On a storage
        whose ``store_path`` is the storage itself (shared_fs / directory) every rank writes
        straight into the one checkpoint directory; otherwise each rank writes a local staging
        directory, a directory shared by several local ranks is uploaded once (lowest rank), a
        file written by more than one rank raises unless every copy has the same content (then
        the lowest rank uploads it), exactly as :meth:`upload` with ``shard=True``."""
        if not shard:
            if self._dist.rank != 0:
                raise RuntimeError("store_path(shard=False) may only be called on the chief "
                                   f"(rank={self._dist.rank})")
            storage_id = str(uuid.uuid4())
            with self._storage_manager.store_path(storage_id) as path:
                yield path, storage_id
                res = _local_resources(path)
            md = dict(metadata or {})
            self._write_metadata(storage_id, md)
            if isinstance(self._storage_manager, storage.SharedFSStorageManager):
                res = self._storage_manager.list_files(storage_id)
            self._report_checkpoint(storage_id, res, md)
            return
        storage_id = self._dist.broadcast(str(uuid.uuid4()) if self._dist.rank == 0 else None)
        if self._storage_manager.store_path_is_direct_access():
            with self._storage_manager.store_path(storage_id) as path:
                yield path, storage_id
            md = self._merge_metadata(metadata)
            self._dist.allgather(None)  # every rank's files are written
            if self._dist.rank == 0:
                self._write_metadata(storage_id, md)
                self._report_checkpoint(storage_id, self._storage_manager.list_files(storage_id), md)
            return
        path = self._storage_manager.pre_store_path(storage_id)
        try:
            yield path, storage_id
            self.upload(path, metadata, shard=True, _storage_id=storage_id)
        finally:
            self._storage_manager.post_store_path(path)

    # ------------------------------------------------------------------ reading
    def _coordinated_selector(self, selector: Optional[Callable[[str], bool]]) -> Optional[Callable[[str], bool]]:
        """On the local chief: a selector that asks every local rank about each file (functions
        do not serialise, file names do) and keeps a file if any rank wants it (reference
        core/_checkpoint.py:429-460)."""
        def sel(path: str) -> bool:
            self._dist.broadcast_local(path)
            votes = self._dist.gather_local(selector(path) if selector is not None else True)
            return any(votes or [True])
        return sel

    def _serve_local_chief(self, selector: Optional[Callable[[str], bool]]) -> None:
        """Non-chief local ranks: answer the chief's per-file questions until it says done. A
        :class:`_ChiefFailed` sentinel (the chief's download raised) is re-raised here, so the
        local ranks fail with the chief instead of waiting for a terminator that never comes."""
        while True:
            name = self._dist.broadcast_local(None)
            if name is None:
                return
            if isinstance(name, dict) and name.get("__chief_failed__"):
                raise RuntimeError(f"checkpoint download failed on the local chief: {name['error']}")
            self._dist.gather_local(selector(name) if selector is not None else True)

    def _chief_failed(self, exc: BaseException) -> None:
        """Tell the waiting local ranks that the chief's download raised (see
        :meth:`_serve_local_chief`)."""
        try:
            self._dist.broadcast_local({"__chief_failed__": True, "error": f"{type(exc).__name__}: {exc}"})
        except Exception:  # the group itself is broken: nothing more to tell
            logger.exception("could not tell the local ranks that the download failed")

    def download(self, storage_id: str, ckpt_dir: os.PathLike,
                 download_mode: DownloadMode = DownloadMode.LocalWorkersShareDownload,
                 selector: Optional[Callable[[str], bool]] = None) -> None:
        """Download a checkpoint into ``ckpt_dir``. ``LocalWorkersShareDownload`` (default): every
        rank calls, only the local chief of each node downloads (the union of the local ranks'
        selectors); ``NoSharedDownload``: each caller downloads for itself."""
        download_mode = DownloadMode(download_mode)
        if download_mode == DownloadMode.NoSharedDownload:
            self._storage_manager.download(storage_id, ckpt_dir, selector)
            return
        want_filter = any(self._dist.allgather(selector is not None))
        if self._dist.local_rank == 0:
            try:
                self._storage_manager.download(storage_id, ckpt_dir,
                                               self._coordinated_selector(selector) if want_filter else None)
            except BaseException as e:
                self._chief_failed(e)
                raise
            self._dist.broadcast_local(None)
        else:
            self._serve_local_chief(selector)

    @contextlib.contextmanager
    def restore_path(self, storage_id: str,
                     download_mode: DownloadMode = DownloadMode.LocalWorkersShareDownload,
                     selector: Optional[Callable[[str], bool]] = None) -> Iterator[pathlib.Path]:
        """Context manager yielding a local path holding the checkpoint (reference :599-675).
        ``LocalWorkersShareDownload``: all ranks must call; only the local chief of each node
        downloads (cloud storage) and the others receive its path; the download is removed when
        every local rank has left the context. ``NoSharedDownload``: each rank for itself."""
        download_mode = DownloadMode(download_mode)
        if download_mode == DownloadMode.NoSharedDownload:
            with self._storage_manager.restore_path(storage_id, selector) as p:
                yield p
            return
        want_filter = any(self._dist.allgather(selector is not None))
        if self._dist.local_rank == 0:
            sel = self._coordinated_selector(selector) if want_filter else None
            with contextlib.ExitStack() as stack:
                try:
                    p = stack.enter_context(self._storage_manager.restore_path(storage_id, sel))
                except BaseException as e:
                    self._chief_failed(e)
                    raise
                self._dist.broadcast_local(None)  # download finished
                self._dist.broadcast_local(str(p))
                try:
                    yield p
                finally:
                    self._dist.gather_local(None)  # local ranks are done with it
        else:
            self._serve_local_chief(selector)
            p = pathlib.Path(self._dist.broadcast_local(None))
            try:
                yield p
            finally:
                self._dist.gather_local(None)

    def get_metadata(self, storage_id: str) -> Dict[str, Any]:
        if isinstance(self._storage_manager, storage.SharedFSStorageManager):
            p = self._storage_manager.path(storage_id) / "metadata.json"
            if p.exists():
                return json.loads(p.read_text())
        if self._session is not None:
            r = self._session.get(f"/api/v1/checkpoints/{storage_id}")
            return (r.get("checkpoint") or {}).get("metadata", {})
        return {}

    def delete(self, storage_id: str, globs: Optional[List[str]] = None) -> None:
        self._storage_manager.delete(storage_id, globs)
        if self._session is not None:
            self._session.post("/api/v1/checkpoints/rm", {"checkpoint_uuids": [storage_id],
                                                          "globs": globs or ["**/*"]})

    # ------------------------------------------------------------------ internals
    def _selected(self, ckpt_dir: os.PathLike, selector: Optional[Callable[[str], bool]]) -> Optional[List[str]]:
        if selector is None:
            return None
        root = pathlib.Path(ckpt_dir)
        return [str(p.relative_to(root)) for p in root.rglob("*") if selector(str(p.relative_to(root)))]

    def _merge_metadata(self, metadata: Optional[Dict[str, Any]]) -> Dict[str, Any]:
        merged, conflicts = merge_metadata(self._dist.allgather(metadata or {}))
        if conflicts:
            self._raise_conflict_error(conflicts, "metadata")
        return merged

    def _resolve_conflicts(self, resources: Dict[str, int], conflicts: Dict[str, List[int]],
                           ckpt_dir: Optional[os.PathLike]) -> Dict[str, int]:
        """Files written by several ranks are fine when every copy is byte-identical (md5,
        compared across ranks in sorted name order); the lowest such rank uploads it. Anything
        else raises (reference core/_checkpoint.py:353-402)."""
        remaining = dict(conflicts)
        for fname in sorted(conflicts):
            digest = None
            if self._dist.rank in conflicts[fname]:
                fpath = os.path.join(os.fspath(ckpt_dir), fname)
                if os.path.isdir(fpath):
                    digest = "this is a directory"
                else:
                    with open(fpath, "rb") as f:
                        digest = hashlib.md5(f.read()).hexdigest()
            if len({d for d in self._dist.allgather(digest) if d is not None}) == 1:
                remaining.pop(fname)
        if remaining:
            self._raise_conflict_error(remaining, "files")
        return {k: v for k, v in resources.items()
                if k not in conflicts or min(conflicts[k]) == self._dist.rank}

    def _raise_conflict_error(self, conflicts: Dict[str, List[int]], what: str) -> None:
        if self._dist.rank > 0:
            raise RuntimeError(f"refusing to upload with {what} conflicts: {conflicts}")
        lines = [f"    {k} uploaded by ranks {r}" for k, r in sorted(conflicts.items())]
        raise RuntimeError(f"refusing to upload with {what} conflicts:\n" + "\n".join(lines))

    def _write_metadata(self, storage_id: str, md: Dict[str, Any]) -> None:
        if isinstance(self._storage_manager, storage.SharedFSStorageManager):
            p = self._storage_manager.path(storage_id)
            p.mkdir(parents=True, exist_ok=True)
            (p / "metadata.json").write_text(json.dumps(md, indent=2, default=str))
        else:
            import tempfile

            with tempfile.TemporaryDirectory() as d:
                pathlib.Path(d, "metadata.json").write_text(json.dumps(md, default=str))
                self._storage_manager.upload(d, storage_id, ["metadata.json"])

    def _report_checkpoint(self, storage_id: str, resources: Dict[str, int],
                           metadata: Dict[str, Any]) -> None:
        if self._session is None:
            return
        self._session.post("/api/v1/checkpoints", {
            "uuid": storage_id, "task_id": self._task_id, "allocation_id": self._allocation_id,
            "resources": resources, "metadata": metadata, "state": "COMPLETED",
        })


def _local_resources(path: Optional[os.PathLike]) -> Dict[str, int]:
    if path is None or not os.path.isdir(path):
        return {}
    return storage._walk(str(path))


class DummyCheckpointContext(CheckpointContext):
    def __init__(self, dist: Any, storage_manager: storage.StorageManager) -> None:
        super().__init__(dist, storage_manager, None)
