"""Core API v2: a singleton-style Core API that also works for UNMANAGED training -- a process
started by hand (a notebook, another scheduler, a laptop) that reports metrics, checkpoints and
logs to the master as an experiment/trial without the cluster launching it.

Reference: ``harness/determined/experimental/core_v2/_core_v2.py`` (DefaultConfig,
UnmanagedConfig, init/init_context/close), ``_unmanaged.py`` (get-or-create of the experiment and
trial by external ids, StartTrial -> ClusterInfo) and ``_core_context_v2.py`` (context assembly).
"""
import atexit
import dataclasses
import logging
import uuid
from typing import Any, Callable, Dict, List, Optional, TypeVar, Union

from determined_clone_amd import _info, core
from determined_clone_amd.common import storage
from determined_clone_amd.core._log_shipper import _UnmanagedTrialLogShipper

logger = logging.getLogger("determined_clone_amd.core")

T = TypeVar("T")

_context: Optional[core.Context] = None
_client: Any = None
_atexit_registered = False


@dataclasses.dataclass
class DefaultConfig:
    """Experiment config values for an unmanaged run (merged under the expconf defaults)."""

    name: Optional[str] = None
    hparams: Optional[Dict[str, Any]] = None
    data: Optional[Dict[str, Any]] = None
    description: Optional[str] = None
    labels: Optional[List[str]] = None
    checkpoint_storage: Optional[Union[str, Dict[str, Any]]] = None
    searcher: Optional[Dict[str, Any]] = None


@dataclasses.dataclass
class UnmanagedConfig:
    """Where the unmanaged experiment lives and how to find it again on resume.

    ``external_experiment_id`` groups several runs (e.g. an HP search done outside the cluster)
    into one experiment; with ``external_trial_id`` too, re-running the script resumes the same
    trial (its ``info.latest_checkpoint`` and steps completed come back from the master)."""

    workspace: Optional[str] = None
    project: Optional[str] = None
    external_experiment_id: Optional[str] = None
    external_trial_id: Optional[str] = None


def _rank0_then_broadcast(fn: Callable[[], T], distributed: Optional[core.DistributedContext]) -> T:
    out = fn() if distributed is None or distributed.rank == 0 else None
    if distributed is not None and distributed.size > 1:
        out = distributed.broadcast(out)
    assert out is not None
    return out


def _project_id(session: Any, workspace: Optional[str], project: Optional[str]) -> Optional[int]:
    if not (workspace and project):
        return None
    for w in session.get("/api/v1/workspaces")["workspaces"]:
        if w["name"] == workspace:
            for p in session.get(f"/api/v1/workspaces/{w['id']}/projects")["projects"]:
                if p["name"] == project:
                    return int(p["id"])
    raise ValueError(f"project {workspace}/{project} not found")


def _get_or_create(session: Any, config: Dict[str, Any], unmanaged: UnmanagedConfig,
                   hparams: Optional[Dict[str, Any]]) -> Dict[str, Any]:
    """Rank-0 side: experiment + trial ids and the StartTrial response."""
    body: Dict[str, Any] = {"config": config, "unmanaged": True,
                            "project_id": _project_id(session, unmanaged.workspace, unmanaged.project)}
    if unmanaged.external_experiment_id is not None:
        exp = session.put(f"/api/v1/experiments/{unmanaged.external_experiment_id}", body)["experiment"]
    elif unmanaged.external_trial_id is not None:
        raise NotImplementedError("external_trial_id requires external_experiment_id")
    else:
        exp = session.post("/api/v1/experiments", body)["experiment"]
    create = {"experiment_id": exp["id"], "hparams": hparams or {}, "unmanaged": True}
    if unmanaged.external_trial_id is not None:
        trial = session.put("/api/v1/trials", {"create_trial_request": create,
                                               "external_trial_id": unmanaged.external_trial_id})["trial"]
    else:
        trial = session.post("/api/v1/trials", create)["trial"]
    start = session.post(f"/api/v1/trials/{trial['id']}/start", {"resume": True})
    master = session.get("/api/v1/master")
    return {"experiment_id": exp["id"], "trial_id": trial["id"], "task_id": trial["taskId"],
            "cluster_id": master["cluster_id"], "start": start, "config": exp.get("config") or config}


def _unmanaged_cluster_info(client: Any, d: Dict[str, Any], hparams: Optional[Dict[str, Any]]) -> _info.ClusterInfo:
    s = d["start"]
    trial = _info.TrialInfo(trial_id=d["trial_id"], experiment_id=d["experiment_id"], trial_seed=0,
                            hparams=hparams or {}, config=d["config"],
                            steps_completed=int(s.get("steps_completed") or 0),
                            trial_run_id=int(s.get("trial_run_id") or 0))
    return _info.ClusterInfo(master_url=client._session.master, cluster_id=d["cluster_id"],
                             agent_id="unmanaged", slot_ids=[], task_id=d["task_id"],
                             allocation_id=d["task_id"], session_token=client._session.token or "",
                             task_type="TRIAL", latest_checkpoint=s.get("latest_checkpoint"),
                             trial_info=trial,
                             rendezvous_info=_info.RendezvousInfo(["127.0.0.1"], 0, [0]))


def _make_unmanaged_context(client: Any, info: _info.ClusterInfo,
                            distributed: Optional[core.DistributedContext],
                            checkpoint_storage: Optional[Union[str, Dict[str, Any]]],
                            preempt_mode: core.PreemptMode, tensorboard_mode: str) -> core.Context:
    session = client._session
    distributed = distributed or core.DummyDistributedContext()
    cfg = info.trial._config
    storage_cfg = checkpoint_storage or cfg.get("checkpoint_storage")
    sm = core._context._get_storage_manager(storage_cfg)
    if sm is None:
        base = core._context._default_local_storage()
        logger.info(f"no checkpoint storage configured; storing checkpoints in {base}")
        sm = storage.SharedFSStorageManager(base)
    tb = writer = None
    if storage_cfg is not None and isinstance(storage_cfg, dict):
        from determined_clone_amd import tensorboard

        tb = tensorboard.build(info.cluster_id, str(info.trial.experiment_id), str(info.trial.trial_id),
                               storage_cfg, rank=distributed.rank)
        if tb is not None and tensorboard_mode == core.TensorboardMode.AUTO:
            writer = tb.metric_writer()
    else:
        tensorboard_mode = core.TensorboardMode.MANUAL
    train = core.TrainContext(session, info.trial.trial_id, info.trial._trial_run_id,
                              info.trial.experiment_id, distributed, tensorboard_mode, tb, writer)
    searcher = core.SearcherContext(session, distributed, info.trial.trial_id,
                                    info.trial._trial_run_id, info.allocation_id,
                                    core._parse_searcher_units(cfg))
    # no allocation for an off-cluster process: checkpoints are reported against the task only
    checkpoint = core.CheckpointContext(distributed, sm, session, info.task_id, None,
                                        tensorboard_manager=tb)
    # detached runs are never preempted by the cluster
    preempt = core.DummyPreemptContext(distributed, preempt_mode)
    heartbeat = core._Heartbeat(session=session, trial_id=info.trial.trial_id) if distributed.rank == 0 else None
    shipper = _UnmanagedTrialLogShipper(session=session, trial_id=info.trial.trial_id,
                                        task_id=info.task_id, distributed=distributed)
    core._context._install_stacktrace_on_sigusr1()
    return core.Context(checkpoint=checkpoint, distributed=distributed, preempt=preempt,
                        train=train, searcher=searcher, info=info, _tensorboard_manager=tb,
                        _heartbeat=heartbeat, _session=session, _log_shipper=shipper)


def _init_context(client: Any, defaults: Optional[DefaultConfig], unmanaged: Optional[UnmanagedConfig],
                  distributed: Optional[core.DistributedContext],
                  checkpoint_storage: Optional[Union[str, Dict[str, Any]]],
                  preempt_mode: core.PreemptMode, tensorboard_mode: str) -> core.Context:
    info = _info.get_cluster_info()
    if info is not None and info.task_type == "TRIAL":
        # launched by the cluster: the classic managed Core API
        return core.init(distributed=distributed, checkpoint_storage=checkpoint_storage,
                         preempt_mode=preempt_mode, tensorboard_mode=tensorboard_mode)
    if defaults is None:
        raise NotImplementedError("either specify `defaults`, or run as a managed experiment")
    um = unmanaged or UnmanagedConfig()
    checkpoint_storage = checkpoint_storage or defaults.checkpoint_storage
    config: Dict[str, Any] = {
        "name": defaults.name or f"unmanaged-{uuid.uuid4().hex[:8]}",
        "searcher": defaults.searcher or {"name": "single", "metric": "unmanaged",
                                          "max_length": 100000000},
        "entrypoint": "unmanaged",
    }
    for k in ("data", "description", "labels"):
        if getattr(defaults, k) is not None:
            config[k] = getattr(defaults, k)
    if isinstance(checkpoint_storage, dict):
        config["checkpoint_storage"] = checkpoint_storage
    if um.workspace:
        config["workspace"] = um.workspace
    if um.project:
        config["project"] = um.project
    if client is None:
        client = _default_client()
    d = _rank0_then_broadcast(lambda: _get_or_create(client._session, config, um, defaults.hparams),
                              distributed)
    info = _unmanaged_cluster_info(client, d, defaults.hparams)
    return _make_unmanaged_context(client, info, distributed, checkpoint_storage, preempt_mode,
                                   tensorboard_mode)


def _default_client() -> Any:
    from determined_clone_amd.experimental import client as sdk

    return sdk.Determined()


def init_context(*, defaults: Optional[DefaultConfig] = None,
                 unmanaged: Optional[UnmanagedConfig] = None, client: Any = None,
                 distributed: Optional[core.DistributedContext] = None,
                 checkpoint_storage: Optional[Union[str, Dict[str, Any]]] = None,
                 preempt_mode: core.PreemptMode = core.PreemptMode.WorkersAskChief,
                 tensorboard_mode: str = core.TensorboardMode.AUTO) -> core.Context:
    """Context-manager style: ``with core_v2.init_context(defaults=...) as ctx: ...``."""
    return _init_context(client, defaults, unmanaged, distributed, checkpoint_storage, preempt_mode,
                         tensorboard_mode)


def _set_globals() -> None:
    from determined_clone_amd.experimental import core_v2

    assert _context is not None
    core_v2.train = _context.train
    core_v2.checkpoint = _context.checkpoint
    core_v2.distributed = _context.distributed
    core_v2.preempt = _context.preempt
    core_v2.searcher = _context.searcher
    core_v2.info = _context.info


def init(*, defaults: Optional[DefaultConfig] = None, unmanaged: Optional[UnmanagedConfig] = None,
         client: Any = None, distributed: Optional[core.DistributedContext] = None,
         checkpoint_storage: Optional[Union[str, Dict[str, Any]]] = None,
         preempt_mode: core.PreemptMode = core.PreemptMode.WorkersAskChief,
         tensorboard_mode: str = core.TensorboardMode.AUTO) -> None:
    """Singleton style: afterwards ``core_v2.train.report_training_metrics(...)`` etc.;
    :func:`close` (also registered ``atexit``) reports the trial COMPLETED."""
    global _context, _client, _atexit_registered
    if _context is not None:
        _context.close()
    _client = client or _default_client()
    _context = _init_context(_client, defaults, unmanaged, distributed, checkpoint_storage,
                             preempt_mode, tensorboard_mode)
    _context.start()
    _set_globals()
    if not _atexit_registered:
        atexit.register(close)
        _atexit_registered = True


def close() -> None:
    global _context
    from determined_clone_amd.experimental import core_v2

    if _context is not None:
        _context.close()
    _context = None
    core_v2.train = None


def url_reverse_webui_exp_view() -> str:
    from determined_clone_amd.experimental import core_v2

    assert core_v2.info is not None and core_v2.info.trial is not None
    assert _client is not None
    return f"{_client._session.master}/det/experiments/{core_v2.info.trial.experiment_id}"
