"""Cluster / trial information handed to a task by the master.

Reference: `harness/determined/_info.py` (ClusterInfo, TrialInfo, RendezvousInfo, ResourcesInfo,
`get_cluster_info()`). The agent writes one JSON document (``DET_CLUSTER_INFO_PATH``) or passes it
inline in ``DET_CLUSTER_INFO``; off-cluster both are absent and ``get_cluster_info()`` is None.
"""
import json
import os
import subprocess
from typing import Any, Dict, List, Optional

DEFAULT_CLUSTER_INFO_PATH = "/run/determined/info/cluster_info.json"


class TrialInfo:
    def __init__(self, trial_id: int, experiment_id: int, trial_seed: int, hparams: Dict[str, Any],
                 config: Dict[str, Any], steps_completed: int = 0, trial_run_id: int = 0,
                 debug: bool = False, inter_node_network_interface: Optional[str] = None) -> None:
        self.trial_id = int(trial_id)
        self.experiment_id = int(experiment_id)
        self.trial_seed = int(trial_seed)
        self.hparams = dict(hparams)
        self._config = dict(config)
        self._steps_completed = int(steps_completed)
        self._trial_run_id = int(trial_run_id)
        self._debug = bool(debug)
        self._inter_node_network_interface = inter_node_network_interface

    def to_dict(self) -> Dict[str, Any]:
        return {"trial_id": self.trial_id, "experiment_id": self.experiment_id,
                "trial_seed": self.trial_seed, "hparams": self.hparams, "config": self._config,
                "steps_completed": self._steps_completed, "trial_run_id": self._trial_run_id,
                "debug": self._debug,
                "inter_node_network_interface": self._inter_node_network_interface}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "TrialInfo":
        return cls(**d)


class RendezvousInfo:
    def __init__(self, container_addrs: List[str], container_rank: int,
                 container_slot_counts: Optional[List[int]] = None,
                 port: Optional[int] = None) -> None:
        self.container_addrs = list(container_addrs)
        self.container_rank = int(container_rank)
        self.container_slot_counts = list(container_slot_counts or [])
        self.port = int(port) if port else None  # c10d port the master reserved on the chief


class ClusterInfo:
    """Everything a task running on the cluster knows about itself."""

    def __init__(self, master_url: str, cluster_id: str, agent_id: str, slot_ids: List[int],
                 task_id: str, allocation_id: str, session_token: str, task_type: str,
                 master_cert_name: Optional[str] = None, latest_checkpoint: Optional[str] = None,
                 trial_info: Optional[TrialInfo] = None,
                 rendezvous_info: Optional[RendezvousInfo] = None,
                 gpu_uuids: Optional[List[str]] = None, user_data: Optional[Dict] = None) -> None:
        self.master_url = master_url
        self.cluster_id = cluster_id
        self.agent_id = agent_id
        self.slot_ids = list(slot_ids)
        self.task_id = task_id
        self.allocation_id = allocation_id
        self.session_token = session_token
        self.task_type = task_type
        self.master_cert_name = master_cert_name
        self._latest_checkpoint = latest_checkpoint
        self._trial_info = trial_info
        self._rendezvous_info = rendezvous_info
        self._gpu_uuids = list(gpu_uuids or [])
        self._user_data = dict(user_data or {})

    @property
    def latest_checkpoint(self) -> Optional[str]:
        return self._latest_checkpoint

    @property
    def user_data(self) -> Dict[str, Any]:
        return self._user_data

    @property
    def trial(self) -> TrialInfo:
        if self._trial_info is None:
            raise RuntimeError(f"ClusterInfo.trial is only available for TRIAL tasks, not {self.task_type}")
        return self._trial_info

    @property
    def container_addrs(self) -> List[str]:
        return self._rendezvous_info.container_addrs if self._rendezvous_info else ["127.0.0.1"]

    @property
    def container_rank(self) -> int:
        return self._rendezvous_info.container_rank if self._rendezvous_info else 0

    @property
    def container_slot_counts(self) -> List[int]:
        if self._rendezvous_info and self._rendezvous_info.container_slot_counts:
            return self._rendezvous_info.container_slot_counts
        return [len(self.slot_ids)]

    @property
    def rendezvous_port(self) -> Optional[int]:
        return self._rendezvous_info.port if self._rendezvous_info else None

    @property
    def gpu_uuids(self) -> List[str]:
        return self._gpu_uuids

    def to_dict(self) -> Dict[str, Any]:
        d = {"master_url": self.master_url, "cluster_id": self.cluster_id,
             "agent_id": self.agent_id, "slot_ids": self.slot_ids, "task_id": self.task_id,
             "allocation_id": self.allocation_id, "session_token": self.session_token,
             "task_type": self.task_type, "master_cert_name": self.master_cert_name,
             "latest_checkpoint": self._latest_checkpoint, "gpu_uuids": self._gpu_uuids,
             "user_data": self._user_data}
        if self._trial_info:
            d["trial"] = self._trial_info.to_dict()
        if self._rendezvous_info:
            d["rendezvous"] = {"container_addrs": self._rendezvous_info.container_addrs,
                               "container_rank": self._rendezvous_info.container_rank,
                               "container_slot_counts": self._rendezvous_info.container_slot_counts,
                               "port": self._rendezvous_info.port}
        return d

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "ClusterInfo":
        d = dict(d)
        trial = d.pop("trial", None)
        rdzv = d.pop("rendezvous", None)
        return cls(trial_info=TrialInfo.from_dict(trial) if trial else None,
                   rendezvous_info=RendezvousInfo(**rdzv) if rdzv else None, **d)

    def _to_file(self, path: str) -> None:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as f:
            json.dump(self.to_dict(), f)


_override: Optional[ClusterInfo] = None


def _set_cluster_info(info: Optional[ClusterInfo]) -> None:
    """Test hook: force the cluster info seen by `get_cluster_info()`."""
    global _override
    _override = info


def get_cluster_info() -> Optional[ClusterInfo]:
    """ClusterInfo of the current task, or None when running off-cluster."""
    if _override is not None:
        return _override
    raw = os.environ.get("DET_CLUSTER_INFO")
    if raw:
        return ClusterInfo.from_dict(json.loads(raw))
    path = os.environ.get("DET_CLUSTER_INFO_PATH")
    if path and os.path.exists(path):
        with open(path) as f:
            return ClusterInfo.from_dict(json.load(f))
    return None


class ResourcesInfo:
    """GPUs assigned to this container (reference: `_info.py` ResourcesInfo): the ROCm device
    UUIDs from the cluster info, or from ``rocm-smi`` when off-cluster."""

    def __init__(self, gpu_uuids: List[str]) -> None:
        self._gpu_uuids = list(gpu_uuids)

    @property
    def gpu_uuids(self) -> List[str]:
        return self._gpu_uuids

    @classmethod
    def _by_inspection(cls) -> "ResourcesInfo":
        info = get_cluster_info()
        if info is not None and info.gpu_uuids:
            return cls(info.gpu_uuids)
        try:
            out = subprocess.run(["rocm-smi", "--showuniqueid", "--json"], capture_output=True,
                                 text=True, timeout=20).stdout
            d = json.loads(out or "{}")
            return cls([str(v.get("Unique ID")) for k, v in sorted(d.items())
                        if k.startswith("card") and v.get("Unique ID")])
        except (OSError, ValueError, subprocess.SubprocessError):
            return cls([])
