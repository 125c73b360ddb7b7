"""Kubernetes resource manager: trials and NTSC tasks run as pods on a Kubernetes cluster whose
nodes expose MI355X GPUs through the AMD GPU device plugin (``amd.com/gpu``).

Reference: `master/internal/rm/kubernetesrm` (Go: `kubernetes_resource_manager.go`, `pods.go`,
`pod.go`, `spec.go`, `informer.go`, `request_queue.go`). What it does there, and here:

* **capacity** -- the RM watches the cluster's nodes; every Ready, schedulable node is one
  schedulable "agent" whose slots are its allocatable ``amd.com/gpu`` count (``slot_type: rocm``)
  or ``floor(allocatable cpu / cpu_per_slot)`` (``slot_type: cpu``); the node label
  ``determined.ai/resource_pool`` names its resource pool;
* **scheduling** -- the same native priority / fair-share / round-robin scheduler as the agent RM
  (`native/scheduler.cpp`) places each allocation on nodes (gang placement, at most
  ``max_slots_per_pod`` slots per pod), so queueing, priorities and preemption behave identically;
  the reference instead leans on the kube-scheduler with pod priority classes, but binding the pod
  to the node chosen here (``spec.nodeName``) keeps a multi-pod trial's gang all-or-nothing;
* **pods** -- one pod per container (``exec.task_runner`` as the command, the task spec in
  ``DET_TASK_SPEC``, ``DET_CONTAINER_ADDR`` = the pod IP through the downward API for the
  rendezvous, GPUs requested as ``resources.limits["amd.com/gpu"]``, a memory-backed ``/dev/shm``
  for RCCL/dataloaders), merged with the experiment's ``environment.pod_spec``;
* **watching** -- pod phases are polled from the API server; Running -> container RUNNING,
  Succeeded/Failed -> TERMINATED with the container's exit code, then the pod is deleted; a pod
  that disappears (node lost, deleted by hand) terminates its container with exit code 1;
* **kill** -- pods are deleted with a grace period (the task's SIGTERM handler checkpoints).

The API client speaks plain REST (bearer token, cluster CA) -- no kubernetes SDK in the image --
configured in-cluster (service-account token) or from ``api_server`` / ``token`` / ``ca_file``.
"""
import copy
import logging
import os
import re
import threading
import time
from typing import Any, Callable, Dict, List, Optional

import requests

from determined_clone_amd.agent.runtime import encode_spec
from determined_clone_amd.master.rm import AgentState, AllocationRequest, ResourceManager

logger = logging.getLogger("determined_clone_amd.master.rm_kubernetes")

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"
MANAGED = "determined.ai/managed"
POOL_LABEL = "determined.ai/resource_pool"
ALLOC_LABEL = "determined.ai/allocation"
RANK_LABEL = "determined.ai/container-rank"
CONTAINER_NAME = "determined-container"
DEFAULT_IMAGE = "determined-clone-amd:rocm7.2-gfx950"


class KubeError(RuntimeError):
    pass


class KubeClient:
    """Minimal Kubernetes core/v1 REST client (nodes and pods)."""

    def __init__(self, server: str, token: Optional[str] = None, ca_file: Optional[str] = None,
                 verify: bool = True, timeout: float = 30.0) -> None:
        self.server = server.rstrip("/")
        self.token = token
        self.verify: Any = ca_file if (ca_file and verify) else verify
        self.timeout = timeout
        self.http = requests.Session()

    @classmethod
    def from_config(cls, cfg: Dict[str, Any]) -> "KubeClient":
        server = cfg.get("api_server")
        token = cfg.get("token")
        ca = cfg.get("ca_file")
        if not server:  # in-cluster configuration (the master runs in a pod)
            host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT", "443")
            if not host:
                raise KubeError("kubernetes RM: no api_server configured and not running in a cluster")
            server = f"https://{host}:{port}"
            ca = ca or os.path.join(SA_DIR, "ca.crt")
        if token is None and cfg.get("token_file"):
            with open(cfg["token_file"]) as f:
                token = f.read().strip()
        if token is None and os.path.exists(os.path.join(SA_DIR, "token")):
            with open(os.path.join(SA_DIR, "token")) as f:
                token = f.read().strip()
        return cls(server, token, ca, bool(cfg.get("verify_tls", True)))

    def request(self, method: str, path: str, body: Any = None,
                params: Optional[Dict[str, Any]] = None) -> Any:
        headers = {"Accept": "application/json"}
        if self.token:
            headers["Authorization"] = f"Bearer {self.token}"
        r = self.http.request(method, self.server + path, json=body, params=params, headers=headers,
                              timeout=self.timeout, verify=self.verify)
        if r.status_code == 404 and method == "DELETE":
            return None
        if r.status_code >= 400:
            raise KubeError(f"{method} {path}: HTTP {r.status_code}: {r.text[:300]}")
        return r.json() if r.content else None

    def list_nodes(self) -> List[Dict[str, Any]]:
        return (self.request("GET", "/api/v1/nodes") or {}).get("items", [])

    def list_pods(self, namespace: str, selector: str) -> List[Dict[str, Any]]:
        return (self.request("GET", f"/api/v1/namespaces/{namespace}/pods",
                             params={"labelSelector": selector}) or {}).get("items", [])

    def create_pod(self, namespace: str, pod: Dict[str, Any]) -> Dict[str, Any]:
        return self.request("POST", f"/api/v1/namespaces/{namespace}/pods", pod)

    def delete_pod(self, namespace: str, name: str, grace_seconds: int = 10) -> None:
        self.request("DELETE", f"/api/v1/namespaces/{namespace}/pods/{name}",
                     {"kind": "DeleteOptions", "apiVersion": "v1", "gracePeriodSeconds": grace_seconds})


def parse_quantity(q: Any) -> float:
    """Kubernetes resource quantity -> number ("8", "7800m", "1Gi", "64G")."""
    s = str(q).strip()
    suffixes = {"m": 1e-3, "k": 1e3, "M": 1e6, "G": 1e9, "T": 1e12, "Ki": 1024.0, "Mi": 1024.0 ** 2,
                "Gi": 1024.0 ** 3, "Ti": 1024.0 ** 4}
    for suf in sorted(suffixes, key=len, reverse=True):
        if s.endswith(suf):
            return float(s[: -len(suf)]) * suffixes[suf]
    return float(s)


def _dns_name(s: str, limit: int = 63) -> str:
    s = re.sub(r"[^a-z0-9-]+", "-", s.lower()).strip("-")
    return s[:limit].rstrip("-") or "x"


def _node_ready(node: Dict[str, Any]) -> bool:
    if (node.get("spec") or {}).get("unschedulable"):
        return False
    for c in (node.get("status") or {}).get("conditions") or []:
        if c.get("type") == "Ready":
            return c.get("status") == "True"
    return False


def node_of(agent_id: str) -> str:
    """Kubernetes node name of a schedulable slot group ("node" or "node#j")."""
    return agent_id.split("#", 1)[0]


def _merge(base: Any, over: Any) -> Any:
    if isinstance(base, dict) and isinstance(over, dict):
        out = dict(base)
        for k, v in over.items():
            out[k] = _merge(base.get(k), v) if k in base else copy.deepcopy(v)
        return out
    return copy.deepcopy(over)


class _PodRecord:
    __slots__ = ("name", "alloc_id", "node", "rank", "running", "done", "killed", "created")

    def __init__(self, name: str, alloc_id: str, node: str, rank: int) -> None:
        self.name, self.alloc_id, self.node, self.rank = name, alloc_id, node, rank
        self.running = self.done = self.killed = False
        self.created = time.time()


class KubernetesResourceManager(ResourceManager):
    def __init__(self, config: Dict[str, Any], scheduler: str = "priority", fit: str = "best",
                 preemption: bool = True,
                 on_start: Optional[Callable[[AllocationRequest], None]] = None,
                 on_preempt: Optional[Callable[[AllocationRequest], None]] = None,
                 client: Optional[KubeClient] = None, start_watcher: bool = True) -> None:
        super().__init__(scheduler, fit, preemption, on_start, on_preempt)
        self.config = dict(config)
        self.client = client or KubeClient.from_config(config)
        self.namespace = config.get("namespace", "default")
        self.slot_type = config.get("slot_type", "rocm")
        self.slot_resource = config.get("slot_resource", "amd.com/gpu")
        self.cpu_per_slot = float(config.get("cpu_per_slot", 1))
        self.max_slots_per_pod = config.get("max_slots_per_pod")
        self.default_image = config.get("default_image", DEFAULT_IMAGE)
        self.poll_interval = float(config.get("poll_interval", 1.0))
        self.missing_grace = float(config.get("missing_pod_grace", 30.0))
        self.default_pool = config.get("default_resource_pool", "default")
        # PVCs every task pod mounts (shared_fs checkpoint storage): [{name, claim_name, mount_path}]
        self.volumes: List[Dict[str, str]] = list(config.get("task_volumes") or [])
        self.on_container_event: Optional[Callable[..., None]] = None
        self.pods: Dict[str, _PodRecord] = {}
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.last_error: Optional[str] = None
        if start_watcher:
            self._thread = threading.Thread(target=self._watch, daemon=True, name="k8s-rm")
            self._thread.start()

    # ------------------------------------------------------------------ capacity (informer)
    def _node_slots(self, node: Dict[str, Any]) -> int:
        alloc = (node.get("status") or {}).get("allocatable") or {}
        if self.slot_type == "cpu":
            return int(parse_quantity(alloc.get("cpu", 0)) // self.cpu_per_slot)
        return int(parse_quantity(alloc.get(self.slot_resource, 0)))

    def sync_nodes(self) -> None:
        nodes = self.client.list_nodes()
        seen = set()
        changed = False
        with self._lock:
            for n in nodes:
                if not _node_ready(n):
                    continue
                name = n["metadata"]["name"]
                labels = n["metadata"].get("labels") or {}
                total = self._node_slots(n)
                pool = labels.get(POOL_LABEL, self.default_pool)
                addrs = [a.get("address") for a in (n.get("status") or {}).get("addresses") or []
                         if a.get("type") == "InternalIP"]
                # a node larger than max_slots_per_pod is scheduled as several slot groups
                # ("node#0", "node#1", ...) so no pod asks for more than max_slots_per_pod
                cap = int(self.max_slots_per_pod) if self.max_slots_per_pod else max(total, 1)
                groups = [(name, total)] if total <= cap else [
                    (f"{name}#{j}", min(cap, total - j * cap)) for j in range((total + cap - 1) // cap)]
                for gid, k in groups:
                    seen.add(gid)
                    cur = self.agents.get(gid)
                    if cur is not None and len(cur.slots) == k and cur.pool == pool:
                        cur.last_seen = time.time()
                        continue
                    slots = [{"id": i, "uuid": f"{gid}/{self.slot_type}{i}", "type": self.slot_type,
                              "brand": "AMD Instinct MI355X" if self.slot_type == "rocm" else "cpu"}
                             for i in range(k)]
                    a = AgentState(gid, slots, pool, labels.get("determined.ai/label", ""), addrs)
                    if cur is not None and len(cur.slot_owner) == k:
                        a.slot_owner = cur.slot_owner
                        a.enabled = cur.enabled
                    self.agents[gid] = a
                    changed = True
            for name in [a for a in self.agents if a not in seen]:
                self.agents.pop(name)
                changed = True
        if changed:
            self.schedule()

    # ------------------------------------------------------------------ pods
    def pod_manifest(self, spec: Dict[str, Any]) -> Dict[str, Any]:
        alloc = spec["allocation_id"]
        rank = int(spec.get("container_rank", 0))
        n_slots = len(spec.get("slots") or [])
        name = _dns_name(f"det-{alloc}-{rank}")
        env_cfg = spec.get("environment") or {}
        image = env_cfg.get("image") or self.default_image
        if isinstance(image, dict):
            image = image.get("rocm") or image.get("cpu") or self.default_image
        env = [
            {"name": "DET_TASK_SPEC", "value": encode_spec(spec)},
            {"name": "DET_MASTER", "value": spec["cluster_info"]["master_url"]},
            {"name": "DET_SESSION_TOKEN", "value": spec["cluster_info"].get("session_token", "")},
            {"name": "DET_CONTAINER_RANK", "value": str(rank)},
            {"name": "DET_AGENT_ID", "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}},
            {"name": "DET_CONTAINER_ADDR", "valueFrom": {"fieldRef": {"fieldPath": "status.podIP"}}},
            {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"},
        ]
        if self.slot_type == "cpu":
            res = {"cpu": str(max(n_slots, 1) * self.cpu_per_slot)}
            limits = dict(res)
        else:
            res = {self.slot_resource: str(n_slots)} if n_slots else {}
            limits = dict(res)
        container = {
            "name": CONTAINER_NAME, "image": image,
            "command": ["python3", "-m", "determined_clone_amd.exec.task_runner"],
            "env": env, "resources": {"requests": res, "limits": limits},
            "volumeMounts": [{"name": "dshm", "mountPath": "/dev/shm"}] + [
                {"name": v["name"], "mountPath": v["mount_path"]} for v in self.volumes],
        }
        pod = {
            "apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": self.namespace,
                         "labels": {MANAGED: "true", ALLOC_LABEL: _dns_name(alloc),
                                    RANK_LABEL: str(rank),
                                    "determined.ai/task-type": str(spec.get("kind", "")).lower()},
                         "annotations": {"determined.ai/allocation-id": alloc}},
            "spec": {"restartPolicy": "Never", "nodeName": node_of(spec["agent_id"]),
                     "containers": [container],
                     "volumes": [{"name": "dshm", "emptyDir": {"medium": "Memory"}}] + [
                         {"name": v["name"], "persistentVolumeClaim": {"claimName": v["claim_name"]}}
                         for v in self.volumes]},
        }
        user = env_cfg.get("pod_spec")
        if user:
            user = copy.deepcopy(user)
            ucont = {}
            for c in (user.get("spec") or {}).pop("containers", None) or []:
                if c.get("name") in (CONTAINER_NAME, None):
                    ucont = c
            pod = _merge(pod, user)
            pod["spec"]["containers"] = [_merge(container, {k: v for k, v in ucont.items() if k != "name"})]
            # the RM owns the identity, binding and command of the pod
            pod["metadata"]["name"] = name
            pod["metadata"]["labels"].update({MANAGED: "true", ALLOC_LABEL: _dns_name(alloc),
                                              RANK_LABEL: str(rank)})
            pod["spec"]["nodeName"] = node_of(spec["agent_id"])
            pod["spec"]["restartPolicy"] = "Never"
            pod["spec"]["containers"][0]["command"] = container["command"]
            pod["spec"]["containers"][0]["env"] = env + [e for e in ucont.get("env", [])
                                                         if not e.get("name", "").startswith("DET_")]
        return pod

    def start_containers(self, req: AllocationRequest, specs: List[Dict[str, Any]]) -> None:
        for s in specs:
            pod = self.pod_manifest(s)
            name = pod["metadata"]["name"]
            rec = _PodRecord(name, s["allocation_id"], node_of(s["agent_id"]), int(s.get("container_rank", 0)))
            with self._lock:
                self.pods[name] = rec
            try:
                self.client.create_pod(self.namespace, pod)
            except Exception as e:
                logger.error(f"could not create pod {name}: {e}")
                self.last_error = str(e)
                self._terminated(rec, 1)

    def kill_containers(self, alloc_id: str, placements: List[Dict[str, Any]]) -> None:
        with self._lock:
            recs = [r for r in self.pods.values() if r.alloc_id == alloc_id and not r.done]
        for r in recs:
            r.killed = True
            try:
                self.client.delete_pod(self.namespace, r.name, int(self.config.get("kill_grace_seconds", 10)))
            except Exception as e:
                logger.warning(f"could not delete pod {r.name}: {e}")

    def _event(self, rec: _PodRecord, state: str, code: Optional[int] = None) -> None:
        if self.on_container_event is not None:
            try:
                self.on_container_event(rec.node, rec.alloc_id, state, code)
            except Exception:
                logger.exception(f"container event for pod {rec.name} failed")

    def _terminated(self, rec: _PodRecord, code: int) -> None:
        if rec.done:
            return
        rec.done = True
        with self._lock:
            self.pods.pop(rec.name, None)
        self._event(rec, "TERMINATED", 137 if rec.killed and code == 0 else code)

    @staticmethod
    def _exit_code(pod: Dict[str, Any]) -> int:
        st = pod.get("status") or {}
        for cs in st.get("containerStatuses") or []:
            term = (cs.get("state") or {}).get("terminated")
            if term is not None and term.get("exitCode") is not None:
                return int(term["exitCode"])
        return 0 if st.get("phase") == "Succeeded" else 1

    def sync_pods(self) -> None:
        pods = {p["metadata"]["name"]: p for p in self.client.list_pods(self.namespace, f"{MANAGED}=true")}
        with self._lock:
            recs = list(self.pods.values())
        for rec in recs:
            p = pods.get(rec.name)
            if p is None:
                if rec.killed or time.time() - rec.created > self.missing_grace or rec.running:
                    self._terminated(rec, 137 if rec.killed else 1)
                continue
            phase = (p.get("status") or {}).get("phase")
            if phase == "Running" and not rec.running:
                rec.running = True
                self._event(rec, "RUNNING")
            elif phase in ("Succeeded", "Failed"):
                if not rec.running:
                    rec.running = True
                    self._event(rec, "RUNNING")
                code = self._exit_code(p)
                try:
                    self.client.delete_pod(self.namespace, rec.name, 0)
                except Exception as e:
                    logger.warning(f"could not clean up pod {rec.name}: {e}")
                self._terminated(rec, code)

    def _watch(self) -> None:
        while not self._stop.is_set():
            try:
                self.sync_nodes()
                self.sync_pods()
                self.last_error = None
            except Exception as e:
                if self.last_error != str(e):
                    logger.warning(f"kubernetes RM sync failed: {e}")
                self.last_error = str(e)
            self._stop.wait(self.poll_interval)

    def close(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)

    def pools(self) -> List[Dict[str, Any]]:
        out = super().pools()
        for p in out:
            p["type"] = "RESOURCE_POOL_TYPE_K8S"
            p["slot_type"] = self.slot_type
        return out
