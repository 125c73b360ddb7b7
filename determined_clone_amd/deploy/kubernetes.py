"""Kubernetes installation of the master (reference: the Helm chart under
`helm/charts/determined/templates/` -- master deployment / service / config map / RBAC /
database -- and `deploy/gke/cli.py`, which installs that chart).

No Helm in this image and no chart toolchain is needed: ``render(values)`` builds the manifests
directly (namespace, service account + the pod/node permissions the Kubernetes resource manager
uses, ``master.yaml`` config map, PVCs for the master database and shared checkpoint storage, the
master Deployment with a health probe, and its Service). ``det deploy k8s render`` prints them;
``up`` / ``down`` pipe them through ``kubectl``.

MI355X specifics: task pods request ``amd.com/gpu`` (the AMD device plugin's resource),
``max_slots_per_pod`` defaults to 8 (one MI355X node = 8 GPUs on one xGMI island, so an 8-slot
trial is one pod and its collectives never leave xGMI), and the shared checkpoint PVC is mounted
into every task pod."""
import copy
import json
import subprocess
from typing import Any, Dict, List, Optional

import yaml

DEFAULTS: Dict[str, Any] = {
    "namespace": "determined",
    "release": "det",
    "image": "determined-clone-amd:rocm7.2-gfx950",
    "image_pull_secret": None,
    "master_port": 8080,
    "service_type": "LoadBalancer",  # ClusterIP | NodePort | LoadBalancer
    "master_cpu": "2",
    "master_memory": "8Gi",
    "db_storage": "10Gi",
    "storage_class": None,
    "checkpoint_storage": {"type": "shared_fs", "size": "1Ti", "access_mode": "ReadWriteMany",
                           "mount_path": "/determined/checkpoints"},
    "max_slots_per_pod": 8,
    "slot_type": "rocm",
    "slot_resource": "amd.com/gpu",
    "task_image": None,
    "default_resource_pool": "default",
    "scheduler": {"type": "priority", "fitting_policy": "best", "preemption": True},
    "cluster_name": "determined-mi355x",
    "authz": "basic",
}


def merge_values(overrides: Optional[Dict[str, Any]]) -> Dict[str, Any]:
    v = copy.deepcopy(DEFAULTS)
    for k, x in (overrides or {}).items():
        if isinstance(x, dict) and isinstance(v.get(k), dict) and k != "checkpoint_storage":
            v[k].update(x)
        elif x is not None:
            v[k] = x
    return v


def _labels(v: Dict[str, Any], component: str) -> Dict[str, str]:
    return {"app.kubernetes.io/name": "determined-clone-amd", "app.kubernetes.io/instance": v["release"],
            "app.kubernetes.io/component": component}


def master_config(v: Dict[str, Any]) -> Dict[str, Any]:
    """The ``master.yaml`` the Deployment mounts."""
    name = f"{v['release']}-master"
    cs = dict(v["checkpoint_storage"])
    rm: Dict[str, Any] = {"type": "kubernetes", "namespace": v["namespace"],
                          "max_slots_per_pod": v["max_slots_per_pod"], "slot_type": v["slot_type"],
                          "slot_resource": v["slot_resource"], "default_image": v["task_image"] or v["image"],
                          "default_resource_pool": v["default_resource_pool"], "scheduler": v["scheduler"]}
    if cs.get("type") == "shared_fs":
        mount = cs.get("mount_path", "/determined/checkpoints")
        rm["task_volumes"] = [{"name": "checkpoints", "claim_name": f"{v['release']}-checkpoints",
                               "mount_path": mount}]
        storage = {"type": "shared_fs", "host_path": mount}
    else:
        storage = {k: x for k, x in cs.items() if k not in ("size", "access_mode", "mount_path")}
    return {"host": "0.0.0.0", "port": v["master_port"], "cluster_name": v["cluster_name"],
            "external_url": f"http://{name}.{v['namespace']}.svc.cluster.local:{v['master_port']}",
            "resource_manager": rm, "checkpoint_storage": storage,
            "security": {"authz": {"type": v["authz"]}}}


def _pvc(v: Dict[str, Any], name: str, size: str, mode: str, component: str) -> Dict[str, Any]:
    spec: Dict[str, Any] = {"accessModes": [mode], "resources": {"requests": {"storage": size}}}
    if v["storage_class"]:
        spec["storageClassName"] = v["storage_class"]
    return {"apiVersion": "v1", "kind": "PersistentVolumeClaim",
            "metadata": {"name": name, "namespace": v["namespace"], "labels": _labels(v, component)},
            "spec": spec}


def render(overrides: Optional[Dict[str, Any]] = None) -> List[Dict[str, Any]]:
    v = merge_values(overrides)
    ns, rel = v["namespace"], v["release"]
    name = f"{rel}-master"
    port = int(v["master_port"])
    cfg = master_config(v)
    out: List[Dict[str, Any]] = [
        {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}},
        {"apiVersion": "v1", "kind": "ServiceAccount",
         "metadata": {"name": name, "namespace": ns, "labels": _labels(v, "master")}},
        # the resource manager creates/deletes task pods in its namespace and reads pod logs/events
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
         "metadata": {"name": name, "namespace": ns, "labels": _labels(v, "master")},
         "rules": [{"apiGroups": [""], "resources": ["pods", "pods/log", "events", "configmaps", "services"],
                    "verbs": ["get", "list", "watch", "create", "delete", "patch", "update"]}]},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
         "metadata": {"name": name, "namespace": ns, "labels": _labels(v, "master")},
         "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role", "name": name},
         "subjects": [{"kind": "ServiceAccount", "name": name, "namespace": ns}]},
        # ... and reads node capacity (allocatable amd.com/gpu) cluster-wide
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
         "metadata": {"name": f"{ns}-{name}-nodes", "labels": _labels(v, "master")},
         "rules": [{"apiGroups": [""], "resources": ["nodes"], "verbs": ["get", "list", "watch"]}]},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
         "metadata": {"name": f"{ns}-{name}-nodes", "labels": _labels(v, "master")},
         "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": f"{ns}-{name}-nodes"},
         "subjects": [{"kind": "ServiceAccount", "name": name, "namespace": ns}]},
        {"apiVersion": "v1", "kind": "ConfigMap",
         "metadata": {"name": f"{name}-config", "namespace": ns, "labels": _labels(v, "master")},
         "data": {"master.yaml": yaml.safe_dump(cfg, sort_keys=False)}},
        _pvc(v, f"{rel}-db", v["db_storage"], "ReadWriteOnce", "database"),
    ]
    mounts = [{"name": "config", "mountPath": "/etc/determined"}, {"name": "db", "mountPath": "/var/lib/determined"}]
    volumes: List[Dict[str, Any]] = [{"name": "config", "configMap": {"name": f"{name}-config"}},
                                     {"name": "db", "persistentVolumeClaim": {"claimName": f"{rel}-db"}}]
    cs = v["checkpoint_storage"]
    if cs.get("type") == "shared_fs":
        out.append(_pvc(v, f"{rel}-checkpoints", cs.get("size", "1Ti"), cs.get("access_mode", "ReadWriteMany"),
                        "checkpoints"))
        mounts.append({"name": "checkpoints", "mountPath": cs.get("mount_path", "/determined/checkpoints")})
        volumes.append({"name": "checkpoints", "persistentVolumeClaim": {"claimName": f"{rel}-checkpoints"}})
    probe = {"httpGet": {"path": "/api/v1/master", "port": port}, "periodSeconds": 10}
    pod_spec: Dict[str, Any] = {
        "serviceAccountName": name,
        "containers": [{
            "name": "determined-master", "image": v["image"], "imagePullPolicy": "IfNotPresent",
            "command": ["python3", "-m", "determined_clone_amd.master", "--config-file",
                        "/etc/determined/master.yaml", "--db", "/var/lib/determined/master.db"],
            "ports": [{"name": "http", "containerPort": port}],
            "env": [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}],
            "resources": {"requests": {"cpu": v["master_cpu"], "memory": v["master_memory"]},
                          "limits": {"memory": v["master_memory"]}},
            "readinessProbe": dict(probe, initialDelaySeconds=5),
            "livenessProbe": dict(probe, initialDelaySeconds=60, failureThreshold=6),
            "volumeMounts": mounts,
        }],
        "volumes": volumes,
    }
    if v["image_pull_secret"]:
        pod_spec["imagePullSecrets"] = [{"name": v["image_pull_secret"]}]
    out.append({"apiVersion": "apps/v1", "kind": "Deployment",
                "metadata": {"name": name, "namespace": ns, "labels": _labels(v, "master")},
                # one master (sqlite on a RWO volume): Recreate so two never share the database
                "spec": {"replicas": 1, "strategy": {"type": "Recreate"},
                         "selector": {"matchLabels": _labels(v, "master")},
                         "template": {"metadata": {"labels": _labels(v, "master")}, "spec": pod_spec}}})
    out.append({"apiVersion": "v1", "kind": "Service",
                "metadata": {"name": name, "namespace": ns, "labels": _labels(v, "master")},
                "spec": {"type": v["service_type"], "selector": _labels(v, "master"),
                         "ports": [{"name": "http", "port": port, "targetPort": port}]}})
    return out


def to_yaml(manifests: List[Dict[str, Any]]) -> str:
    return "---\n".join(yaml.safe_dump(m, sort_keys=False) for m in manifests)


def kubectl(args: List[str], stdin: Optional[str] = None, kubectl_bin: str = "kubectl",
            check: bool = True) -> subprocess.CompletedProcess:
    try:
        return subprocess.run([kubectl_bin] + args, input=stdin, text=True, capture_output=True, check=check)
    except FileNotFoundError:
        raise RuntimeError(f"{kubectl_bin} not found on PATH: install kubectl or use `det deploy k8s render`")
    except subprocess.CalledProcessError as e:
        raise RuntimeError(f"kubectl {' '.join(args)} failed: {e.stderr.strip()}")


def up(overrides: Optional[Dict[str, Any]] = None, kubectl_bin: str = "kubectl",
       wait: bool = True, timeout: str = "600s") -> Dict[str, Any]:
    v = merge_values(overrides)
    kubectl(["apply", "-f", "-"], to_yaml(render(v)), kubectl_bin)
    if wait:
        kubectl(["-n", v["namespace"], "rollout", "status", f"deployment/{v['release']}-master",
                 f"--timeout={timeout}"], kubectl_bin=kubectl_bin)
    svc = json.loads(kubectl(["-n", v["namespace"], "get", "service", f"{v['release']}-master", "-o", "json"],
                             kubectl_bin=kubectl_bin).stdout or "{}")
    ingress = ((svc.get("status") or {}).get("loadBalancer") or {}).get("ingress") or []
    host = (ingress[0].get("ip") or ingress[0].get("hostname")) if ingress else None
    return {"namespace": v["namespace"], "service": f"{v['release']}-master",
            "master_url": f"http://{host}:{v['master_port']}" if host else None}


def down(overrides: Optional[Dict[str, Any]] = None, kubectl_bin: str = "kubectl",
         delete_volumes: bool = False) -> None:
    v = merge_values(overrides)
    keep = {"PersistentVolumeClaim"} if not delete_volumes else set()
    objs = [m for m in render(v) if m["kind"] not in keep | {"Namespace"}]
    kubectl(["delete", "--ignore-not-found", "-f", "-"], to_yaml(objs), kubectl_bin)
    # task pods the resource manager started
    kubectl(["-n", v["namespace"], "delete", "pods", "-l", "determined.ai/managed=true", "--ignore-not-found"],
            kubectl_bin=kubectl_bin, check=False)
