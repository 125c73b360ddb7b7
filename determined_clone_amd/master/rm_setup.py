"""Build the master's resource manager from the master config (reference:
`master/internal/rm/setup.go`, `master/internal/config/resource_config.go`).

``resource_manager.type``: ``agent`` (default: agents register their MI355X slots), ``kubernetes``
(pods, ``master/rm_kubernetes.py``), ``slurm`` / ``pbs`` (batch jobs, ``master/rm_dispatcher.py``).
``resource_pools[*].provider`` (agent RM only) attaches a cloud provisioner
(``master/provisioner.py``) to that pool.
"""
from typing import Any, Callable, Dict, List, Optional

from determined_clone_amd.master.rm import ResourceManager


def make_resource_manager(rm_config: Optional[Dict[str, Any]], scheduler: str, fit: str,
                          preemption: bool, on_start: Callable, on_preempt: Callable,
                          on_container_event: Callable,
                          resource_pools: Optional[List[Dict[str, Any]]] = None) -> ResourceManager:
    cfg = dict(rm_config or {})
    kind = cfg.get("type", "agent")
    if kind == "agent":
        rm: ResourceManager = ResourceManager(scheduler, fit, preemption, on_start, on_preempt)
    elif kind == "kubernetes":
        from determined_clone_amd.master.rm_kubernetes import KubernetesResourceManager

        rm = KubernetesResourceManager(cfg, scheduler, fit, preemption, on_start, on_preempt)
    elif kind in ("slurm", "pbs"):
        from determined_clone_amd.master.rm_dispatcher import DispatcherResourceManager

        rm = DispatcherResourceManager(cfg, scheduler, fit, preemption, on_start, on_preempt)
    else:
        raise ValueError(f"unknown resource_manager.type {kind!r} (agent | kubernetes | slurm | pbs)")
    rm.on_container_event = on_container_event
    if kind == "agent":
        # providers bake the master URL into their instances' startup script: they are built
        # when the master starts serving (ResourceManager.start_provisioners)
        rm.provisioner_configs = [(p.get("pool_name", "default"), p["provider"])
                                  for p in resource_pools or [] if p.get("provider")]
    return rm
