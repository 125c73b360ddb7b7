"""GPU inventory for the harness (``det.gpu``): the devices a task can see, their load and memory,
and the processes holding GPU memory.

Reference: `harness/determined/gpu.py` asks ``nvidia-smi`` (then ``rocm-smi --json``) for
``GPU(id, uuid, load, memoryUtil)`` and ``nvidia-smi --query-compute-apps`` for GPU processes.
Here everything comes straight from the amdgpu / KFD sysfs interfaces, so it needs no CLI tool
and no HIP initialisation (safe in a process that will fork, e.g. the agent's zygote):

* devices: KFD topology nodes with SIMDs (``/sys/class/kfd/kfd/topology/nodes/N``), in the order
  HIP enumerates them, ``unique_id`` as the uuid (the native ``detect_kfd_gpus`` walk,
  ``native/scheduler.cpp``, when the extension is built);
* load / memory: the node's DRM device (``/sys/class/drm/renderD<minor>/device``):
  ``gpu_busy_percent``, ``mem_info_vram_used`` / ``mem_info_vram_total``;
* processes: ``/sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>`` (bytes of VRAM each process holds
  on each device).

``rocm-smi --showuniqueid --json`` is the fallback when KFD sysfs is unreadable (containers that
hide /sys/class/kfd).
"""
import json
import logging
import os
import subprocess
from typing import Dict, List, NamedTuple, Optional, Tuple

logger = logging.getLogger("determined_clone_amd")

KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"
KFD_PROC = "/sys/class/kfd/kfd/proc"


class GPU(NamedTuple):
    id: int
    uuid: str
    load: float
    memoryUtil: float


class GPUProcess(NamedTuple):
    pid: int
    process_name: str
    gpu_uuid: str
    used_memory: str  # with units, e.g. "123 MiB" (the reference's nvidia-smi format)


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _props(node_dir: str) -> Dict[str, str]:
    out: Dict[str, str] = {}
    for line in (_read(os.path.join(node_dir, "properties")) or "").splitlines():
        parts = line.split()
        if len(parts) == 2:
            out[parts[0]] = parts[1]
    return out


def _kfd_nodes(root: Optional[str] = None) -> List[Dict[str, str]]:
    """GPU nodes of the KFD topology in node order: {index, node, gpu_id, uuid, render_minor}."""
    root = root or KFD_TOPOLOGY
    if not os.path.isdir(root):
        return []
    nodes = []
    for name in sorted(os.listdir(root), key=lambda s: int(s) if s.isdigit() else 1 << 30):
        d = os.path.join(root, name)
        p = _props(d)
        if not p or p.get("simd_count", "0") == "0":
            continue  # CPU node
        uid = p.get("unique_id", "0")
        nodes.append({"index": str(len(nodes)), "node": name, "gpu_id": _read(os.path.join(d, "gpu_id")) or "",
                      # the raw KFD unique_id: the same string the agent reports as the slot's uuid
                      "uuid": uid if uid != "0" else f"node-{name}",
                      "render_minor": p.get("drm_render_minor", "")})
    return nodes


def _drm_device(render_minor: str) -> Optional[str]:
    d = f"/sys/class/drm/renderD{render_minor}/device"
    return d if render_minor and os.path.isdir(d) else None


def _load_and_mem(render_minor: str) -> Tuple[float, float]:
    d = _drm_device(render_minor)
    if d is None:
        return 0.0, 0.0
    busy = _read(os.path.join(d, "gpu_busy_percent"))
    used = _read(os.path.join(d, "mem_info_vram_used"))
    total = _read(os.path.join(d, "mem_info_vram_total"))
    load = float(busy) / 100.0 if busy and busy.isdigit() else 0.0
    mem = float(used) / float(total) if used and total and used.isdigit() and total.isdigit() and int(total) else 0.0
    return load, mem


def _visible(n: int) -> List[int]:
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if not vis:
        return list(range(n))
    return [int(x) for x in vis.split(",") if x.strip().isdigit() and int(x) < n]


def _rocm_smi_gpus() -> List[GPU]:
    try:
        out = subprocess.run(["rocm-smi", "--showid", "--showuniqueid", "--json"], check=True,
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=30).stdout
        data = json.loads(out)
    except FileNotFoundError:
        logger.info("rocm-smi not found")
        return []
    except Exception as e:  # noqa: BLE001 - inventory is best effort
        logger.warning(f"rocm-smi error: {e}")
        return []
    return [GPU(id=int(k[len("card"):]), uuid=str(v.get("Unique ID", k)), load=0.0, memoryUtil=0.0)
            for k, v in sorted(data.items()) if k.startswith("card")]


def get_gpus() -> Tuple[List[GPU], str]:
    """``([GPU], "rocm")`` for the devices this process may use (HIP_VISIBLE_DEVICES applied),
    ``([], "")`` when there are none."""
    nodes = _kfd_nodes()
    if nodes:
        gpus = []
        for i in _visible(len(nodes)):
            load, mem = _load_and_mem(nodes[i]["render_minor"])
            gpus.append(GPU(id=i, uuid=nodes[i]["uuid"], load=load, memoryUtil=mem))
        logger.info(f"detected {len(gpus)} rocm gpus")
        return gpus, "rocm"
    gpus = _rocm_smi_gpus()
    return (gpus, "rocm") if gpus else ([], "")


class GPUStats(NamedTuple):
    uuid: str
    util_percent: float  # amdgpu gpu_busy_percent
    free_memory_gb: float  # VRAM total - used, in 1e9 bytes (the reference's pynvml unit)


def get_gpu_stats() -> List[GPUStats]:
    """Utilisation and free VRAM of the visible devices from the amdgpu sysfs files (no HIP
    initialisation, no CLI tool): what the profiler's system-metrics thread samples."""
    out: List[GPUStats] = []
    nodes = _kfd_nodes()
    for i in _visible(len(nodes)):
        d = _drm_device(nodes[i]["render_minor"])
        if d is None:
            continue
        busy = _read(os.path.join(d, "gpu_busy_percent"))
        used = _read(os.path.join(d, "mem_info_vram_used"))
        total = _read(os.path.join(d, "mem_info_vram_total"))
        if not (busy and busy.isdigit()):
            continue
        free = (int(total) - int(used)) / 1e9 if used and total and used.isdigit() and total.isdigit() else 0.0
        out.append(GPUStats(uuid=nodes[i]["uuid"], util_percent=float(busy), free_memory_gb=free))
    return out


def get_gpu_uuids() -> List[str]:
    gpus, _ = get_gpus()
    return [g.uuid for g in sorted(gpus, key=lambda g: g.id)]


def _fmt_mib(nbytes: int) -> str:
    return f"{nbytes // (1024 * 1024)} MiB"


def get_gpu_processes(proc_root: Optional[str] = None, topology_root: Optional[str] = None) -> List[GPUProcess]:
    """Processes holding VRAM on any GPU (KFD's per-process ``vram_<gpu_id>`` counters)."""
    proc_root = proc_root or KFD_PROC
    by_gpu_id = {n["gpu_id"]: n["uuid"] for n in _kfd_nodes(topology_root) if n["gpu_id"]}
    if not os.path.isdir(proc_root):
        return []
    out = []
    for pid in sorted((p for p in os.listdir(proc_root) if p.isdigit()), key=int):
        d = os.path.join(proc_root, pid)
        try:
            entries = os.listdir(d)
        except OSError:
            continue
        name = (_read(f"/proc/{pid}/comm") or "?")
        for e in sorted(entries):
            if not e.startswith("vram_"):
                continue
            used = _read(os.path.join(d, e))
            gid = e[len("vram_"):]
            if used and used.isdigit() and int(used) > 0:
                out.append(GPUProcess(pid=int(pid), process_name=name, gpu_uuid=by_gpu_id.get(gid, gid),
                                      used_memory=_fmt_mib(int(used))))
    return out
