"""det.gpu equivalent (reference: harness/determined/gpu.py) over a fake KFD sysfs tree."""
import os

from determined_clone_amd import gpu


def _node(root, n, props, gpu_id=None):
    d = root / str(n)
    d.mkdir(parents=True)
    (d / "properties").write_text("\n".join(f"{k} {v}" for k, v in props.items()) + "\n")
    if gpu_id is not None:
        (d / "gpu_id").write_text(f"{gpu_id}\n")


def test_gpus_and_processes_from_kfd(tmp_path, monkeypatch):
    topo = tmp_path / "nodes"
    _node(topo, 0, {"simd_count": 0, "unique_id": 0})  # CPU node
    _node(topo, 1, {"simd_count": 1024, "unique_id": 1234, "drm_render_minor": 128}, gpu_id=4242)
    _node(topo, 2, {"simd_count": 1024, "unique_id": 5678, "drm_render_minor": 136}, gpu_id=777)
    monkeypatch.setattr(gpu, "KFD_TOPOLOGY", str(topo))
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    gpus, kind = gpu.get_gpus()
    assert kind == "rocm" and [g.id for g in gpus] == [0, 1]
    assert gpus[0].uuid == "1234" and gpu.get_gpu_uuids() == [g.uuid for g in gpus]
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert [g.uuid for g in gpu.get_gpus()[0]] == ["5678"]

    proc = tmp_path / "proc"
    mine = proc / str(os.getpid())
    mine.mkdir(parents=True)
    (mine / "vram_777").write_text(str(3 * 1024 * 1024) + "\n")
    (mine / "vram_4242").write_text("0\n")  # holds nothing there
    ps = gpu.get_gpu_processes(str(proc), str(topo))
    assert len(ps) == 1 and ps[0].pid == os.getpid() and ps[0].gpu_uuid == "5678"
    assert ps[0].used_memory == "3 MiB"


def test_no_gpus(tmp_path, monkeypatch):
    monkeypatch.setattr(gpu, "KFD_TOPOLOGY", str(tmp_path / "missing"))
    monkeypatch.setattr(gpu, "_rocm_smi_gpus", lambda: [])
    assert gpu.get_gpus() == ([], "") and gpu.get_gpu_uuids() == []
    assert gpu.get_gpu_processes(str(tmp_path / "noproc")) == []
