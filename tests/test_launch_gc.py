"""Horovod launch layer compatibility (reference: launch/horovod.py) and the checkpoint-GC task
(reference: exec/gc_checkpoints.py)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    e = dict(os.environ, PYTHONPATH=ROOT)
    e.pop("DET_CLUSTER_INFO", None)
    e.update(kw)
    return e


def test_horovod_layer_single_and_multi_slot(tmp_path):
    script = tmp_path / "s.py"
    script.write_text("import os\nos.write(1, ('<R%s:%s>\\n' % (os.environ.get('HOROVOD_RANK'), "
                      "os.environ.get('HOROVOD_SIZE'))).encode())\n")
    out = subprocess.run([sys.executable, "-m", "determined_clone_amd.launch.horovod", "--autohorovod",
                          "--", "python3", str(script)], env=_env(DET_SLOTS="1"), capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0 and "<RNone:None>" in out.stdout
    out = subprocess.run([sys.executable, "-m", "determined_clone_amd.launch.horovod", "-np", "2",
                          "--", "python3", str(script)], env=_env(DET_SLOTS="2"), capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    import re

    got = sorted(re.findall(r"<R(\d):(\d)>", out.stdout))
    got = [f"{a} {b}" for a, b in got]
    assert got == ["0 2", "1 2"], (out.stdout, out.stderr[-3000:])


def test_gc_checkpoints_task(tmp_path):
    root = tmp_path / "store"
    for sid in ("a", "b"):
        d = root / sid / "sub"
        d.mkdir(parents=True)
        (d / "w.pt").write_text("x")
        (root / sid / "keep.json").write_text("{}")
    cfg = {"type": "shared_fs", "host_path": str(root)}
    env = _env(DET_STORAGE_CONFIG=json.dumps(cfg), DET_DELETE=json.dumps(["a"]))
    subprocess.run([sys.executable, "-m", "determined_clone_amd.exec.gc_checkpoints"], env=env, check=True,
                   timeout=120)
    assert not (root / "a").exists() and (root / "b").exists()
    (tmp_path / "globs.json").write_text(json.dumps(["sub/*.pt"]))
    (tmp_path / "del.json").write_text(json.dumps(["b"]))
    (tmp_path / "cfg.json").write_text(json.dumps(cfg))
    out = subprocess.run([sys.executable, "-m", "determined_clone_amd.exec.gc_checkpoints",
                          "--storage-config", str(tmp_path / "cfg.json"), "--delete", str(tmp_path / "del.json"),
                          "--globs", str(tmp_path / "globs.json")], env=_env(), capture_output=True, text=True,
                         timeout=120, check=True)
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["storage_id"] == "b" and "keep.json" in res["resources"]
    assert not (root / "b" / "sub" / "w.pt").exists() and (root / "b" / "keep.json").exists()
