"""The HIP extension loader: the in-tree build and a DCA_OPS_SO override both import (CPU: the
module loads without a GPU; no kernel is launched)."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SO = os.path.join(ROOT, "determined_clone_amd", "ops", "_C.so")

pytestmark = pytest.mark.skipif(not os.path.exists(SO), reason="extension not built")


def _run(env_extra):
    code = ("from determined_clone_amd.ops import _ext; m = _ext.load(); print(m.__file__); "
            "import sys; assert sys.modules['determined_clone_amd.ops._C'] is m")
    env = dict(os.environ, DCA_AUTOBUILD="0", **env_extra)
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return out.stdout.strip()


def test_loads_in_tree_build():
    assert _run({}) == SO


def test_loads_override_file(tmp_path):
    alt = tmp_path / "_C_variant.so"
    alt.write_bytes(open(SO, "rb").read())
    assert _run({"DCA_OPS_SO": str(alt)}) == str(alt)


def test_stale_binary_is_refused(monkeypatch):
    """a ``_C.so`` whose embedded source hash differs from the ``csrc/`` tree next to it
    is refused (StaleExtensionError), the current build passes, and the hash covers every source."""
    from determined_clone_amd.ops import _ext, build

    class Fake:
        __file__ = "_C.so"
        source_hash = "0" * 64

    with pytest.raises(_ext.StaleExtensionError):
        _ext.check_fresh(Fake())
    Fake.source_hash = build.source_hash()
    _ext.check_fresh(Fake())  # matching hash: accepted


def test_stale_binary_refused_in_fresh_process(tmp_path):
    """End to end: a copy of the ops sources with one edited kernel file and the unchanged binary
    fails to load with a clear message instead of running stale kernels."""
    import shutil

    pkg = tmp_path / "determined_clone_amd"
    shutil.copytree(os.path.join(ROOT, "determined_clone_amd"), pkg,
                    ignore=shutil.ignore_patterns("_build", "__pycache__", "_san", "bin", "tuned"))
    hip = sorted((pkg / "ops" / "csrc").glob("*.hip"))[0]
    hip.write_text(hip.read_text() + "\n// edited after the build\n")
    code = "from determined_clone_amd.ops import _ext; _ext.load()"
    env = dict(os.environ, DCA_AUTOBUILD="0", PYTHONPATH=str(tmp_path))
    out = subprocess.run([sys.executable, "-c", code], cwd=tmp_path, env=env, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode != 0
    assert "is stale" in out.stderr, out.stderr[-2000:]
