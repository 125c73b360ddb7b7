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
