"""Agent zygote (exec/zygote.py): forked task processes get the task's env / cwd / sys.path /
argv, stream output through the pipe, report exit codes, and die with their process group."""
import os
import signal
import sys
import tempfile
import time

from determined_clone_amd.exec.zygote import ZygoteClient

MOD = '''
import os, sys
print("x=" + os.environ["X"], "argv=" + ",".join(sys.argv[1:]), "cwd=" + os.getcwd(), flush=True)
if sys.argv[1:] == ["sleep"]:
    import time; time.sleep(60)
import determined_clone_amd
print("fresh", "determined_clone_amd.exec.zygote" not in sys.modules, flush=True)
sys.exit(3)
'''


def test_zygote_spawn_exit_and_kill():
    tmp = tempfile.mkdtemp(prefix="zyg-")
    with open(os.path.join(tmp, "zmod.py"), "w") as f:
        f.write(MOD)
    z = ZygoteClient.start(tmp)
    assert z is not None
    try:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env = {"X": "42", "PYTHONPATH": os.pathsep.join([tmp, root]), "PATH": os.environ.get("PATH", "")}
        p = z.spawn("zmod", ["a", "b"], env, tmp)
        out = p.stdout.read().decode()
        assert p.wait() == 3
        assert f"x=42 argv=a,b cwd={tmp}" in out
        assert "fresh True" in out  # framework modules re-imported in the child
        p2 = z.spawn("zmod", ["sleep"], env, tmp)
        line = p2.stdout.readline().decode()
        assert "argv=sleep" in line
        os.killpg(p2.pid, signal.SIGTERM)
        assert p2.wait() == -signal.SIGTERM
    finally:
        z.close()


def test_incompatible_env_falls_back(tmp_path):
    """Variables a forked interpreter cannot honour route the task to a plain subprocess."""
    from determined_clone_amd.exec.zygote import incompatible_reason

    base = {"PATH": "/bin", "LD_LIBRARY_PATH": "/opt/rocm/lib"}
    assert incompatible_reason(dict(base, DET_X="1"), base) is None
    assert "LD_PRELOAD" in incompatible_reason(dict(base, LD_PRELOAD="/x.so"), base)
    assert "LD_LIBRARY_PATH" in incompatible_reason(dict(base, LD_LIBRARY_PATH="/other"), base)
    assert "PYTHONHASHSEED" in incompatible_reason(dict(base, PYTHONHASHSEED="0"), base)
    shadow = tmp_path / "venv_site"
    (shadow / "numpy").mkdir(parents=True)
    why = incompatible_reason(dict(base, PYTHONPATH=str(shadow)), base)
    assert why and "numpy" in why
    assert incompatible_reason(dict(base, PYTHONPATH=str(shadow)), base, skip_paths=[str(shadow)]) is None
