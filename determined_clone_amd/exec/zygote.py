"""Pre-warmed fork server for task processes (the agent's "zygote").

A trial process spends its first seconds importing PyTorch (2+ s warm, much more on a fresh box)
before it does any work; an HP search with many short trials (adaptive ASHA: most trials are
stopped after the first rung) pays that per trial. The agent therefore keeps one Python process
that has imported the heavy third-party modules -- and NOTHING that touches the GPU: HIP is never
initialised here, so forking is safe -- and asks it to fork each task process:

* request (over a UNIX socket, one connection per task): ``{"module", "argv", "env", "cwd"}`` plus
  the write end of the task's output pipe as an ancillary fd (``socket.send_fds``);
* the child: ``setsid`` (its own process group, so the agent's kill signals reach the task tree),
  stdout/stderr -> the pipe, the task's environment / cwd / ``sys.path`` (PYTHONPATH entries
  first), fresh ``random`` state, ``torch.set_num_threads`` from ``OMP_NUM_THREADS`` (the OpenMP
  pool size was fixed when the zygote loaded it), then ``runpy.run_module(module)`` as
  ``__main__``; its exit status is the task's;
* replies on the connection: ``{"pid"}`` right after the fork, ``{"exit"}`` when the child ends
  (the zygote reaps it).

Only this framework's modules are imported fresh in each child (they read ``DCA_*`` / ``DET_*``
environment variables at import time). The agent falls back to a plain subprocess when the zygote
is unavailable or ``DET_ZYGOTE=0``, and when the task's environment asks for something a forked,
already-initialised interpreter cannot honour (``incompatible_reason``): a different
``LD_PRELOAD`` / ``LD_LIBRARY_PATH`` (or any ``LD_*``), ``PYTHONHASHSEED``, a virtualenv, or a
``PYTHONPATH`` entry that would shadow one of the pre-imported ``WARM_MODULES``.
"""
import json
import os
import random
import runpy
import signal
import socket
import sys
import threading
import time
import traceback
from typing import Any, Dict, List, Optional

# torch.optim's first Optimizer() imports torch._dynamo (+ sympy, torch.fx, torch._inductor):
# 2.1 s of every trial's start-up on this image unless the zygote has it warm
WARM_MODULES = ("numpy", "torch", "torch.nn", "torch.nn.functional", "torch.utils.data",
                "torch.distributed", "torch.optim", "torch._dynamo", "yaml", "requests")


def gpu_touched() -> bool:
    """True if this process holds the KFD / DRM render device open -- i.e. some import initialised
    the HIP runtime. A process in that state must not fork task processes (whatever module did it,
    not only torch.cuda)."""
    try:
        for fd in os.listdir("/proc/self/fd"):
            try:
                target = os.readlink(f"/proc/self/fd/{fd}")
            except OSError:
                continue
            if target == "/dev/kfd" or target.startswith("/dev/dri/renderD"):
                return True
    except OSError:
        pass
    return False


# variables the dynamic loader / interpreter only read at process start
_START_ONLY = ("PYTHONHASHSEED", "VIRTUAL_ENV", "PYTHONHOME", "PYTHONNOUSERSITE", "PYTHONSTARTUP")


def incompatible_reason(env: Dict[str, str], base_env: Optional[Dict[str, str]] = None,
                        skip_paths: Optional[List[str]] = None) -> Optional[str]:
    """Why a task with environment ``env`` must not be forked from a zygote started under
    ``base_env`` (default: this process's environment), or None if forking is equivalent to a
    fresh interpreter. ``skip_paths``: PYTHONPATH entries known not to shadow anything (the
    task's context directory is checked, the framework root is not)."""
    base = dict(os.environ if base_env is None else base_env)
    for k in sorted(set(env) | set(base)):
        if (k.startswith("LD_") or k in _START_ONLY) and env.get(k) != base.get(k):
            return f"{k} differs from the agent's environment"
    skip = set(skip_paths or ())
    for entry in (env.get("PYTHONPATH") or "").split(os.pathsep):
        if not entry or entry in skip or not os.path.isdir(entry):
            continue
        for mod in {m.split(".")[0] for m in WARM_MODULES}:
            if os.path.exists(os.path.join(entry, mod)) or os.path.exists(os.path.join(entry, mod + ".py")):
                return f"PYTHONPATH entry {entry} shadows pre-imported module {mod}"
    return None


def _send(conn: socket.socket, obj: Dict[str, Any]) -> None:
    conn.sendall(json.dumps(obj).encode() + b"\n")


def _child(req: Dict[str, Any], out_fd: int) -> None:
    os.setsid()
    devnull = os.open(os.devnull, os.O_RDONLY)
    os.dup2(devnull, 0)
    os.dup2(out_fd, 1)
    os.dup2(out_fd, 2)
    os.close(out_fd)
    os.close(devnull)
    signal.signal(signal.SIGTERM, signal.SIG_DFL)
    signal.signal(signal.SIGINT, signal.default_int_handler)
    code = 0
    try:
        os.chdir(req.get("cwd") or "/")
        os.environ.clear()
        os.environ.update(req["env"])
        os.environ["DET_SPAWN_TIME"] = repr(time.time())  # start-up trace origin (exec/harness.py)
        extra = [p for p in req["env"].get("PYTHONPATH", "").split(os.pathsep) if p]
        sys.path[:0] = [p for p in extra if p not in sys.path]
        random.seed()
        n = req["env"].get("OMP_NUM_THREADS")
        if n and n.isdigit():
            import torch

            torch.set_num_threads(int(n))
        # this framework's modules re-import under the task's environment (they read DCA_* /
        # DET_* variables at import time); only third-party modules stay warm
        for name in [m for m in sys.modules if m == "determined_clone_amd" or m.startswith("determined_clone_amd.")]:
            del sys.modules[name]
        sys.argv = [req["module"]] + list(req["argv"])
        runpy.run_module(req["module"], run_name="__main__", alter_sys=True)
    except SystemExit as e:
        code = e.code if isinstance(e.code, int) else (0 if e.code is None else 1)
    except BaseException:  # noqa: BLE001 - report any failure as the task's exit status
        traceback.print_exc()
        code = 1
    try:
        sys.stdout.flush()
        sys.stderr.flush()
    finally:
        os._exit(code)


def _handle(conn: socket.socket, srv: socket.socket) -> None:
    msg, fds, _, _ = socket.recv_fds(conn, 1 << 20, 4)
    req = json.loads(msg.decode())
    if ("torch" in sys.modules and sys.modules["torch"].cuda.is_initialized()) or gpu_touched():
        _send(conn, {"error": "zygote has initialised the GPU; refusing to fork"})
        return
    pid = os.fork()
    if pid == 0:
        srv.close()
        conn.close()
        _child(req, fds[0])
    for fd in fds:
        os.close(fd)
    _send(conn, {"pid": pid})

    def reap() -> None:
        _, status = os.waitpid(pid, 0)
        code = os.waitstatus_to_exitcode(status)
        try:
            _send(conn, {"exit": code})
        finally:
            conn.close()

    threading.Thread(target=reap, daemon=True).start()


def serve(path: str) -> None:
    for m in WARM_MODULES:
        try:
            __import__(m)
        except Exception:  # pragma: no cover - optional module
            pass
    if gpu_touched():  # the agent then starts plain subprocesses
        print("zygote: an import opened the GPU device; not serving", flush=True)
        return
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    if os.path.exists(path):
        os.unlink(path)
    srv.bind(path)
    srv.listen(64)
    print("ready", flush=True)
    parent = os.getppid()

    def watchdog() -> None:  # the agent died without stopping us: do not linger as an orphan
        while True:
            time.sleep(2.0)
            if os.getppid() != parent:
                os._exit(0)

    threading.Thread(target=watchdog, daemon=True).start()
    quiet = os.open(os.devnull, os.O_WRONLY)  # nobody reads our pipe after "ready"
    os.dup2(quiet, 1)
    os.dup2(quiet, 2)
    while True:
        conn, _ = srv.accept()
        try:
            _handle(conn, srv)
        except Exception:  # keep serving: one bad request must not take the zygote down
            traceback.print_exc()
            conn.close()


# ----------------------------------------------------------------------------- agent side
class ZygoteProcess:
    """``subprocess.Popen``-like handle of a zygote-forked task (``pid``, ``stdout``, ``poll``,
    ``wait``, ``returncode``)."""

    def __init__(self, conn: socket.socket, pid: int, stdout: Any) -> None:
        self._conn = conn
        self._file: Any = None  # the connection's reader (set by ZygoteClient.spawn)
        self.pid = pid
        self.stdout = stdout
        self.returncode: Optional[int] = None
        self._lock = threading.Lock()

    def wait(self, timeout: Optional[float] = None) -> int:
        with self._lock:
            if self.returncode is None:
                line = self._file.readline()
                self.returncode = json.loads(line)["exit"] if line else -9
                self._conn.close()
        return self.returncode

    def poll(self) -> Optional[int]:
        return self.returncode


class ZygoteClient:
    def __init__(self, path: str, proc: Any) -> None:
        self.path = path
        self.proc = proc

    @classmethod
    def start(cls, workdir: str) -> Optional["ZygoteClient"]:
        import subprocess

        if os.environ.get("DET_ZYGOTE", "1") == "0":
            return None
        path = os.path.join(workdir, "zygote.sock")
        proc = subprocess.Popen([sys.executable, "-m", "determined_clone_amd.exec.zygote", path],
                                stdout=subprocess.PIPE, start_new_session=True)
        line = proc.stdout.readline()
        if line.strip() != b"ready":
            proc.kill()
            return None
        return cls(path, proc)

    def spawn(self, module: str, argv: List[str], env: Dict[str, str], cwd: str) -> ZygoteProcess:
        r, w = os.pipe()
        conn = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        try:
            conn.connect(self.path)
            socket.send_fds(conn, [json.dumps({"module": module, "argv": argv, "env": env,
                                               "cwd": cwd}).encode()], [w])
        finally:
            os.close(w)
        f = conn.makefile("rb")
        reply = json.loads(f.readline() or b"{}")
        if "pid" not in reply:
            os.close(r)
            conn.close()
            raise RuntimeError(f"zygote refused: {reply.get('error', 'no reply')}")
        p = ZygoteProcess(conn, reply["pid"], os.fdopen(r, "rb"))
        p._file = f
        return p

    def close(self) -> None:
        if self.proc.poll() is None:
            self.proc.kill()
            self.proc.wait()


if __name__ == "__main__":
    serve(sys.argv[1])
