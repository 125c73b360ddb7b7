"""Container runtimes of the agent: Docker / Podman (Engine API over a unix socket) and Apptainer.

Reference: ``agent/pkg/docker/docker.go:118-345`` (pull with registry auth, create / run / signal /
remove, reattach to running containers after an agent restart by label),
``agent/internal/containers/spec.go:99-142`` (ROCm device mapping: ``/dev/kfd`` plus each
assigned GPU's ``/dev/dri/card*`` and ``renderD*`` resolved through
``/dev/dri/by-path/pci-<bus>-{card,render}``, ``--group-add video``, ``seccomp=unconfined``),
``master/pkg/tasks/mounts.go:12-29`` (bind mounts; relative container paths under the work dir),
``task.go:254`` (``shm_size``), ``agent/pkg/podman``, ``agent/pkg/singularity`` (Apptainer).

No Docker SDK: :class:`EngineClient` speaks the Engine REST API over ``AF_UNIX`` with
``http.client``; Podman serves the same API on its own socket. A task container gets its context
directory at ``/run/determined/workdir`` and this framework read-only at ``/run/determined/dca``;
the task command runs through ``exec/entrypoint.sh`` (``startup-hook.sh``). Containers carry
``ai.det.clone.*`` labels (agent, allocation, slots), which is how a restarted agent finds and
re-attaches to the tasks it left running.
"""
import base64
import http.client
import json
import logging
import os
import shlex
import socket
import subprocess
import threading
import time
import urllib.parse
from typing import Any, Dict, Iterator, List, Optional, Tuple

logger = logging.getLogger("determined_clone_amd.agent")

WORKDIR = "/run/determined/workdir"
FRAMEWORK_MOUNT = "/run/determined/dca"
LABEL_AGENT = "ai.det.clone.agent"
LABEL_ALLOC = "ai.det.clone.allocation"
LABEL_TASK = "ai.det.clone.task"
LABEL_SLOTS = "ai.det.clone.slots"
LABEL_VERSION = "ai.det.clone.version"
DEFAULT_DOCKER_SOCKET = "/var/run/docker.sock"


def default_podman_socket() -> str:
    run = os.environ.get("XDG_RUNTIME_DIR")
    user = os.path.join(run, "podman", "podman.sock") if run else ""
    return user if user and os.path.exists(user) else "/run/podman/podman.sock"


# ----------------------------------------------------------------------------- Engine API client
class _UnixConnection(http.client.HTTPConnection):
    def __init__(self, path: str, timeout: Optional[float] = None) -> None:
        super().__init__("localhost", timeout=timeout)
        self._path = path

    def connect(self) -> None:
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        if self.timeout is not None:
            s.settimeout(self.timeout)
        s.connect(self._path)
        self.sock = s


class EngineError(RuntimeError):
    def __init__(self, status: int, message: str) -> None:
        super().__init__(f"container engine: HTTP {status}: {message}")
        self.status = status


class EngineClient:
    """Docker Engine API (also Podman's Docker-compatible API) over a unix socket."""

    def __init__(self, socket_path: str = DEFAULT_DOCKER_SOCKET, api_version: str = "v1.41",
                 timeout: float = 60.0) -> None:
        self.socket_path = socket_path
        self.prefix = f"/{api_version}" if api_version else ""
        self.timeout = timeout

    def _open(self, method: str, path: str, params: Optional[Dict[str, Any]] = None,
              body: Any = None, headers: Optional[Dict[str, str]] = None,
              timeout: Optional[float] = -1.0) -> http.client.HTTPResponse:
        q = ("?" + urllib.parse.urlencode(params)) if params else ""
        conn = _UnixConnection(self.socket_path, self.timeout if timeout == -1.0 else timeout)
        data = None
        hdrs = dict(headers or {})
        if body is not None:
            data = json.dumps(body).encode()
            hdrs["Content-Type"] = "application/json"
        conn.request(method, self.prefix + path + q, body=data, headers=hdrs)
        resp = conn.getresponse()
        if resp.status >= 400:
            raw = resp.read().decode(errors="replace")
            try:
                msg = json.loads(raw).get("message", raw)
            except ValueError:
                msg = raw
            conn.close()
            raise EngineError(resp.status, msg)
        return resp

    def _json(self, method: str, path: str, **kw: Any) -> Any:
        resp = self._open(method, path, **kw)
        raw = resp.read()
        return json.loads(raw) if raw.strip() else None

    def ping(self) -> bool:
        try:
            return self._open("GET", "/_ping", timeout=5.0).read().strip() == b"OK"
        except (OSError, EngineError, http.client.HTTPException):
            return False

    # ------------------------------------------------------------------ images
    def image_exists(self, image: str) -> bool:
        try:
            self._json("GET", f"/images/{urllib.parse.quote(image, safe='')}/json")
            return True
        except EngineError as e:
            if e.status == 404:
                return False
            raise

    def pull(self, image: str, auth: Optional[Dict[str, Any]] = None) -> List[Dict[str, Any]]:
        """POST /images/create, following the progress stream; raises on an error message."""
        name, tag = split_image(image)
        headers = {}
        if auth:
            headers["X-Registry-Auth"] = base64.urlsafe_b64encode(
                json.dumps({k: v for k, v in auth.items() if v}).encode()).decode()
        resp = self._open("POST", "/images/create", params={"fromImage": name, "tag": tag},
                          headers=headers, timeout=None)
        events = []
        for line in resp:
            line = line.strip()
            if not line:
                continue
            ev = json.loads(line)
            events.append(ev)
            if ev.get("error") or ev.get("errorDetail"):
                raise EngineError(500, f"pulling {image}: {ev.get('error') or ev.get('errorDetail')}")
        return events

    # ------------------------------------------------------------------ containers
    def create(self, name: str, config: Dict[str, Any]) -> str:
        return self._json("POST", "/containers/create", params={"name": name}, body=config)["Id"]

    def start(self, cid: str) -> None:
        self._open("POST", f"/containers/{cid}/start").read()

    def wait(self, cid: str) -> int:
        r = self._json("POST", f"/containers/{cid}/wait", timeout=None)
        return int(r.get("StatusCode", 1))

    def kill(self, cid: str, sig: str = "SIGTERM") -> None:
        try:
            self._open("POST", f"/containers/{cid}/kill", params={"signal": sig}).read()
        except EngineError as e:
            if e.status not in (404, 409):  # gone / not running
                raise

    def remove(self, cid: str, force: bool = True) -> None:
        try:
            self._open("DELETE", f"/containers/{cid}", params={"force": int(force)}).read()
        except EngineError as e:
            if e.status != 404:
                raise

    def inspect(self, cid: str) -> Dict[str, Any]:
        return self._json("GET", f"/containers/{cid}/json")

    def list(self, labels: Dict[str, str], all: bool = True) -> List[Dict[str, Any]]:
        f = {"label": [f"{k}={v}" for k, v in labels.items()]}
        return self._json("GET", "/containers/json",
                          params={"all": int(all), "filters": json.dumps(f)}) or []

    def logs(self, cid: str, since: Optional[float] = None) -> Iterator[bytes]:
        """Follow stdout+stderr; yields raw byte chunks of the demultiplexed stream."""
        params = {"follow": 1, "stdout": 1, "stderr": 1}
        if since is not None:
            params["since"] = int(since)
        resp = self._open("GET", f"/containers/{cid}/logs", params=params, timeout=None)
        while True:
            head = _read_exact(resp, 8)
            if not head:
                return
            if head[0] in (0, 1, 2) and head[1:4] == b"\x00\x00\x00":  # multiplexed frame
                n = int.from_bytes(head[4:8], "big")
                yield _read_exact(resp, n)
            else:  # TTY container: raw stream
                yield head
                chunk = resp.read1(65536) if hasattr(resp, "read1") else resp.read(65536)
                if not chunk:
                    return
                yield chunk


def _read_exact(resp: Any, n: int) -> bytes:
    out = b""
    while len(out) < n:
        chunk = resp.read(n - len(out))
        if not chunk:
            break
        out += chunk
    return out


def split_image(image: str) -> Tuple[str, str]:
    """``registry:5000/ns/name:tag`` -> (``registry:5000/ns/name``, ``tag``); default tag latest;
    a digest reference (``@sha256:...``) is passed whole with an empty tag."""
    if "@" in image:
        return image, ""
    slash = image.rfind("/")
    colon = image.rfind(":")
    if colon > slash:
        return image[:colon], image[colon + 1:]
    return image, "latest"


# ----------------------------------------------------------------------------- container spec
def rocm_device_paths(devices: List[Dict[str, Any]], dev_root: str = "/dev") -> List[str]:
    """``/dev/kfd`` + each ROCm slot's DRM card and render nodes, resolved through
    ``/dev/dri/by-path/pci-<bus>-{card,render}`` (reference spec.go:99-142); a device without a
    by-path entry falls back to ``renderD<drm_render_minor>``. Shared GPUs (several slots of
    one device) are mapped once."""
    out = [os.path.join(dev_root, "kfd")]
    seen = set()
    for d in devices:
        if d.get("type") != "rocm":
            continue
        bus = d.get("pci_bus")
        key = bus or d.get("device_index", d.get("id"))
        if key in seen:
            continue
        seen.add(key)
        found = False
        if bus:
            for kind in ("card", "render"):
                link = os.path.join(dev_root, "dri", "by-path", f"pci-{str(bus).lower()}-{kind}")
                if os.path.lexists(link):
                    out.append(os.path.realpath(link))
                    found = True
        if not found and d.get("render_minor") is not None:
            out.append(os.path.join(dev_root, "dri", f"renderD{int(d['render_minor'])}"))
            found = True
        if not found:
            raise RuntimeError(f"no /dev/dri node found for ROCm device {d.get('uuid')} (bus {bus})")
    return out


def container_mounts(spec: Dict[str, Any], ctx_dir: str, framework_root: str) -> List[Dict[str, Any]]:
    mounts = [{"Type": "bind", "Source": ctx_dir, "Target": WORKDIR, "ReadOnly": False},
              {"Type": "bind", "Source": framework_root, "Target": FRAMEWORK_MOUNT, "ReadOnly": True}]
    for m in (spec.get("container") or {}).get("bind_mounts") or []:
        target = m["container_path"]
        if not target.startswith("/"):
            target = os.path.join(WORKDIR, target)
        mounts.append({"Type": "bind", "Source": m["host_path"], "Target": target,
                       "ReadOnly": bool(m.get("read_only")),
                       "BindOptions": {"Propagation": m.get("propagation") or "rprivate"}})
    return mounts


def to_container_paths(env: Dict[str, str], ctx_dir: str, framework_root: str) -> Dict[str, str]:
    """The task environment as seen inside the container (host paths of the context directory
    and of the framework replaced by their mount points; host-only variables dropped)."""
    out = {}
    for k, v in env.items():
        if k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
            continue  # the device mapping confines the container; in-container indices restart at 0
        out[k] = v.replace(ctx_dir, WORKDIR).replace(framework_root, FRAMEWORK_MOUNT)
    out["PYTHONPATH"] = os.pathsep.join([WORKDIR, FRAMEWORK_MOUNT])
    out["DET_CONTEXT_DIR"] = WORKDIR
    return out


def container_cmd(cmd: List[str], python: str = "python3") -> List[str]:
    """The task command inside the container: the host interpreter becomes the image's
    ``python3`` ($DET_PYTHON_EXECUTABLE), and it always runs through exec/entrypoint.sh so a
    startup-hook.sh in the context directory is sourced first."""
    import sys

    from determined_clone_amd.agent import runtime

    cmd = list(cmd)
    if cmd[:2] == ["bash", runtime.ENTRYPOINT_SH]:
        cmd = cmd[2:]
    cmd = [python if c == sys.executable else c for c in cmd]
    return ["bash", f"{FRAMEWORK_MOUNT}/determined_clone_amd/exec/entrypoint.sh"] + cmd


DEFAULT_IMAGES = {"cpu": "determined-clone-amd/environments:py-3.10-cpu",
                  "rocm": "determined-clone-amd/environments:py-3.10-rocm-7.2-gfx950"}


def image_for(c: Dict[str, Any], devices: List[Dict[str, Any]]) -> str:
    """``environment.image`` (a string, or the per-flavour map) for the task's device type."""
    img = c.get("image")
    flavour = "rocm" if any(d.get("type") == "rocm" for d in devices) else "cpu"
    if isinstance(img, str) and img:
        return img
    if isinstance(img, dict):
        got = img.get(flavour) or (img.get("cuda") or img.get("gpu") if flavour == "rocm" else None)
        if got:
            return got
    return DEFAULT_IMAGES[flavour]


def engine_config(spec: Dict[str, Any], cmd: List[str], env: Dict[str, str], ctx_dir: str,
                  devices: List[Dict[str, Any]], agent_id: str, framework_root: str,
                  dev_root: str = "/dev", network_mode: str = "host") -> Dict[str, Any]:
    """``POST /containers/create`` body for one task container (reference ToDockerSpec +
    overwriteSpec)."""
    c = spec.get("container") or {}
    host: Dict[str, Any] = {
        "Mounts": container_mounts(spec, ctx_dir, framework_root),
        "NetworkMode": network_mode,
        "CapAdd": list(c.get("add_capabilities") or []),
        "CapDrop": list(c.get("drop_capabilities") or []),
        "Devices": [{"PathOnHost": d["host_path"], "PathInContainer": d["container_path"],
                     "CgroupPermissions": d.get("mode") or "mrw"} for d in c.get("devices") or []],
        "SecurityOpt": [], "GroupAdd": [],
    }
    if c.get("shm_size"):
        host["ShmSize"] = int(c["shm_size"])
    rocm = [d for d in devices if d.get("type") == "rocm"]
    if rocm:
        host["SecurityOpt"].append("seccomp=unconfined")
        host["GroupAdd"].append("video")
        for p in rocm_device_paths(rocm, dev_root):
            host["Devices"].append({"PathOnHost": p, "PathInContainer": p, "CgroupPermissions": "rwm"})
    cenv = to_container_paths(env, ctx_dir, framework_root)
    cenv["DET_CONTAINER_ID"] = spec["allocation_id"]
    cenv["DET_SLOT_IDS"] = "[" + ",".join(str(d["id"]) for d in devices) + "]"
    return {
        "Image": image_for(c, devices),
        "Cmd": container_cmd(cmd), "Env": [f"{k}={v}" for k, v in sorted(cenv.items())],
        "WorkingDir": WORKDIR, "Tty": False,
        "Labels": {LABEL_AGENT: agent_id, LABEL_ALLOC: spec["allocation_id"], LABEL_TASK: spec["task_id"],
                   LABEL_SLOTS: ",".join(str(d["id"]) for d in devices), LABEL_VERSION: "1"},
        "HostConfig": host,
    }


# ----------------------------------------------------------------------------- process adapters
class _LineReader:
    """File-like ``readline()`` over a byte-chunk iterator (the container's log stream)."""

    def __init__(self, chunks: Iterator[bytes]) -> None:
        self._chunks = chunks
        self._buf = b""
        self._eof = False

    def readline(self) -> bytes:
        while b"\n" not in self._buf and not self._eof:
            try:
                self._buf += next(self._chunks)
            except (StopIteration, OSError, http.client.HTTPException):
                self._eof = True
        if b"\n" in self._buf:
            line, self._buf = self._buf.split(b"\n", 1)
            return line + b"\n"
        line, self._buf = self._buf, b""
        return line


class ContainerProcess:
    """A running task container with the subset of ``subprocess.Popen`` the agent uses:
    ``stdout.readline()`` (its logs), ``wait()``, ``poll()``, ``send_signal()``; ``remove()``
    deletes it once its exit was reported."""

    def __init__(self, client: EngineClient, cid: str, since: Optional[float] = None) -> None:
        self.client, self.id = client, cid
        self.pid = None
        self.returncode: Optional[int] = None
        self.stdout = _LineReader(client.logs(cid, since=since))
        self._lock = threading.Lock()

    def wait(self) -> int:
        with self._lock:
            if self.returncode is None:
                self.returncode = self.client.wait(self.id)
            return self.returncode

    def poll(self) -> Optional[int]:
        if self.returncode is not None:
            return self.returncode
        st = self.client.inspect(self.id).get("State") or {}
        if st.get("Running"):
            return None
        self.returncode = int(st.get("ExitCode", 0))
        return self.returncode

    def send_signal(self, sig: str) -> None:
        self.client.kill(self.id, sig)

    def remove(self) -> None:
        self.client.remove(self.id, force=True)


class EngineRuntime:
    """Docker (or Podman) container runtime of an agent."""

    kind = "docker"

    def __init__(self, agent_id: str, socket_path: str = DEFAULT_DOCKER_SOCKET,
                 dev_root: str = "/dev", network_mode: str = "host", kind: str = "docker") -> None:
        self.client = EngineClient(socket_path)
        self.agent_id = agent_id
        self.dev_root = dev_root
        self.network_mode = network_mode
        self.kind = kind

    def available(self) -> bool:
        return self.client.ping()

    def ensure_image(self, spec: Dict[str, Any], image: str) -> None:
        c = spec.get("container") or {}
        if c.get("force_pull_image") or not self.client.image_exists(image):
            self.client.pull(image, c.get("registry_auth"))

    def launch(self, spec: Dict[str, Any], cmd: List[str], env: Dict[str, str], ctx_dir: str,
               devices: List[Dict[str, Any]], framework_root: str) -> ContainerProcess:
        config = engine_config(spec, cmd, env, ctx_dir, devices, self.agent_id, framework_root,
                               self.dev_root, self.network_mode)
        self.ensure_image(spec, config["Image"])
        name = "det-" + spec["allocation_id"].replace("/", "_").replace(".", "-")
        cid = self.client.create(name, config)
        self.client.start(cid)
        return ContainerProcess(self.client, cid)  # logs are kept: none missed after the start

    def reattach(self) -> List[Tuple[Dict[str, str], ContainerProcess, Optional[int]]]:
        """This agent's containers left by a previous agent process: (labels, process, exit
        code if it already exited). Running ones are followed from now on."""
        out = []
        for c in self.client.list({LABEL_AGENT: self.agent_id}, all=True):
            labels = c.get("Labels") or {}
            proc = ContainerProcess(self.client, c["Id"], since=time.time())
            code = proc.poll()
            out.append((labels, proc, code))
        return out


class ApptainerProcess(subprocess.Popen):
    def remove(self) -> None:
        pass


class ApptainerRuntime:
    """Apptainer / Singularity: the task runs as ``apptainer exec`` (reference
    agent/pkg/singularity): ``--rocm`` binds the GPU stack and ``ROCR_VISIBLE_DEVICES`` selects
    the task's devices; bind mounts become ``--bind src:dst[:ro]``; the image is a ``docker://``
    reference or a local ``.sif`` path."""

    kind = "apptainer"

    def __init__(self, binary: str = "apptainer") -> None:
        self.binary = binary

    def available(self) -> bool:
        import shutil

        return shutil.which(self.binary) is not None

    def argv(self, spec: Dict[str, Any], cmd: List[str], env: Dict[str, str], ctx_dir: str,
             devices: List[Dict[str, Any]], framework_root: str) -> Tuple[List[str], Dict[str, str]]:
        c = spec.get("container") or {}
        image = image_for(c, devices)
        if not (image.startswith(("docker://", "oras://", "library://", "/")) or image.endswith(".sif")):
            image = "docker://" + image
        argv = [self.binary, "exec", "--pwd", WORKDIR, "--bind", f"{ctx_dir}:{WORKDIR}",
                "--bind", f"{framework_root}:{FRAMEWORK_MOUNT}:ro"]
        for m in container_mounts(spec, ctx_dir, framework_root)[2:]:
            argv += ["--bind", f"{m['Source']}:{m['Target']}" + (":ro" if m["ReadOnly"] else "")]
        rocm = [d for d in devices if d.get("type") == "rocm"]
        cenv = to_container_paths(env, ctx_dir, framework_root)
        if rocm:
            argv.append("--rocm")
            cenv["ROCR_VISIBLE_DEVICES"] = ",".join(
                str(i) for i in sorted({int(d.get("device_index", d["id"])) for d in rocm}))
        # APPTAINERENV_* is how apptainer passes variables into the container
        host_env = {k: v for k, v in os.environ.items() if k in ("PATH", "HOME", "USER", "TMPDIR")}
        host_env.update({f"APPTAINERENV_{k}": v for k, v in cenv.items()})
        return argv + [image] + container_cmd(cmd), host_env

    def launch(self, spec: Dict[str, Any], cmd: List[str], env: Dict[str, str], ctx_dir: str,
               devices: List[Dict[str, Any]], framework_root: str) -> subprocess.Popen:
        argv, henv = self.argv(spec, cmd, env, ctx_dir, devices, framework_root)
        logger.info("apptainer: " + " ".join(shlex.quote(a) for a in argv))
        return ApptainerProcess(argv, cwd=ctx_dir, env=henv, stdout=subprocess.PIPE,
                                stderr=subprocess.STDOUT, start_new_session=True)

    def reattach(self) -> List[Any]:
        return []  # apptainer containers are children of the agent: they end with it


def make_runtime(kind: str, agent_id: str, socket_path: Optional[str] = None,
                 dev_root: str = "/dev") -> Optional[Any]:
    """``process`` -> None (plain process groups); ``docker`` / ``podman`` / ``apptainer`` ->
    that runtime (an error if it is unreachable); ``auto`` -> Docker, then Podman, when their
    socket answers, else None (the process runtime is the fallback)."""
    kind = (kind or "auto").lower()
    if kind == "process":
        return None
    if kind == "apptainer":
        rt = ApptainerRuntime()
        if not rt.available():
            raise RuntimeError("apptainer not found on PATH")
        return rt
    cands = []
    if kind in ("auto", "docker"):
        cands.append(("docker", socket_path or os.environ.get("DOCKER_HOST", "").replace("unix://", "")
                      or DEFAULT_DOCKER_SOCKET))
    if kind in ("auto", "podman"):
        cands.append(("podman", socket_path or default_podman_socket()))
    for name, sock in cands:
        rt = EngineRuntime(agent_id, sock, dev_root=dev_root, kind=name)
        if os.path.exists(sock) and rt.available():
            logger.info(f"container runtime: {name} at {sock}")
            return rt
    if kind != "auto":
        raise RuntimeError(f"{kind} daemon not reachable at {cands[0][1]}")
    logger.info("no container daemon reachable: tasks run as process groups")
    return None
