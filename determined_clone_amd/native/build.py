"""In-tree build of the native runtime module ``determined_clone_amd.native._native`` (C++17,
pybind11): scheduler (priority / fair-share / round-robin, best/worst fit, gang placement) and KFD
device detection. ``python -m determined_clone_amd.native.build``."""
import os
import pathlib
import subprocess
import sys
import sysconfig

HERE = pathlib.Path(__file__).resolve().parent
SOURCES = [HERE / "scheduler.cpp"]
TARGET = HERE / ("_native" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
PIDWATCH_SRC = HERE / "pidwatch.cpp"
PIDWATCH = HERE / "bin" / "dca-pidwatch"


def build_pidwatch(force: bool = False) -> pathlib.Path:
    """Standalone launcher-side failure detector (no Python, no GPU)."""
    if not force and PIDWATCH.exists() and PIDWATCH.stat().st_mtime >= PIDWATCH_SRC.stat().st_mtime:
        return PIDWATCH
    PIDWATCH.parent.mkdir(exist_ok=True)
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-Wall", str(PIDWATCH_SRC), "-o", str(PIDWATCH)]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("pidwatch build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return PIDWATCH


def build(force: bool = False) -> pathlib.Path:
    import pybind11

    if not force and TARGET.exists() and all(TARGET.stat().st_mtime >= s.stat().st_mtime for s in SOURCES):
        return TARGET
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wno-unused-function",
           f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
           *[str(s) for s in SOURCES], "-o", str(TARGET)]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return TARGET


# ------------------------------------------------------------------ sanitizer builds (CPU only)
# The reference tests its Go master with `go test -race`; the native pieces of ours (the scheduler
# module the threaded Python master calls with the GIL released, and the pidwatch launcher) get
# AddressSanitizer(+UBSan) and ThreadSanitizer builds instead, exercised by
# tests/test_native_sanitizers.py from multiple Python threads / processes.
SANITIZERS = {
    "asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"],
    "tsan": ["-fsanitize=thread"],
}
RUNTIME_LIB = {"asan": "libasan.so", "tsan": "libtsan.so"}


def sanitizer_runtime(kind: str) -> str:
    """Path of the sanitizer runtime to LD_PRELOAD into an uninstrumented Python."""
    cxx = os.environ.get("CXX", "g++")
    out = subprocess.run([cxx, f"-print-file-name={RUNTIME_LIB[kind]}"], stdout=subprocess.PIPE,
                         text=True).stdout.strip()
    return out if os.path.isabs(out) and os.path.exists(out) else ""


def build_sanitized(kind: str, force: bool = False) -> "tuple[pathlib.Path, pathlib.Path]":
    """(scheduler module, pidwatch binary) built with the ``kind`` sanitizer under native/_san/."""
    import pybind11

    out = HERE / "_san" / kind
    out.mkdir(parents=True, exist_ok=True)
    mod = out / TARGET.name
    pw = out / "dca-pidwatch"
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O1", "-g", "-std=c++17", *SANITIZERS[kind]]
    jobs = []
    if force or not mod.exists() or mod.stat().st_mtime < max(s.stat().st_mtime for s in SOURCES):
        jobs.append([cxx, *flags, "-shared", "-fPIC", "-Wno-unused-function", f"-I{pybind11.get_include()}",
                     f"-I{sysconfig.get_paths()['include']}", *[str(s) for s in SOURCES], "-o", str(mod)])
    if force or not pw.exists() or pw.stat().st_mtime < PIDWATCH_SRC.stat().st_mtime:
        jobs.append([cxx, *flags, str(PIDWATCH_SRC), "-o", str(pw)])
    for cmd in jobs:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"{kind} build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return mod, pw


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
    print(build_pidwatch(force="--force" in sys.argv))
