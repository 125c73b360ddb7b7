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


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
    print(build_pidwatch(force="--force" in sys.argv))
