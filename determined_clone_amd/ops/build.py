"""In-tree build of the MI355X (gfx950) HIP kernel extension ``determined_clone_amd.ops._C``.

No hipify, no torch JIT cache: every ``csrc/*.hip`` is compiled by ``hipcc --offload-arch=gfx950``
and the pybind11 glue (``csrc/*.cpp``) by hipcc as host C++, then linked against the torch
libraries of the running interpreter into ``ops/_C.so`` next to this file. Objects are rebuilt only
when a source or header is newer (``python -m determined_clone_amd.ops.build [--force]``).
"""
import argparse
import concurrent.futures
import os
import pathlib
import subprocess
import sys
import sysconfig
from typing import List

HERE = pathlib.Path(__file__).resolve().parent
CSRC = HERE / "csrc"
BUILD = HERE / "_build"
TARGET = HERE / "_C.so"
ARCH = os.environ.get("DCA_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    return os.path.join(rocm, "bin", "hipcc")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension

    inc = cpp_extension.include_paths()
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _common_flags(abi: int) -> List[str]:
    return ["-O3", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
            "-D__HIP_PLATFORM_AMD__=1", "-Wno-unused-result", "-Wno-deprecated-declarations"]


# per-source extra flags. attention.hip: no SLP vectorizer -- it packs the softmax-gradient
# subtract/multiply pairs into v_pk_add_f32 / v_pk_mul_f32, which cost ~24 extra cycles each beside
# MFMAs on gfx950 (cdna guide: packed f32 VALU is an anti-lever in MFMA loops)
_FILE_FLAGS = {"attention": [] if os.environ.get("DCA_BUILD_SLP") else ["-fno-slp-vectorize"]}


def _newer(src: pathlib.Path, obj: pathlib.Path, headers: List[pathlib.Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(h.stat().st_mtime > t for h in headers)


def _compile(cmd: List[str]) -> None:
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError("compile failed:\n" + " ".join(cmd) + "\n" + proc.stdout)


def build(force: bool = False, verbose: bool = False, jobs: int = 0) -> pathlib.Path:
    inc, lib, abi = _torch_paths()
    BUILD.mkdir(exist_ok=True)
    headers = sorted(CSRC.glob("*.h"))
    cmds, objs = [], []
    for src in sorted(CSRC.glob("*.hip")):
        obj = BUILD / (src.stem + ".hip.o")
        objs.append(obj)
        if force or _newer(src, obj, headers):
            cmds.append([_hipcc(), "-c", str(src), "-o", str(obj), f"--offload-arch={ARCH}",
                         "-munsafe-fp-atomics", f"-I{CSRC}"] + _common_flags(abi)
                        + _FILE_FLAGS.get(src.stem, []))
    py_inc = sysconfig.get_paths()["include"]
    for src in sorted(CSRC.glob("*.cpp")):
        obj = BUILD / (src.stem + ".cpp.o")
        objs.append(obj)
        if force or _newer(src, obj, headers):
            cmds.append([_hipcc(), "-c", str(src), "-o", str(obj), f"-I{CSRC}", f"-I{py_inc}",
                         "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H"]
                        + [f"-I{p}" for p in inc] + _common_flags(abi))
    jobs = jobs or min(8, os.cpu_count() or 4)
    with concurrent.futures.ThreadPoolExecutor(max_workers=jobs) as ex:
        for cmd in cmds:
            if verbose:
                print(" ".join(cmd), flush=True)
        list(ex.map(_compile, cmds))
    if cmds or force or not TARGET.exists():
        link = [_hipcc(), "-shared", "-fPIC", "-o", str(TARGET)] + [str(o) for o in objs] + [
            f"--offload-arch={ARCH}", f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
            "-ltorch_hip", "-ltorch_python", "-lamdhip64", "-lhipblaslt", f"-Wl,-rpath,{lib}"]
        if verbose:
            print(" ".join(link), flush=True)
        _compile(link)
    return TARGET


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    args = ap.parse_args()
    out = build(force=args.force, verbose=args.verbose, jobs=args.jobs)
    print(f"built {out}")


if __name__ == "__main__":
    sys.exit(main())
