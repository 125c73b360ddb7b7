"""In-tree build of the MI355X (gfx950) HIP kernel extension ``determined_clone_amd.ops._C``.

No hipify, no torch JIT cache: every ``csrc/*.hip`` is compiled by ``hipcc --offload-arch=gfx950``
and the pybind11 glue (``csrc/*.cpp``) by hipcc as host C++, then linked against the torch
libraries of the running interpreter into ``ops/_C.so`` next to this file
(``python -m determined_clone_amd.ops.build [--force]``).

Staleness is decided by CONTENT, not mtime: every object carries a sidecar with the hash of its
source, the headers and the compile command, and is rebuilt when that differs. The hash of the whole
``csrc/`` tree (:func:`source_hash`) is compiled into the extension (``_C.source_hash``), and
``ops._ext.load()`` refuses a binary whose hash does not match the sources next to it.
"""
import argparse
import concurrent.futures
import hashlib
import os
import pathlib
import subprocess
import sys
import sysconfig
from typing import List, Optional, Sequence

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


def source_hash() -> str:
    """sha256 over the names and bytes of every ``csrc/`` source and header plus the target arch and
    per-file flags: the identity of a correct ``_C.so`` for this tree."""
    h = hashlib.sha256()
    h.update(f"arch={ARCH};flags={sorted(_FILE_FLAGS.items())}".encode())
    for f in sorted(CSRC.iterdir()):
        if f.suffix in (".hip", ".cpp", ".h"):
            h.update(f.name.encode() + b"\0" + f.read_bytes() + b"\0")
    return h.hexdigest()


def _obj_key(src: pathlib.Path, headers: List[pathlib.Path], cmd: List[str]) -> str:
    h = hashlib.sha256(" ".join(cmd[3:]).encode())  # flags (not the object path)
    for f in [src] + headers:
        h.update(f.read_bytes())
    return h.hexdigest()


def _stale(obj: pathlib.Path, key: str) -> bool:
    side = obj.with_suffix(obj.suffix + ".key")
    return not obj.exists() or not side.exists() or side.read_text() != key


def _compile(cmd: List[str], key: str = "") -> None:
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError("compile failed:\n" + " ".join(cmd) + "\n" + proc.stdout)
    if key:  # record what the object was built from (after a successful compile only)
        out = pathlib.Path(cmd[cmd.index("-o") + 1])
        out.with_suffix(out.suffix + ".key").write_text(key)


def build(force: bool = False, verbose: bool = False, jobs: int = 0, defines: Sequence[str] = (),
          target: Optional[pathlib.Path] = None) -> pathlib.Path:
    """Build ``_C.so`` (or, with ``defines`` / ``target``, an A/B variant of it in its own object
    directory -- loaded through ``DCA_OPS_SO``, never by default)."""
    inc, lib, abi = _torch_paths()
    variant = bool(defines) or target is not None
    TARGET_ = target or TARGET
    BUILD_ = BUILD if not variant else BUILD / ("variant_" + hashlib.sha1(" ".join(defines).encode()).hexdigest()[:10])
    dflags = [f"-D{d}" for d in defines]
    BUILD_.mkdir(parents=True, exist_ok=True)
    headers = sorted(CSRC.glob("*.h"))
    jobs_list, objs = [], []
    for src in sorted(CSRC.glob("*.hip")):
        obj = BUILD_ / (src.stem + ".hip.o")
        objs.append(obj)
        cmd = [_hipcc(), "-c", str(src), "-o", str(obj), f"--offload-arch={ARCH}",
               "-munsafe-fp-atomics", f"-I{CSRC}"] + _common_flags(abi) + _FILE_FLAGS.get(src.stem, []) + dflags
        key = _obj_key(src, headers, cmd)
        if force or _stale(obj, key):
            jobs_list.append((cmd, key))
    py_inc = sysconfig.get_paths()["include"]
    for src in sorted(CSRC.glob("*.cpp")):
        obj = BUILD_ / (src.stem + ".cpp.o")
        objs.append(obj)
        cmd = [_hipcc(), "-c", str(src), "-o", str(obj), f"-I{CSRC}", f"-I{py_inc}",
               "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H"] + [f"-I{p}" for p in inc] \
            + _common_flags(abi)
        key = _obj_key(src, headers, cmd)
        if force or _stale(obj, key):
            jobs_list.append((cmd, key))
    # the source hash as a linked-in symbol (bindings.cpp exposes it as _C.source_hash)
    digest = source_hash()
    hsrc, hobj = BUILD_ / "source_hash.cpp", BUILD_ / "source_hash.cpp.o"
    objs.append(hobj)
    hcode = f'extern "C" const char dca_source_hash[] = "{digest}";\n'
    if not hsrc.exists() or hsrc.read_text() != hcode:
        hsrc.write_text(hcode)
    hcmd = [_hipcc(), "-c", str(hsrc), "-o", str(hobj), "-fPIC", "-O1"]
    if force or _stale(hobj, digest):
        jobs_list.append((hcmd, digest))
    jobs = jobs or min(8, os.cpu_count() or 4)
    with concurrent.futures.ThreadPoolExecutor(max_workers=jobs) as ex:
        for cmd, _ in jobs_list:
            if verbose:
                print(" ".join(cmd), flush=True)
        list(ex.map(lambda ck: _compile(*ck), jobs_list))
    if variant:
        if jobs_list or force or not TARGET_.exists():
            _compile([_hipcc(), "-shared", "-fPIC", "-o", str(TARGET_)] + [str(o) for o in objs]
                     + _link_flags(lib))
        return TARGET_
    if jobs_list or force or not TARGET.exists() or linked_hash() != digest:
        link = [_hipcc(), "-shared", "-fPIC", "-o", str(TARGET)] + [str(o) for o in objs] + [
            f"--offload-arch={ARCH}", f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
            "-ltorch_hip", "-ltorch_python", "-lamdhip64", "-lhipblaslt", f"-Wl,-rpath,{lib}"]
        if verbose:
            print(" ".join(link), flush=True)
        _compile(link)
        LINKED.write_text(digest)
    return TARGET


def _link_flags(lib: str) -> List[str]:
    return [f"--offload-arch={ARCH}", f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
            "-ltorch_hip", "-ltorch_python", "-lamdhip64", "-lhipblaslt", f"-Wl,-rpath,{lib}"]


LINKED = HERE / "_C.so.hash"  # next to _C.so (travels with it); the embedded hash stays authoritative


def linked_hash() -> str:
    """The source hash recorded when ``_C.so`` was last linked ("" if unknown)."""
    return LINKED.read_text().strip() if LINKED.exists() and TARGET.exists() else ""


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("-D", dest="defines", action="append", default=[],
                    help="A/B variant: compile with this define (needs --out)")
    ap.add_argument("--out", default=None, help="A/B variant: output .so path (load via DCA_OPS_SO)")
    args = ap.parse_args()
    out = build(force=args.force, verbose=args.verbose, jobs=args.jobs, defines=args.defines,
                target=pathlib.Path(args.out).resolve() if args.out else None)
    print(f"built {out}")


if __name__ == "__main__":
    sys.exit(main())
