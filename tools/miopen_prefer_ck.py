"""Write a copy of the shipped MIOpen find DB in which, for forward / backward-data problems, the
CK implicit-GEMM solution (``ConvHipImplicitGemmGroup*Xdlops``: writes bf16 directly, no
workspace) is preferred over the ASM one (``ConvAsmImplicitGemmGTCDynamic*XdlopsNHWC``: fp32
workspace + zero-fill + cast passes, profiles/round2_miopen_subtensor_ops.txt) whenever its
isolated find time is within ``--slack`` of the ASM time. Immediate mode picks the fastest
recorded time, so the ASM time is raised just above the CK one.

    python tools/miopen_prefer_ck.py SRC_DB_DIR DST_DB_DIR [--slack 1.10] [--dirs F,B]
"""
import argparse
import os
import shutil


def rewrite(line: str, slack: float, dirs: str) -> str:
    key, _, rest = line.rstrip("\n").partition("=")
    if not rest or key[-1:] not in dirs:
        return line
    sols = [s.split(":", 1) for s in rest.split(";")]
    times = {}
    for name, val in sols:
        times[name] = float(val.split(",")[0])
    ck = next((n for n in times if n.startswith("ConvHipImplicitGemmGroup")), None)
    asm = next((n for n in times if n.startswith("ConvAsmImplicitGemmGTCDynamic")), None)
    if ck is None or asm is None or times[ck] <= times[asm] or times[ck] > slack * times[asm]:
        return line
    out = []
    for name, val in sols:
        parts = val.split(",")
        if name == asm:
            parts[0] = f"{times[ck] * 1.01:.6g}"
        out.append(name + ":" + ",".join(parts))
    return key + "=" + ";".join(out) + "\n"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--slack", type=float, default=1.10)
    ap.add_argument("--dirs", default="F,B")
    a = ap.parse_args()
    dirs = "".join(a.dirs.split(","))
    os.makedirs(a.dst, exist_ok=True)
    changed = 0
    for f in os.listdir(a.src):
        src, dst = os.path.join(a.src, f), os.path.join(a.dst, f)
        if f.endswith(".ufdb.txt"):
            with open(src) as fi, open(dst, "w") as fo:
                for line in fi:
                    new = rewrite(line, a.slack, dirs)
                    changed += new != line
                    fo.write(new)
        else:
            shutil.copy2(src, dst)
    print(f"{changed} find-DB entries now prefer the CK solution")


if __name__ == "__main__":
    main()
