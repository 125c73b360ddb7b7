"""Check every shipped TunableOp result (``ops/tuned/gemm_gfx950.csv``) for correct numbers.

TunableOp keeps the fastest solution per GEMM shape without comparing its output to anything
(its numerical check is off by default), so a solution that is fast because it computes the wrong
thing can be shipped. This replays the file and, for each row, runs that exact GEMM (transposes,
m/n/k, leading dimensions; the bias epilogue for GemmAndBias rows) through torch on random inputs
and compares it with an fp32 reference computed in row chunks. Prints one JSON line per row and
a summary; ``--drop-bad OUT`` writes the file without the failing rows.

Usage: python tools/validate_tuned_gemms.py [--csv PATH] [--drop-bad OUT] [--tol 0.1]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from determined_clone_amd.ops import gemm_tuning  # noqa: E402


def parse(line: str):
    parts = line.rstrip("\n").split(",")
    if len(parts) < 3 or parts[0] == "Validator":
        return None
    op, key = parts[0], parts[1]
    if not (op.startswith("GemmTunableOp_BFloat16_") or op.startswith("GemmAndBiasTunableOp_BFloat16_")):
        return None
    f = key.split("_")
    # "<ta><tb>_<m>_<n>_<k>_ld_<lda>_<ldb>_<ldc>"
    ta, tb = f[0][0], f[0][1]
    m, n, k = int(f[1]), int(f[2]), int(f[3])
    lda, ldb, ldc = int(f[5]), int(f[6]), int(f[7])
    return dict(op=op, key=key, ta=ta, tb=tb, m=m, n=n, k=k, lda=lda, ldb=ldb, ldc=ldc,
                bias=op.startswith("GemmAndBias"), solution=parts[2])


def operands(r, g, dev="cuda"):
    """torch operands L [n, k], R [k, m] whose ``L @ R`` is the column-major GEMM of row ``r``."""
    dt = torch.bfloat16
    m, n, k = r["m"], r["n"], r["k"]
    s = 1.0 / k ** 0.5
    if r["ta"] == "n":  # A: column-major [m x k], lda >= m  ->  R = row-major [k, lda][:, :m]
        R = (torch.randn(k, r["lda"], device=dev, generator=g) * s).to(dt)[:, :m]
    else:  # A^T: column-major [k x m], lda >= k  ->  R = ([m, lda][:, :k]).t()
        R = (torch.randn(m, r["lda"], device=dev, generator=g) * s).to(dt)[:, :k].t()
    if r["tb"] == "n":  # B: column-major [k x n], ldb >= k  ->  L = [n, ldb][:, :k]
        L = torch.randn(n, r["ldb"], device=dev, generator=g).to(dt)[:, :k]
    else:  # B^T: column-major [n x k], ldb >= n  ->  L = ([k, ldb][:, :n]).t()
        L = torch.randn(k, r["ldb"], device=dev, generator=g).to(dt)[:, :n].t()
    return L, R


def check(r, tol: float, g) -> dict:
    out = dict(op=r["op"], key=r["key"], solution=r["solution"])
    if r["ldc"] != r["m"]:
        out["skipped"] = "ldc != m"
        return out
    L, R = operands(r, g)
    bias = None
    if r["bias"]:
        bias = torch.randn(r["m"], device="cuda", generator=g).to(torch.bfloat16)
        got = torch.addmm(bias, L, R)
    else:
        got = torch.mm(L, R)
    import torch.cuda.tunable as tunable

    tunable.enable(False)  # the fp32 reference GEMMs run untuned (and are never tuned)
    Rf = R.float()
    worst, scale, where = 0.0, 0.0, -1
    step = max(1, (1 << 28) // max(1, r["m"] + r["k"]))
    for lo in range(0, r["n"], step):
        ref = L[lo:lo + step].float() @ Rf
        if bias is not None:
            ref += bias.float()
        e = (got[lo:lo + step].float() - ref).abs()
        mx = e.max().item()
        scale = max(scale, ref.abs().max().item())
        if mx > worst:
            worst, where = mx, lo + int(e.max(dim=1).values.argmax().item())
    tunable.enable(True)
    out.update(max_err=round(worst, 5), ref_max=round(scale, 3), worst_row=where, ok=worst <= tol)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--csv", default=gemm_tuning.RESULTS)
    ap.add_argument("--drop-bad", default="")
    ap.add_argument("--tol", type=float, default=0.1)
    ap.add_argument("--also", action="append", default=[],
                    help="extra 'op,key' rows to run (with DCA_GEMM_TUNE=<file>: tuned into it)")
    a = ap.parse_args()
    os.environ["DCA_GEMM_TUNED"] = "1"
    if not gemm_tuning.enable(a.csv):
        raise SystemExit("TunableOp could not be enabled")
    g = torch.Generator(device="cuda").manual_seed(0)
    lines = open(a.csv).read().splitlines(keepends=True)
    extra = [f"{x},extra,0\n" for x in a.also]
    # tuning run (DCA_GEMM_TUNE): only the extra rows (the file's rows are replayed as they are)
    todo = extra if os.environ.get("DCA_GEMM_TUNE") else lines + extra
    bad = set()
    n_ok = 0
    for line in todo:
        r = parse(line)
        if r is None:
            continue
        res = check(r, a.tol, g)
        print(json.dumps(res), flush=True)
        if res.get("ok") is False:
            bad.add((r["op"], r["key"]))
        elif res.get("ok"):
            n_ok += 1
        torch.cuda.empty_cache()
    print(json.dumps({"summary": {"ok": n_ok, "bad": sorted(k for _, k in bad)}}), flush=True)
    if a.drop_bad:
        with open(a.drop_bad, "w") as f:
            for line in lines:
                r = parse(line)
                if r is None or ((r["op"], r["key"]) not in bad and r["solution"] != "extra"):
                    f.write(line)


if __name__ == "__main__":
    main()
