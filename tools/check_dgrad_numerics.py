"""Numerics of the big data-gradient GEMMs dX = dY @ W, NN (W as stored) and TN (transposed copy),
against an fp32 reference computed in 131072-row chunks, with the shipped TunableOp results
replayed (DCA_GEMM_TUNED=1, default) or the library heuristic (DCA_GEMM_TUNED=0).
Usage: python tools/check_dgrad_numerics.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DCA_GEMM_TUNED", "1")

import torch  # noqa: E402

from determined_clone_amd.ops import gemm_tuning  # noqa: E402

SHAPES = [(3211264, 64, 256), (3211264, 256, 64), (3211264, 128, 256), (3211264, 64, 64),
          (802816, 128, 512), (200704, 256, 1024), (32768, 4096, 1024)]


def main():
    tuned = gemm_tuning.enable()
    torch.manual_seed(0)
    for rows, out, inp in SHAPES:
        dy = torch.randn(rows, out, device="cuda", dtype=torch.bfloat16)
        w = (torch.randn(out, inp, device="cuda") * 0.05).to(torch.bfloat16)
        res = {"rows": rows, "out": out, "in": inp, "tuned": tuned}
        nn = torch.mm(dy, w)
        tn = torch.mm(dy, w.t().contiguous().t())
        wf = w.float()
        for name, got in (("nn", nn), ("tn", tn)):
            worst, where = 0.0, -1
            for lo in range(0, rows, 131072):
                ref = dy[lo:lo + 131072].float() @ wf
                e = (got[lo:lo + 131072].float() - ref).abs()
                m = e.max().item()
                if m > worst:
                    worst, where = m, lo + int(e.max(dim=1).values.argmax().item())
            res[f"{name}_max_err"] = round(worst, 5)
            res[f"{name}_worst_row"] = where
        print(json.dumps(res), flush=True)
        del dy, w, nn, tn


if __name__ == "__main__":
    main()
