"""Data-gradient GEMM layout probe: dX = dY @ W with W [out, in] as stored (NN) vs on a transposed
copy (TN, the forward GEMMs' layout; the copy's time included), on the GPT-2-medium linears
(32k tokens) and ResNet-50's 1x1 convolutions (bs 1024), replaying the shipped TunableOp results.
Prints one JSON line per shape. Usage: python tools/probe_dgrad_tn.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DCA_GEMM_TUNED", "1")

import torch  # noqa: E402

from determined_clone_amd.ops import gemm_tuning  # noqa: E402

# (rows, out, in): GPT-2 linears, then ResNet-50 pointwise convolutions (rows = N*H*W)
SHAPES = [(32768, 3072, 1024), (32768, 1024, 1024), (32768, 4096, 1024), (32768, 1024, 4096),
          (32768, 50304, 1024),
          (3211264, 64, 256), (3211264, 256, 64), (3211264, 64, 64), (3211264, 128, 256),
          (802816, 128, 512), (802816, 512, 128), (802816, 256, 512), (802816, 512, 256),
          (200704, 256, 1024), (200704, 1024, 256), (200704, 512, 1024), (200704, 1024, 512),
          (50176, 512, 2048), (50176, 2048, 512), (50176, 1024, 2048)]


def _time(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    gemm_tuning.enable()
    torch.manual_seed(0)
    for rows, out, inp in SHAPES:
        dy = torch.randn(rows, out, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(out, inp, device="cuda", dtype=torch.bfloat16) * 0.05
        nn_us = _time(lambda: torch.mm(dy, w))
        tn_us = _time(lambda: torch.mm(dy, w.t().contiguous().t()))
        wt = w.t().contiguous()
        tn_only_us = _time(lambda: torch.mm(dy, wt.t()))
        ref = torch.mm(dy, w).float()
        err = (torch.mm(dy, wt.t()).float() - ref).abs().max().item()
        fl = 2.0 * rows * out * inp
        print(json.dumps({"rows": rows, "out": out, "in": inp, "nn_us": round(nn_us, 1),
                          "tn_with_copy_us": round(tn_us, 1), "tn_us": round(tn_only_us, 1),
                          "nn_tf": round(fl / nn_us / 1e6, 1), "tn_tf": round(fl / tn_only_us / 1e6, 1),
                          "max_abs_diff": err}), flush=True)
        del dy, w, wt, ref


if __name__ == "__main__":
    main()
