"""ResNet-50 (bs256, NHWC bf16) pointwise convolutions: MIOpen vs the MFMA kernels of
ops/csrc/conv1x1.hip, per pass (fwd / dgrad / wgrad), weighted by each shape's count in the net.

Prints one JSON line per shape plus a total; HBM-roofline time (in+out bytes at 5 TB/s) for scale.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(ROOT, "tools", "miopen", "db"))
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(ROOT, "tools", "miopen", "cache"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from determined_clone_amd.ops import _ext  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


# (H, Cin, Cout, count of stride-1 1x1 convolutions of this shape in ResNet-50)
SHAPES = [(56, 64, 64, 1), (56, 256, 64, 2), (56, 64, 256, 4), (56, 256, 128, 1),
          (28, 128, 512, 4), (28, 512, 128, 3), (28, 512, 256, 1),
          (14, 256, 1024, 6), (14, 1024, 256, 5), (14, 1024, 512, 1),
          (7, 512, 2048, 3), (7, 2048, 512, 2)]


def main():
    torch.backends.cudnn.benchmark = True
    C = _ext.load()
    N = int(os.environ.get("BATCH", "256"))
    tot = {k: 0.0 for k in ("mi_fwd", "mi_dgrad", "mi_wgrad", "our_fwd", "our_dgrad", "our_wgrad", "roof")}
    for H, ci, co, cnt in SHAPES:
        x = torch.randn(N, ci, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, 1, 1, device="cuda") / ci ** 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, co, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        acc = torch.zeros(co, ci, 1, 1, device="cuda", dtype=torch.bfloat16)

        def mi_bwd(mask):
            return torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (0, 0), (1, 1), False,
                                                       (0, 0), 1, mask)

        r = {
            "mi_fwd": timeit(lambda: F.conv2d(x, w)),
            "mi_dgrad": timeit(lambda: mi_bwd([True, False, False])),
            "mi_wgrad": timeit(lambda: mi_bwd([False, True, False])),
            "our_fwd": timeit(lambda: C.conv1x1_fwd(x, w, True)),
            "our_dgrad": timeit(lambda: C.conv1x1_dgrad(dy, w)),
            "our_wgrad": timeit(lambda: C.conv1x1_wgrad(dy, x, w, acc)),
        }
        M = N * H * H
        r["roof"] = 3 * (M * (ci + co) * 2) / 5e12 * 1e3
        for k, v in r.items():
            tot[k] += v * cnt
        fl = 2 * M * ci * co
        out = {"H": H, "cin": ci, "cout": co, "count": cnt}
        out.update({k: round(v, 4) for k, v in r.items()})
        out["our_fwd_tflops"] = round(fl / r["our_fwd"] / 1e9, 1)
        out["our_wgrad_tflops"] = round(fl / r["our_wgrad"] / 1e9, 1)
        out["our_fwd_GBps"] = round(M * (ci + co) * 2 / r["our_fwd"] / 1e6, 0)
        print(json.dumps(out), flush=True)
    tot = {k: round(v, 3) for k, v in tot.items()}
    tot["miopen_total"] = round(tot["mi_fwd"] + tot["mi_dgrad"] + tot["mi_wgrad"], 3)
    tot["ours_total"] = round(tot["our_fwd"] + tot["our_dgrad"] + tot["our_wgrad"], 3)
    print(json.dumps({"per_step_ms_weighted": tot}), flush=True)


if __name__ == "__main__":
    main()
