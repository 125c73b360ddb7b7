"""1x1 convolutions of ResNet-50 (bs256, NHWC bf16): MIOpen (F.conv2d) vs hipBLASLt GEMM (torch.mm)
for fwd / bwd-data / bwd-weight. Decides whether 1x1 convs should bypass MIOpen."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from determined_clone_amd.ops import miopen_db  # noqa: E402

miopen_db.use_private_copy("tools")  # never write the shipped DB from a bench

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def t(fn, it=10):
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


def main():
    torch.backends.cudnn.benchmark = True
    N = 256
    # (H, Cin, Cout, count in resnet50)
    shapes = [(56, 64, 64, 1), (56, 256, 64, 2), (56, 64, 256, 4), (28, 128, 512, 4), (28, 512, 128, 3),
              (14, 256, 1024, 6), (14, 1024, 256, 5), (7, 512, 2048, 3), (7, 2048, 512, 2)]
    tot = {"miopen": 0.0, "gemm": 0.0}
    for H, ci, co, cnt in shapes:
        x = torch.randn(N, ci, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(co, ci, 1, 1, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, co, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        xr = x.requires_grad_(True)
        wr = w.requires_grad_(True)

        def conv_all():
            y = F.conv2d(xr, wr)
            gx, gw = torch.autograd.grad(y, (xr, wr), dy)
            return gx, gw

        m = t(conv_all)
        X = x.detach().permute(0, 2, 3, 1).reshape(-1, ci)
        W = w.detach().reshape(co, ci)
        DY = dy.permute(0, 2, 3, 1).reshape(-1, co)

        def gemm_all():
            y = torch.mm(X, W.t())
            gx = torch.mm(DY, W)
            gw = torch.mm(DY.t(), X)
            return y, gx, gw

        g = t(gemm_all)
        fl = 3 * 2 * N * H * H * ci * co
        tot["miopen"] += m * cnt
        tot["gemm"] += g * cnt
        print(json.dumps({"H": H, "cin": ci, "cout": co, "miopen_ms": round(m, 3), "gemm_ms": round(g, 3),
                          "miopen_tflops": round(fl / m / 1e9, 1), "gemm_tflops": round(fl / g / 1e9, 1)}), flush=True)
    print(json.dumps({"total_1x1_ms_per_step": {k: round(v, 3) for k, v in tot.items()}}))
    # 3x3 for reference
    for H, c, cnt in [(56, 64, 3), (28, 128, 4), (14, 256, 6), (7, 512, 3)]:
        x = torch.randn(N, c, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        w = torch.randn(c, c, 3, 3, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        dy = torch.randn(N, c, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)

        def c3():
            y = F.conv2d(x, w, padding=1)
            return torch.autograd.grad(y, (x, w), dy)

        m = t(c3)
        fl = 3 * 2 * N * H * H * c * c * 9
        print(json.dumps({"conv3x3_H": H, "c": c, "miopen_ms": round(m, 3), "tflops": round(fl / m / 1e9, 1), "count": cnt}), flush=True)


if __name__ == "__main__":
    main()
