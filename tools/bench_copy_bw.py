"""Practical HBM roofline on this MI355X: device-to-device copy / fill bandwidth for large buffers
(the yardstick for the streaming BatchNorm kernels, profiles/s2_bn_rowtile_bandwidth.txt)."""
import json

import torch


def bw(fn, nbytes: int, iters: int = 20) -> float:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return nbytes * iters / (s.elapsed_time(e) / 1e3) / 1e12


def main() -> None:
    out = {}
    for mb in (256, 1024, 2048):
        n = mb * 2 ** 20 // 2
        x = torch.randn(n, device="cuda").to(torch.bfloat16)
        y = torch.empty_like(x)
        out[f"copy_{mb}MB_TBps"] = round(bw(lambda: y.copy_(x), 2 * x.numel() * 2), 3)
        out[f"fill_{mb}MB_TBps"] = round(bw(lambda: y.fill_(1.0), x.numel() * 2), 3)
        out[f"add_{mb}MB_TBps"] = round(bw(lambda: torch.add(x, x, out=y), 3 * x.numel() * 2), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
