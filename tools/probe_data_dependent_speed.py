"""Does kernel speed depend on the data? Times the implicit-GEMM 3x3 forward (csrc/conv_igemm.hip) and
a hipBLASLt GEMM on random operands vs operands with most entries zero (as ReLU outputs of corrupted
activations would be), back-to-back on one GPU. On a power-limited part, MFMA work on low-toggle data
draws less power and runs at higher clocks. Usage: python tools/probe_data_dependent_speed.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from determined_clone_amd.ops import _ext  # noqa: E402


def _time(fn, reps=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    C = _ext.load()
    torch.manual_seed(0)
    x = torch.randn(1024, 128, 28, 28, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(128, 128, 3, 3, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    a = torch.randn(32768, 4096, device="cuda").to(torch.bfloat16)
    b = torch.randn(4096, 1024, device="cuda").to(torch.bfloat16)
    variants = {
        "random": lambda t: t,
        "relu_of_random (50% zeros)": lambda t: t.clamp_min(0),
        "90% zeros": lambda t: t * (torch.rand_like(t, dtype=torch.float32) < 0.1).to(t.dtype),
        "all zeros": lambda t: torch.zeros_like(t),
    }
    for rnd in range(2):
        for name, f in variants.items():
            xv, av = f(x), f(a)
            conv_us = _time(lambda: C.conv_igemm_fwd(xv, w, 1, 1, False))
            gemm_us = _time(lambda: torch.mm(av, b))
            print(json.dumps({"round": rnd, "data": name, "igemm_3x3_fwd_us": round(conv_us, 1),
                              "hipblaslt_gemm_us": round(gemm_us, 1)}), flush=True)


if __name__ == "__main__":
    main()
