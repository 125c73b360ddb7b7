"""Split-K weight-gradient GEMM of the GPT-2 linears (4 K-slices as one batched GEMM): fp32 slice
outputs (shipped) vs bf16 slice outputs, isolated timing (HIP events, median of 20)."""
import json

import torch


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[iters // 2] * 1e3


T, s = 32768, 4
for m, n in ((4096, 1024), (1024, 4096), (3072, 1024), (1024, 1024)):
    dy = torch.randn(T, m, device="cuda").bfloat16()
    x = torch.randn(T, n, device="cuda").bfloat16()
    a = dy.reshape(s, T // s, m).transpose(1, 2)
    b = x.reshape(s, T // s, n)
    f32 = timeit(lambda: torch.bmm(a, b, out_dtype=torch.float32))
    b16 = timeit(lambda: torch.bmm(a, b))
    full = timeit(lambda: dy.t() @ x)
    fl = 2 * T * m * n
    print(json.dumps({"m": m, "n": n, "bmm_f32_us": round(f32, 1), "tf_f32": round(fl / f32 / 1e6, 1),
                      "bmm_bf16_us": round(b16, 1), "tf_bf16": round(fl / b16 / 1e6, 1),
                      "mm_nosplit_us": round(full, 1), "tf_nosplit": round(fl / full / 1e6, 1)}), flush=True)
