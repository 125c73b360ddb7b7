"""Phase-by-phase timing of the GPT-2 training step on one GPU (debug/profiling helper)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from determined_clone_amd.models import gpt2  # noqa: E402
from determined_clone_amd.pytorch import deepspeed as det_ds  # noqa: E402


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def timed(name, fn, n=1):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        out = fn()
    torch.cuda.synchronize()
    log(f"{name}: {(time.perf_counter() - t) / n * 1000:.2f} ms")
    return out


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "gpt2-medium"
    micro = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    stage = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    S = 1024
    log("building model", name)
    torch.manual_seed(0)
    model = gpt2.gpt2(name, max_seq_len=S)
    cfg = {"train_micro_batch_size_per_gpu": micro, "gradient_accumulation_steps": 1,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-4, "weight_decay": 0.1}},
           "gradient_clipping": 1.0, "bf16": {"enabled": True},
           "zero_optimization": {"stage": stage}}
    eng, _, _, _ = det_ds.initialize(model=model, config=cfg)
    log("engine ready; params", sum(p.numel() for p in model.parameters()))
    x = torch.randint(0, 50257, (micro, S), device="cuda")
    y = torch.randint(0, 50257, (micro, S), device="cuda")
    log("first forward")
    _, loss = timed("fwd (first)", lambda: eng(x, y))
    log("loss", float(loss))
    timed("bwd (first)", lambda: eng.backward(loss))
    timed("step (first)", lambda: eng.step())

    def full():
        _, l = eng(x, y)
        eng.backward(l)
        eng.step()
        return l

    timed("full step x5", full, 5)
    with torch.no_grad():
        timed("fwd only x5", lambda: eng(x, y), 5)
    log("done")


if __name__ == "__main__":
    main()
