"""Where a fresh trial process spends its first training batch (ASHA trials are short, so this is
part of every trial's cost): times, each behind a device synchronize, of HIP context creation, model
build + move, the first forward, backward and optimizer step, and a second (warm) batch.

Usage: ``python tools/probe_trial_startup.py`` in a fresh process (one JSON line). Compare
environments (e.g. ``MIOPEN_CUSTOM_CACHE_DIR`` set / unset, ``DCA_GEMM_TUNED=0``) across processes.
"""
import json
import os
import sys
import time

t_start = time.time()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "examples", "cifar10_asha"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main() -> None:
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=32)
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--find", action="store_true",
                    help="MIOpen find (cudnn.benchmark): record the shapes' best solvers in the DB")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = a.find
    out = {"import_torch_s": round(time.time() - t_start, 3), "width": a.width, "find": a.find}

    def mark(name: str, t0: float) -> float:
        torch.cuda.synchronize()
        t = time.time()
        out[name] = round(t - t0, 3)
        return t

    t = time.time()
    torch.zeros(1, device="cuda")
    t = mark("hip_context_s", t)
    from determined_clone_amd.models import cifar
    from determined_clone_amd.ops import _ext

    _ext.load()
    t = mark("ext_load_s", t)
    hp = {"width": a.width, "hidden": a.hidden, "dropout": 0.25, "dropout2": 0.5}
    model = cifar.CifarCNN(hp).cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    x = torch.randn(128, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (128,), device="cuda")
    t = mark("model_build_s", t)
    # training and evaluation (validation runs the forward at the evaluation batch too)
    for i in range(2):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits = model(x)
        t = mark(f"fwd{i}_s", t)
        loss = F.cross_entropy(logits.float(), y)
        loss.backward()
        t = mark(f"bwd{i}_s", t)
        opt.step()
        opt.zero_grad()
        t = mark(f"opt{i}_s", t)
    model.eval()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        model(x)
    t = mark("eval_fwd_s", t)
    out["total_s"] = round(time.time() - t_start, 3)
    out["env"] = {k: os.environ.get(k) for k in ("MIOPEN_CUSTOM_CACHE_DIR", "MIOPEN_USER_DB_PATH",
                                                   "DCA_GEMM_TUNED")}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
