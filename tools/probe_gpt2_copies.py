"""Which call sites issue the large device-to-device copies of the GPT-2 training step.

Runs a few DeepSpeed-engine steps of GPT-2 (default gpt2-medium, micro 32, seq 1024, ZeRO-2) under
``torch.profiler`` with CPU + GPU activities and Python stacks, and prints, per distinct
(op, shapes, stack), how many times per step an ATen op ran whose GPU side was a memcpy
(``__amd_rocclr_copyBuffer`` in rocprof; "Memcpy DtoD" in the profiler). GPU only.

Usage: python tools/probe_gpt2_copies.py [--model gpt2-medium --micro 32 --steps 2]
"""
import argparse
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--micro", type=int, default=32)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--stage", type=int, default=2)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()

    import torch
    from torch.profiler import ProfilerActivity, profile

    from determined_clone_amd.models import gpt2
    from determined_clone_amd.pytorch import deepspeed as det_ds

    os.environ.setdefault("DCA_GEMM_TUNED", "1")
    torch.manual_seed(0)
    model = gpt2.gpt2(a.model, max_seq_len=a.seq)
    cfg = {"train_micro_batch_size_per_gpu": a.micro, "gradient_accumulation_steps": 1,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-4, "weight_decay": 0.1}},
           "gradient_clipping": 1.0, "bf16": {"enabled": True},
           "zero_optimization": {"stage": a.stage, "overlap_comm": True}}
    eng, _, _, _ = det_ds.initialize(model=model, config=cfg)
    V = model.cfg.vocab_size
    x = torch.randint(0, V, (a.micro, a.seq), device="cuda")
    y = torch.randint(0, V, (a.micro, a.seq), device="cuda")

    def step():
        _, loss = eng(x, y)
        eng.backward(loss)
        eng.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()

    events = list(prof.events())
    # GPU memcpy events and the CPU op that launched them (correlation through the linked event)
    memcpy_total = Counter()
    by_site = Counter()
    bytes_site = Counter()
    for ev in events:
        if ev.device_type.name != "CUDA" and "Memcpy" not in ev.name and "copyBuffer" not in ev.name:
            continue
        nm = ev.name
        if "Memcpy" not in nm and "copyBuffer" not in nm and "memcpy" not in nm.lower():
            continue
        memcpy_total[nm] += 1
        par = getattr(ev, "linked_correlation_id", None)
        cpu = None
        # walk up from the runtime launch to the enclosing ATen op
        p = ev.cpu_parent
        chain = []
        while p is not None and len(chain) < 6:
            chain.append(p.name)
            if cpu is None and p.name.startswith("aten::"):
                cpu = p
            p = p.cpu_parent
        st = []
        src = cpu or ev
        for s in (getattr(src, "stack", None) or []):
            if "determined_clone_amd" in s or "torch/autograd" in s or "tools/" in s:
                st.append(s)
            if len(st) >= 6:
                break
        shapes = str(getattr(cpu, "input_shapes", "")) if cpu is not None else ""
        key = (nm, " <- ".join(chain[:4]), shapes[:160], " | ".join(st))
        by_site[key] += 1
        del par
    print("memcpy-like GPU events per step:")
    for nm, n in memcpy_total.most_common():
        print(f"  {n / a.steps:7.1f}  {nm}")
    print("\nby call site (per step):")
    for (nm, chain, shapes, st), n in by_site.most_common(40):
        print(f"{n / a.steps:6.1f}  {nm}\n        ops: {chain}\n        shapes: {shapes}\n        stack: {st}")
    # ATen copies/clones on CUDA tensors regardless of how the GPU ran them
    cnt = Counter()
    for ev in events:
        if ev.name in ("aten::copy_", "aten::clone", "aten::contiguous", "aten::cat", "aten::_to_copy"):
            shp = str(ev.input_shapes)[:120]
            st = [s for s in (ev.stack or []) if "determined_clone_amd" in s or "torch/autograd" in s][:4]
            par = ev.cpu_parent.name if ev.cpu_parent is not None else ""
            cnt[(ev.name, par, shp, " | ".join(st))] += 1
    print("\nATen copy-family ops per step (top 40):")
    for (nm, par, shp, st), n in cnt.most_common(40):
        print(f"{n / a.steps:6.1f}  {nm} <- {par}  {shp}\n        {st}")


if __name__ == "__main__":
    main()
