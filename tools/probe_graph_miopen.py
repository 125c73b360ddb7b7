"""Find the first op whose HIP-graph replay differs from the eager run.

One forward + backward of the tiny bottleneck ResNet (MIOpen / hipBLASLt / our igemm convs, fused
BN) with FIXED parameters and input, run eagerly (twice: the noise floor of nondeterministic
kernels) and then captured into a HIP graph and replayed. Forward hooks copy every conv / BN
output into per-module buffers (the copies are captured too), and every parameter gradient is
copied after backward. Prints, in execution order, the relative difference eager-vs-eager and
eager-vs-replay of each activation and gradient. Usage: python tools/probe_graph_miopen.py
[--no-miopen] [--graph-safe]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from determined_clone_amd.models import resnet  # noqa: E402
from determined_clone_amd.ops import _ext  # noqa: E402


def main() -> None:
    _ext.load()
    if "--no-miopen" in sys.argv:
        torch.backends.cudnn.enabled = False
    torch.manual_seed(0)
    dev = torch.device("cuda")
    model = resnet.to_mi355x_layout(resnet.resnet18_bottleneck_tiny(10)).to(dev)
    x = torch.randn(8, 3, 32, 32, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=dev)
    order, bufs = [], {}

    def hook(name):
        def f(mod, inp, out):
            o = out[0] if isinstance(out, (tuple, list)) else out
            if name not in bufs:
                bufs[name] = torch.empty_like(o)
                order.append(name)
            bufs[name].copy_(o)
        return f

    for name, m in model.named_modules():
        if name and not list(m.children()):
            m.register_forward_hook(hook("act " + name))
    gbufs = {}

    def step():
        for p in model.parameters():
            p.grad = None
        loss = F.cross_entropy(model(x).float(), y)
        loss.backward()
        for n, p in model.named_parameters():
            if p.grad is None:
                continue
            if n not in gbufs:
                gbufs[n] = torch.empty_like(p.grad)
            gbufs[n].copy_(p.grad)
        return loss

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    snap = lambda: ({k: v.float().clone() for k, v in bufs.items()}, {k: v.float().clone() for k, v in gbufs.items()})  # noqa: E731
    ref_a, ref_g = snap()
    print("=== PHASE eager", file=sys.stderr, flush=True)
    step()
    torch.cuda.synchronize()
    e2_a, e2_g = snap()
    print("=== PHASE capture", file=sys.stderr, flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    print("=== PHASE end", file=sys.stderr, flush=True)
    # zero the buffers so a node that is missing from the graph shows up as a difference of 1
    for v in list(bufs.values()) + list(gbufs.values()):
        v.zero_()
    g.replay()
    torch.cuda.synchronize()
    gr_a, gr_g = snap()

    def rel(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()

    print(f"{'tensor':48s} {'eager-vs-eager':>15s} {'eager-vs-replay':>16s}")
    first = None
    for k in order:
        r1, r2 = rel(e2_a[k], ref_a[k]), rel(gr_a[k], ref_a[k])
        flag = " <==" if r2 > max(10 * r1, 1e-6) else ""
        if flag and first is None:
            first = k
        print(f"{k:48s} {r1:15.2e} {r2:16.2e}{flag}")
    for k in reversed(list(ref_g)):
        r1, r2 = rel(e2_g[k], ref_g[k]), rel(gr_g[k], ref_g[k])
        flag = " <==" if r2 > max(10 * r1, 1e-6) else ""
        if flag and first is None:
            first = "grad " + k
        print(f"grad {k:43s} {r1:15.2e} {r2:16.2e}{flag}")
    print("first divergent:", first, flush=True)


if __name__ == "__main__":
    main()
