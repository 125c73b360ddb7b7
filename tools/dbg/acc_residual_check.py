"""conv1 dgrad accumulated into the shortcut gradient: per-parameter relative gradient differences
between the separate path (sep), the accumulate path (acc) and an emulation of acc built from the
separate path (emu: dx + d(shortcut) rounded to bf16 by a plain add) -- acc vs emu isolates the
implementation from the extra bf16 rounding of the summed gradient."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from determined_clone_amd.models import resnet  # noqa: E402
from determined_clone_amd.ops import conv as conv_ops  # noqa: E402

torch.manual_seed(0)
torch.backends.cudnn.deterministic = True  # MIOpen: no atomics-based solvers (run-to-run identical)
dev = torch.device("cuda")
base = resnet.to_mi355x_layout(resnet.ResNet([2, 2, 1, 1], num_classes=10, zero_init_residual=False)).to(dev)
x = torch.randn(16, 3, 64, 64, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (16,), device=dev)
conv_ops._choose = lambda key, cands: 1 if key[0] == "dgrad" else 0
orig_bwd = conv_ops._PointwiseLib.backward


def emu_bwd(ctx, dy):
    dx, dw, _ = orig_bwd(ctx, dy)
    sink = getattr(ctx, "sink_emu", None)
    if sink is not None and sink.grad is not None and dx is not None:
        dx = (dx.float() + sink.grad.float()).bfloat16()
        sink.grad = None
    return dx, dw, None


def run(mode):
    conv_ops.ACC_RESIDUAL = mode == "acc"
    if mode == "emu":
        orig_fwd = conv_ops._PointwiseLib.forward

        def fwd(ctx, xx, w, st):
            out = orig_fwd(ctx, xx, w, st)
            ctx.sink_emu = getattr(xx, "_dca_grad_sink", None)
            return out
        conv_ops._PointwiseLib.forward = staticmethod(fwd)
        conv_ops._PointwiseLib.backward = staticmethod(emu_bwd)
    m = copy.deepcopy(base)
    F.cross_entropy(m(x).float(), y).backward()
    torch.cuda.synchronize()
    if mode == "emu":
        conv_ops._PointwiseLib.forward = staticmethod(orig_fwd)
        conv_ops._PointwiseLib.backward = staticmethod(orig_bwd)
    return [p.grad.float().clone() for p in m.parameters()]


g = {mode: run(mode) for mode in ("sep", "acc", "emu", "sep2")}
for i, (n, _) in enumerate(base.named_parameters()):
    a = g["sep"][i]
    nrm = a.norm().item() + 1e-12
    d = lambda u, v: (g[u][i] - g[v][i]).norm().item() / nrm  # noqa: E731
    print(f"{n:32s} norm={nrm:.3e} sep-acc={d('sep','acc'):.4f} acc-emu={d('acc','emu'):.4f} "
          f"sep-emu={d('sep','emu'):.4f} sep-sep2={d('sep','sep2'):.4f}")
print("hits", conv_ops.ACC_HITS)
