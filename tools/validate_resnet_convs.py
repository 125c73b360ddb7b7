"""Numerics of every ResNet-50 convolution at the bench shape (bs 1024, bf16, channels_last) on the
production dispatch (ops/conv.py: shipped chooser decisions, TunableOp results, implicit-GEMM
kernels, MIOpen find DB), forward, data gradient and weight gradient, against fp32 references
computed in 64-image chunks (torch.nn.grad on fp32 copies of the same bf16 inputs).

The shipped tuning artefacts pick kernels by speed alone; this checks, at the exact shapes the
bench runs, that what they picked computes the right numbers (profiles/round6_tuned_gemm_validation.txt).
Prints one JSON line per distinct convolution and a summary.
Usage: python tools/validate_resnet_convs.py [--batch 1024]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DCA_GEMM_TUNED", "1")

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from determined_clone_amd.models import resnet  # noqa: E402
from determined_clone_amd.ops import conv as conv_ops  # noqa: E402

BATCH = 1024
CHUNK = 64
TOL = 0.03  # max |err| / max |ref|; bf16 rounding gives < 0.01


def record_calls(model):
    """(kind, conv(s), input shape, bn_stats) of every convolution call in one small forward."""
    calls = []
    orig = (resnet.pointwise_conv, resnet.pointwise_dual, conv_ops.spatial_conv, conv_ops.stem_conv)

    def pw(conv, x, bn_stats=False):
        calls.append(("pointwise", (conv,), tuple(x.shape), bool(bn_stats)))
        return orig[0](conv, x, bn_stats)

    def dual(c1, c2, x, bn_stats=False):
        calls.append(("dual", (c1, c2), tuple(x.shape), bool(bn_stats)))
        return orig[1](c1, c2, x, bn_stats)

    def sp(conv, x, bn_stats=False):
        calls.append(("spatial", (conv,), tuple(x.shape), bool(bn_stats)))
        return orig[2](conv, x, bn_stats)

    def stem(conv, x, bn_stats=False):
        calls.append(("stem", (conv,), tuple(x.shape), bool(bn_stats)))
        return orig[3](conv, x, bn_stats)

    resnet.pointwise_conv, resnet.pointwise_dual = pw, dual
    conv_ops.spatial_conv, conv_ops.stem_conv = sp, stem
    try:
        x = torch.randn(2, 3, 224, 224, device="cuda").to(torch.bfloat16)
        model(x.contiguous(memory_format=torch.channels_last))
    finally:
        resnet.pointwise_conv, resnet.pointwise_dual = orig[0], orig[1]
        conv_ops.spatial_conv, conv_ops.stem_conv = orig[2], orig[3]
    return calls


def ref_conv(x, w, conv, dy):
    """fp32 forward / data gradient / weight gradient in CHUNK-image slices."""
    wf = w.float()
    ys, dxs, dw = [], [], torch.zeros_like(wf)
    for lo in range(0, x.shape[0], CHUNK):
        xf = x[lo:lo + CHUNK].float()
        ys.append(F.conv2d(xf, wf, stride=conv.stride, padding=conv.padding))
        if dy is not None:
            dyf = dy[lo:lo + CHUNK].float()
            dxs.append(torch.nn.grad.conv2d_input(xf.shape, wf, dyf, conv.stride, conv.padding))
            dw += torch.nn.grad.conv2d_weight(xf, wf.shape, dyf, conv.stride, conv.padding)
    return torch.cat(ys), (torch.cat(dxs) if dxs else None), dw


def rel_err(got, ref):
    return ((got.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()


def check(kind, convs, shape, bn_stats, g):
    shape = (BATCH,) + shape[1:]
    needs_dx = kind != "stem"  # the bench's stem input is an image without gradient
    x = torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(needs_dx)
    for c in convs:
        c.weight.grad = None
    if kind == "dual":
        outs = conv_ops.pointwise_dual(convs[0], convs[1], x, bn_stats)
    elif kind == "pointwise":
        outs = (conv_ops.pointwise_conv(convs[0], x, bn_stats),)
    elif kind == "spatial":
        outs = (conv_ops.spatial_conv(convs[0], x, bn_stats),)
    else:
        outs = (conv_ops.stem_conv(convs[0], x, bn_stats),)
    dys = [torch.randn(o.shape, device="cuda", generator=g).to(torch.bfloat16)
           .contiguous(memory_format=torch.channels_last) for o in outs]
    torch.autograd.backward(list(outs), dys)
    res = {"kind": kind, "x": list(shape), "convs": [[c.out_channels, c.in_channels, c.kernel_size[0],
                                                     c.stride[0]] for c in convs], "bn_stats": bn_stats}
    dx_ref = None
    errs = {}
    for i, (c, y, dy) in enumerate(zip(convs, outs, dys)):
        y_ref, dx_i, dw_ref = ref_conv(x.detach(), c.weight.detach(), c, dy)
        errs[f"fwd{i}"] = rel_err(y, y_ref)
        errs[f"wgrad{i}"] = rel_err(c.weight.grad, dw_ref)
        if needs_dx:
            dx_ref = dx_i if dx_ref is None else dx_ref + dx_i
    if needs_dx:
        errs["dgrad"] = rel_err(x.grad, dx_ref)
    res.update({k: round(v, 5) for k, v in errs.items()})
    res["ok"] = all(v <= TOL for v in errs.values())
    return res


def main():
    global BATCH
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=BATCH)
    BATCH = ap.parse_args().batch
    torch.manual_seed(0)
    model = resnet.to_mi355x_layout(resnet.resnet50()).cuda().train()
    calls = record_calls(model)
    seen, todo = set(), []
    for kind, convs, shape, bn_stats in calls:
        key = (kind, tuple((c.out_channels, c.in_channels, c.kernel_size, c.stride) for c in convs),
               shape, bn_stats)
        if key not in seen:
            seen.add(key)
            todo.append((kind, convs, shape, bn_stats))
    g = torch.Generator(device="cuda").manual_seed(0)
    bad = []
    for kind, convs, shape, bn_stats in todo:
        r = check(kind, convs, shape, bn_stats, g)
        print(json.dumps(r), flush=True)
        if not r["ok"]:
            bad.append(r)
        torch.cuda.empty_cache()
    print(json.dumps({"summary": {"checked": len(todo), "bad": len(bad)}}), flush=True)


if __name__ == "__main__":
    main()
