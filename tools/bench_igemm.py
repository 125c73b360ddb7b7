"""Implicit-GEMM k x k convolutions (ops/csrc/conv_igemm.hip) vs MIOpen on ResNet-50's 3x3 shapes:
numerics against fp32 MIOpen on a small batch, then forward / stride-1 data-gradient timing at the
bench batch, interleaved in one process (guide rule 24). Usage:
``python tools/bench_igemm.py [--batch 1024] [--check-only]``."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from determined_clone_amd.ops import miopen_db  # noqa: E402

miopen_db.use_private_copy("tools")

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from determined_clone_amd.ops import _ext  # noqa: E402

# (H_in, Cin, Cout, stride, count per ResNet-50 step)
SHAPES = [(56, 64, 64, 1, 3), (56, 128, 128, 2, 1), (28, 128, 128, 1, 3), (28, 256, 256, 2, 1),
          (14, 256, 256, 1, 5), (14, 512, 512, 2, 1), (7, 512, 512, 1, 2)]


# 1x1 convolutions (H_in, Cin, Cout, stride, count): weight gradients only (their forward / data
# gradient run as library GEMMs, ops/conv.py)
SHAPES1 = [(56, 64, 64, 1, 1), (56, 256, 64, 1, 2), (56, 64, 256, 1, 4), (56, 256, 128, 1, 1),
           (56, 256, 512, 2, 1), (28, 512, 128, 1, 3), (28, 128, 512, 1, 4), (28, 512, 256, 1, 1),
           (28, 512, 1024, 2, 1), (14, 1024, 256, 1, 5), (14, 256, 1024, 1, 6), (14, 1024, 512, 1, 1),
           (14, 1024, 2048, 2, 1), (7, 2048, 512, 1, 2), (7, 512, 2048, 1, 3)]


def timed(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3  # us


def rel_err(got, ref):
    return ((got.float() - ref).abs().max() / (ref.abs().max() + 1e-6)).item()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--check-only", action="store_true")
    a = ap.parse_args()
    C = _ext.load()
    torch.manual_seed(0)
    tot = {"mi_fwd": 0.0, "ig_fwd": 0.0, "mi_dgrad": 0.0, "ig_dgrad": 0.0, "mi_wgrad": 0.0, "ig_wgrad": 0.0}
    for H, ci, co, st, cnt in SHAPES:
        # numerics on a small batch against fp32
        x = torch.randn(3, ci, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, 3, 3, device="cuda") / (9 * ci) ** 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
        ref = F.conv2d(x.float(), w.float(), stride=st, padding=1)
        y, part = C.conv_igemm_fwd(x, w, st, 1, True)
        yc = y.float().permute(0, 2, 3, 1).reshape(-1, co)
        stat_err = rel_err(part.sum(0)[0], yc.sum(0))
        res = {"H": H, "cin": ci, "cout": co, "stride": st, "fwd_rel_err": round(rel_err(y, ref), 5),
               "stats_rel_err": round(stat_err, 5)}
        dy = torch.randn_like(ref).bfloat16().contiguous(memory_format=torch.channels_last)
        wref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [st, st], [1, 1],
                                                   [1, 1], False, [0, 0], 1, [False, True, False])[1]
        res["wgrad_rel_err"] = round(rel_err(C.conv_igemm_wgrad(dy, x, w, st, 1), wref), 5)
        if st == 1:
            dref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [1, 1], [1, 1],
                                                       [1, 1], False, [0, 0], 1, [True, False, False])[0]
            res["dgrad_rel_err"] = round(rel_err(C.conv_igemm_dgrad(dy, w, 1), dref), 5)
        if not a.check_only:
            n = a.batch
            x = torch.randn(n, ci, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            y = F.conv2d(x, w, stride=st, padding=1)
            dy = torch.randn_like(y)
            Ho = y.shape[2]
            flops = 2.0 * n * Ho * Ho * co * ci * 9
            for rnd in range(2):  # interleaved rounds, report the last
                mi = timed(lambda: F.conv2d(x, w, stride=st, padding=1))
                ig = timed(lambda: C.conv_igemm_fwd(x, w, st, 1, True))
                res.update({"mi_fwd_us": round(mi, 1), "ig_fwd_us": round(ig, 1),
                            "mi_fwd_tf": round(flops / mi / 1e6, 1), "ig_fwd_tf": round(flops / ig / 1e6, 1)})
                miw = timed(lambda: torch.ops.aten.convolution_backward(
                    dy, x, w, None, [st, st], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
                igw = timed(lambda: C.conv_igemm_wgrad(dy, x, w, st, 1))
                res.update({"mi_wgrad_us": round(miw, 1), "ig_wgrad_us": round(igw, 1),
                            "mi_wgrad_tf": round(flops / miw / 1e6, 1), "ig_wgrad_tf": round(flops / igw / 1e6, 1)})
                if st == 1:
                    mid = timed(lambda: torch.ops.aten.convolution_backward(
                        dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]))
                    igd = timed(lambda: C.conv_igemm_dgrad(dy, w, 1))
                    res.update({"mi_dgrad_us": round(mid, 1), "ig_dgrad_us": round(igd, 1),
                                "ig_dgrad_tf": round(flops / igd / 1e6, 1)})
            tot["mi_wgrad"] += res["mi_wgrad_us"] * cnt
            tot["ig_wgrad"] += res["ig_wgrad_us"] * cnt
            tot["mi_fwd"] += res["mi_fwd_us"] * cnt
            tot["ig_fwd"] += res["ig_fwd_us"] * cnt
            if st == 1:
                tot["mi_dgrad"] += res["mi_dgrad_us"] * cnt
                tot["ig_dgrad"] += res["ig_dgrad_us"] * cnt
            del x, y, dy
            torch.cuda.empty_cache()
        print(json.dumps(res), flush=True)
    tw = {"mi_wgrad1": 0.0, "ig_wgrad1": 0.0, "lib_fwd1": 0.0, "ig_fwd1": 0.0}
    for H, ci, co, st, cnt in SHAPES1:
        x = torch.randn(3, ci, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, 1, 1, device="cuda") / ci ** 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
        y = F.conv2d(x.float(), w.float(), stride=st)
        dy = torch.randn_like(y).bfloat16().contiguous(memory_format=torch.channels_last)
        wref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [st, st], [0, 0],
                                                   [1, 1], False, [0, 0], 1, [False, True, False])[1]
        res = {"k": 1, "H": H, "cin": ci, "cout": co, "stride": st,
               "wgrad_rel_err": round(rel_err(C.conv_igemm_wgrad(dy, x, w, st, 0), wref), 5),
               "fwd_rel_err": round(rel_err(C.conv_igemm_fwd(x, w, st, 0, True)[0], y), 5)}
        if not a.check_only:
            n = a.batch
            x = torch.randn(n, ci, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            y = F.conv2d(x, w, stride=st)
            dy = torch.randn_like(y)
            flops = 2.0 * n * y.shape[2] * y.shape[3] * co * ci
            W2 = w.view(co, ci)

            def gemm_fwd():
                v = x.permute(0, 2, 3, 1)
                if st > 1:
                    v = v[:, ::st, ::st, :]
                return torch.mm(v.reshape(-1, ci), W2.t())

            for rnd in range(2):
                miw = timed(lambda: torch.ops.aten.convolution_backward(
                    dy, x, w, None, [st, st], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]))
                igw = timed(lambda: C.conv_igemm_wgrad(dy, x, w, st, 0))
                mif = timed(lambda: F.conv2d(x, w, stride=st))
                gmf = timed(gemm_fwd)
                igf = timed(lambda: C.conv_igemm_fwd(x, w, st, 0, True))
            io = (x.numel() // (st * st) + y.numel()) * 2
            res.update({"mi_wgrad_us": round(miw, 1), "ig_wgrad_us": round(igw, 1),
                        "ig_wgrad_tf": round(flops / igw / 1e6, 1), "mi_fwd_us": round(mif, 1),
                        "gemm_fwd_us": round(gmf, 1), "ig_fwd_us": round(igf, 1),
                        "ig_fwd_TBps": round(io / igf / 1e6, 2)})
            tw["lib_fwd1"] += min(mif, gmf) * cnt
            tw["ig_fwd1"] += igf * cnt
            tw["mi_wgrad1"] += miw * cnt
            tw["ig_wgrad1"] += igw * cnt
            del x, y, dy
            torch.cuda.empty_cache()
        print(json.dumps(res), flush=True)
    if not a.check_only:
        tot.update(tw)
        print(json.dumps({"per_step_ms": {k: round(v / 1e3, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
