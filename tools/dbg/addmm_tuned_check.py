"""beta = 1 backward-data GEMMs (ops/conv.py shortcut accumulation) under the shipped TunableOp
replay at the bs-1024 ResNet-50 conv1 shapes: rows.addmm_(dy, W) vs fp32 dy @ W + C."""
import os
import sys

os.environ.setdefault("DCA_GEMM_TUNED", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from determined_clone_amd.ops import _ext  # noqa: E402

_ext.load()  # enables the tuned replay
print("tunable enabled:", torch.cuda.tunable.is_enabled())
for n_hw, cin, cout in ((1024 * 56 * 56, 256, 64), (1024 * 28 * 28, 512, 128),
                        (1024 * 14 * 14, 1024, 256), (1024 * 7 * 7, 2048, 512)):
    g = torch.Generator(device="cuda").manual_seed(0)
    dy = torch.randn(n_hw, cout, device="cuda", generator=g).bfloat16()
    W = (torch.randn(cout, cin, device="cuda", generator=g) / cout ** 0.5).bfloat16()
    c = torch.randn(n_hw, cin, device="cuda", generator=g).bfloat16()
    ref = dy.float() @ W.float() + c.float()
    acc = c.clone()
    acc.addmm_(dy, W)
    err = (acc.float() - ref).norm().item() / ref.norm().item()
    plain = (torch.mm(dy, W).float() + c.float())
    err2 = (plain - ref).norm().item() / ref.norm().item()
    print(f"rows={n_hw} cin={cin} cout={cout} rel_err addmm_={err:.2e} mm+add={err2:.2e}")
    assert err < 1e-2, err
