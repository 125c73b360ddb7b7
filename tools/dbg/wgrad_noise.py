"""Per-parameter relative difference of the ResNet weight gradients: inline vs inline (noise floor),
inline vs side stream, side vs side -- with the fused optimizer's flat .grad views in place."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from determined_clone_amd.models import resnet  # noqa: E402
from determined_clone_amd.ops import _grad  # noqa: E402
from determined_clone_amd.ops import optim as fopt  # noqa: E402

torch.manual_seed(0)
dev = torch.device("cuda")
model = resnet.to_mi355x_layout(resnet.resnet18_bottleneck_tiny(num_classes=10)).to(dev)
opt = fopt.FusedSGD(model.parameters(), lr=0.1, momentum=0.9)
x = torch.randn(16, 3, 64, 64, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (16,), device=dev)
names = [n for n, _ in model.named_parameters()]
for rep in range(3):
    runs = []
    for side in (False, False, True, True):
        _grad.SIDE_STREAM = side
        opt.zero_grad()
        F.cross_entropy(model(x).float(), y).backward()
        if side:
            assert _grad.pending()
        _grad.join()
        torch.cuda.synchronize()
        runs.append([p.grad.float().clone() for p in model.parameters()])
    print(f"--- rep {rep}")
    for i, n in enumerate(names):
        a, a2, b, b2 = (r[i] for r in runs)
        nrm = a.norm().item() + 1e-12
        ii, is_, ss = ((u - v).norm().item() / nrm for u, v in ((a, a2), (a, b), (b, b2)))
        if max(ii, is_, ss) > 1e-4:
            print(f"{n:40s} norm={nrm:.4e} ii={ii:.4f} is={is_:.4f} ss={ss:.4f}")
