"""Per-parameter eager vs HIP-graph training comparison (diagnostic for tests/test_graph_gpu.py).
``--no-miopen`` runs the ResNet convolutions through PyTorch's native kernels instead of MIOpen."""
import os
import pathlib
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tests import test_graph_gpu as t  # noqa: E402

if "--no-miopen" in sys.argv:
    torch.backends.cudnn.enabled = False
classes = (t._ResNetTrial,) if "--resnet" in sys.argv else (t._GPTTrial, t._ResNetTrial)
for cls in classes:
    with tempfile.TemporaryDirectory() as d:
        e, _, _, _ = t._run(cls, False, pathlib.Path(d))
        g, runner, _, _ = t._run(cls, True, pathlib.Path(d))
    print(cls.__name__, "miopen" if torch.backends.cudnn.enabled else "native-conv",
          "replays", runner.replays if runner else None, flush=True)
    for n, x in e.items():
        err = (g[n] - x).norm().item() / max(x.norm().item(), 1e-12)
        print(f"  {n:40s} {err:.2e}", flush=True)
