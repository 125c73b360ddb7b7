"""Run the stem weight-gradient kernel alone (bs 1024) a few times, for rocprofv3 --pmc passes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from determined_clone_amd.ops import _ext  # noqa: E402

C = _ext.load()
x = torch.randn(1024, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
xs = C.stem_s2d(x)
dy = torch.randn(1024, 64, 112, 112, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
for _ in range(3):
    C.stem_wgrad(dy, xs)
torch.cuda.synchronize()
print("ok")
