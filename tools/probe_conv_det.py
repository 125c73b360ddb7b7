"""Which kernel runs F.conv2d for a small strided 1x1 bf16 NHWC convolution, and is it
deterministic (with and without torch.backends.cudnn.deterministic)."""
import sys

import torch
import torch.nn.functional as F

torch.manual_seed(0)
det = "--det" in sys.argv
torch.backends.cudnn.deterministic = det
x = torch.randn(8, 512, 4, 4, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
w = (torch.randn(1024, 512, 1, 1, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
outs = [F.conv2d(x, w, stride=2).float() for _ in range(20)]
torch.cuda.synchronize()
diff = max(((o - outs[0]).norm() / outs[0].norm()).item() for o in outs)
print(f"deterministic={det} max rel diff over 20 runs: {diff:.2e}", flush=True)
