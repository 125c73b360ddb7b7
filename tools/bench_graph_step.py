"""Eager vs HIP-graph training step time (pytorch/_graph.py) for launch-bound transformer steps.

For each GPT config: build the trial through pytorch.init (fused AdamW + device-side clipping, a
per-batch LR schedule), then time N steps of ``trial.train_batch`` eagerly and through
``GraphedTrainStep`` (3 eager warm-up steps, capture, replays). Prints one JSON line per config.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from determined_clone_amd import pytorch  # noqa: E402
from determined_clone_amd.models import gpt2  # noqa: E402
from determined_clone_amd.pytorch import _graph  # noqa: E402


def run(preset: str, batch: int, seq: int, steps: int, graphed: bool) -> float:
    with pytorch.init(hparams={"global_batch_size": batch}, exp_conf={"optimizations": {}}) as ctx:
        torch.manual_seed(0)
        model = ctx.wrap_model(gpt2.cast_for_mi355x(gpt2.gpt2(preset, max_seq_len=seq)))
        opt = ctx.wrap_optimizer(torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01))

        def train_batch(batch, epoch_idx, batch_idx):
            _, loss = model(batch, batch)
            ctx.backward(loss)
            ctx.step_optimizer(opt, pytorch.clip_grad_norm(1.0))
            return {"loss": loss}

        fn = _graph.GraphedTrainStep(ctx, train_batch, 3) if graphed else train_batch
        data = [torch.randint(0, 512, (batch, seq), device=ctx.device) for _ in range(4)]
        t0 = None
        for i in range(steps + 5):
            ctx._current_batch_idx = i
            if i == 5:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            fn(batch=data[i % 4], epoch_idx=0, batch_idx=i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3


def main() -> None:
    for preset, batch, seq in (("tiny", 8, 128), ("tiny", 32, 256), ("gpt2-small", 8, 256)):
        eager = run(preset, batch, seq, 50, False)
        graph = run(preset, batch, seq, 50, True)
        print(json.dumps({"model": preset, "batch": batch, "seq": seq, "eager_ms": round(eager, 3),
                          "hip_graph_ms": round(graph, 3), "speedup": round(eager / graph, 3)}), flush=True)


if __name__ == "__main__":
    main()
