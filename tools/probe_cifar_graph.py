"""One CIFAR ASHA trial (examples/cifar10_asha) trained locally for N batches, eager vs the
HIP-graph-captured step (optimizations.hip_graph): wall ms per batch after warm-up. Diagnoses the
graphed-trial stall seen in profiles/round5_asha_hip_graph_attempt.txt."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples", "cifar10_asha"))

import torch  # noqa: E402

from determined_clone_amd import pytorch  # noqa: E402


def run(graph: bool, batches: int, deterministic: bool = False) -> dict:
    import model_def
    from determined_clone_amd.pytorch import _graph

    runners = []
    orig = _graph.GraphedTrainStep.__init__

    def rec(self, *a, **k):
        orig(self, *a, **k)
        runners.append(self)

    _graph.GraphedTrainStep.__init__ = rec
    torch.backends.cudnn.deterministic = deterministic

    hp = {"global_batch_size": 128, "learning_rate": 0.01, "momentum": 0.9, "width": 64, "dropout": 0.2,
          "dropout2": 0.3, "hidden": 512, "train_records": 128 * batches, "val_records": 1280}
    exp_conf = {"optimizations": {"hip_graph": graph}, "records_per_epoch": 128 * batches}
    with pytorch.init(hparams=hp, exp_conf=exp_conf) as ctx:
        trial = model_def.CIFARTrial(ctx)
        trainer = pytorch.Trainer(trial, ctx)
        t0 = time.time()
        trainer.fit(max_length=pytorch.Batch(batches), reporting_period=pytorch.Batch(batches),
                    checkpoint_policy="none", validation_period=pytorch.Batch(10 ** 9))
        torch.cuda.synchronize()
        out = {"hip_graph": graph, "deterministic_solvers": deterministic, "batches": batches,
               "wall_s": round(time.time() - t0, 2)}
        if runners:
            out.update(calls=runners[0].calls, replays=runners[0].replays,
                       captured=runners[0].graph is not None)
        return out


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    mode = sys.argv[2] if len(sys.argv) > 2 else "0"
    print(json.dumps(run(mode == "1", n, deterministic=(mode == "det"))), flush=True)
