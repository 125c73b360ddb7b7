"""Batch inference of a trained MNIST PyTorchTrial with ``torch_batch_process`` (reference:
examples/features/inference_mnist_pytorch/inference.py).

The model comes from, in order of preference, the hyperparameters ``model_name`` +
``model_version`` (model registry), ``checkpoint_uuid`` (any checkpoint known to the master), or
the ``MNIST_CHECKPOINT_PATH`` environment variable (a local checkpoint directory). The trained
trial is rebuilt with ``pytorch.load_trial_from_checkpoint_path``; the job records which
model version / checkpoint it used, shards the test set over its ranks and reports accuracy and
the fraction of predicted nines, reduced across ranks.
"""
import json
import os
import sys
from typing import Any, Dict, List

import torch

from determined_clone_amd import pytorch
from determined_clone_amd.models import mnist
from determined_clone_amd.pytorch import experimental

HERE = os.path.dirname(os.path.abspath(__file__))


class _Counts(pytorch.MetricReducer):
    """Sums (correct, nines, total) per slot, then across slots."""

    def __init__(self) -> None:
        self.reset()

    def reset(self) -> None:
        self.c = [0, 0, 0]

    def update(self, correct: int, nines: int, total: int) -> None:
        self.c = [self.c[0] + correct, self.c[1] + nines, self.c[2] + total]

    def per_slot_reduce(self) -> List[int]:
        return self.c

    def cross_slot_reduce(self, per_slot: List[List[int]]) -> Dict[str, float]:
        correct, nines, total = (sum(v[i] for v in per_slot) for i in range(3))
        return {"accuracy": correct / max(total, 1), "nine_ratio": nines / max(total, 1),
                "total": float(total)}


def _mnist_trial_class() -> Any:
    sys.path.insert(0, os.path.join(HERE, "..", "..", "mnist_pytorch"))
    import train  # examples/mnist_pytorch/train.py

    return train.MNistTrial


def _checkpoint_path(context: experimental.TorchBatchProcessorContext) -> str:
    hp = context.get_hparams()
    if hp.get("model_name") or hp.get("checkpoint_uuid"):
        from determined_clone_amd.experimental import client

        d = client.Determined()
        if hp.get("model_name"):
            version = d.get_model(hp["model_name"]).get_version(int(hp.get("model_version", -1)))
            context.report_task_using_model_version(version)
            return version.checkpoint.download()
        ckpt = d.get_checkpoint(hp["checkpoint_uuid"])
        context.report_task_using_checkpoint(ckpt)
        return ckpt.download()
    return os.environ["MNIST_CHECKPOINT_PATH"]


class MNISTInferenceProcessor(experimental.TorchBatchProcessor):
    def __init__(self, context: experimental.TorchBatchProcessorContext) -> None:
        self.context = context
        path = _checkpoint_path(context)
        trial_cls = _mnist_trial_class()
        hparams = json.loads(open(os.path.join(path, "load_data.json")).read()).get("hparams", {})
        trained = pytorch.load_trial_from_checkpoint_path(
            path, trial_class=trial_cls, trial_kwargs={"hparams": hparams},
            torch_load_kwargs={"map_location": "cpu"})
        self.model = context.prepare_model_for_inference(trained.model)
        self.counts = context.wrap_reducer(_Counts(), name=None)

    def process_batch(self, batch: Any, batch_idx: int) -> None:
        x, labels = batch
        x, labels = self.context.to_device(x), self.context.to_device(labels)
        with torch.no_grad():
            pred = self.model(x).argmax(1)
        self.counts.update(int((pred == labels).sum()), int((pred == 9).sum()), len(labels))


def main(n: int = 1000, batch_size: int = 100) -> None:
    experimental.torch_batch_process(MNISTInferenceProcessor,
                                     mnist.get_dataset(None, train=False, synthetic_size=n),
                                     batch_size=batch_size, checkpoint_interval=5)


if __name__ == "__main__":
    main()
