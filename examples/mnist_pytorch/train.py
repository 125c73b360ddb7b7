"""MNIST PyTorchTrial (reference tutorial: examples/tutorials/mnist_pytorch/train.py) on
determined_clone_amd. Runs locally (``python train.py``) or on-cluster (``det experiment create
const.yaml .``) with the same code. Data: IDX files under ./data if present, else offline synthetic
MNIST-shaped data."""
import logging
import pathlib
from typing import Any, Dict

import torch
import yaml
from torch import nn

import determined_clone_amd as det
from determined_clone_amd import pytorch
from determined_clone_amd.models import mnist


class MNistTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext, hparams: Dict) -> None:
        self.context = context
        self.data_dir = pathlib.Path("data")
        self.batch_size = 64
        self.per_slot_batch_size = self.batch_size // self.context.distributed.get_size()
        self.loss_fn = nn.NLLLoss()
        self.model = self.context.wrap_model(mnist.build_model(hparams=hparams))
        self.optimizer = self.context.wrap_optimizer(
            torch.optim.Adadelta(self.model.parameters(), lr=hparams["learning_rate"]))

    def build_training_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(mnist.get_dataset(self.data_dir, train=True),
                                  batch_size=self.per_slot_batch_size, shuffle=True)

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(mnist.get_dataset(self.data_dir, train=False),
                                  batch_size=self.per_slot_batch_size)

    def train_batch(self, batch: pytorch.TorchData, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        data, labels = batch
        loss = self.loss_fn(self.model(data), labels)
        self.context.backward(loss)
        self.context.step_optimizer(self.optimizer)
        return {"loss": loss}

    def evaluate_batch(self, batch: pytorch.TorchData, batch_idx: int) -> Dict[str, Any]:
        data, labels = batch
        output = self.model(data)
        pred = output.argmax(dim=1, keepdim=True)
        return {"validation_loss": self.loss_fn(output, labels).item(),
                "accuracy": pred.eq(labels.view_as(pred)).sum().item() / len(data)}


def run(local: bool = False, max_batches: int = 100) -> None:
    info = det.get_cluster_info()
    if local:
        conf = yaml.safe_load((pathlib.Path(__file__).parent / "const.yaml").read_text())
        hparams = conf["hyperparameters"]
        max_length = pytorch.Batch(max_batches)
        latest_checkpoint = None
    else:
        hparams = info.trial.hparams
        max_length = None
        latest_checkpoint = info.latest_checkpoint
    with pytorch.init() as train_context:
        trial = MNistTrial(train_context, hparams=hparams)
        trainer = pytorch.Trainer(trial, train_context)
        trainer.fit(max_length=max_length, latest_checkpoint=latest_checkpoint,
                    validation_period=pytorch.Batch(max_batches) if local else None)


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format=det.LOG_FORMAT)
    run(local=det.get_cluster_info() is None)
