"""CIFAR-10 CNN PyTorchTrial for the adaptive_asha search config (BASELINE: "CIFAR-10 adaptive_asha
HP search, 16 concurrent trials gang-scheduled across 8 MI355X"). bf16 NHWC on the GPU with the
fused BN+ReLU HIP kernel; offline synthetic CIFAR-shaped data."""
import torch
import torch.nn.functional as F

from determined_clone_amd import pytorch
from determined_clone_amd.models import cifar


class CIFARTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        model = cifar.CifarCNN(hp)
        if context.device.type == "cuda":
            model = model.to(memory_format=torch.channels_last)
        self.model = context.wrap_model(model)
        self.opt = context.wrap_optimizer(torch.optim.SGD(
            self.model.parameters(), lr=hp["learning_rate"], momentum=hp.get("momentum", 0.9),
            weight_decay=hp.get("weight_decay", 5e-4)))

    def _prep(self, x):
        # fp16 records (the dataset's stored precision) -> fp32, NHWC on the GPU: one kernel
        if self.context.device.type == "cuda":
            return x.to(dtype=torch.float32, memory_format=torch.channels_last)
        return x.float()

    def train_batch(self, batch, epoch_idx, batch_idx):
        x, y = batch
        with torch.autocast(self.context.device.type, dtype=torch.bfloat16,
                            enabled=self.context.device.type == "cuda"):
            logits = self.model(self._prep(x))
        loss = F.cross_entropy(logits.float(), y)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss}

    def evaluate_batch(self, batch, batch_idx):
        x, y = batch
        with torch.autocast(self.context.device.type, dtype=torch.bfloat16,
                            enabled=self.context.device.type == "cuda"):
            logits = self.model(self._prep(x)).float()
        return {"validation_loss": F.cross_entropy(logits, y),
                "validation_error": (logits.argmax(1) != y).float().mean()}

    def build_training_data_loader(self):
        n = int(self.context.get_hparams().get("train_records", 50000))
        return pytorch.DataLoader(cifar.SyntheticCIFAR10(n, seed=0), collate_fn=cifar.collate,
                                  batch_size=self.context.get_per_slot_batch_size(), shuffle=True)

    def build_validation_data_loader(self):
        n = int(self.context.get_hparams().get("val_records", 10000))
        return pytorch.DataLoader(cifar.SyntheticCIFAR10(n, seed=1, label_noise=0.0),
                                  collate_fn=cifar.collate,
                                  batch_size=self.context.get_per_slot_batch_size())
