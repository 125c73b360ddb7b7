"""ResNet-50 PyTorchTrial (the headline benchmark model; reference uses torchvision ResNet-50 in
examples/deepspeed_autotune/torchvision). bf16 NHWC, fused BN(+add)(+ReLU) HIP kernels, fused SGD,
bucketed RCCL all-reduce for slots_per_trial > 1. Synthetic ImageNet-shaped data resident in HBM."""
import torch
import torch.nn.functional as F

from determined_clone_amd import pytorch
from determined_clone_amd.models import resnet


class ResNet50Trial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.model = context.wrap_model(resnet.to_mi355x_layout(resnet.resnet50()))
        lr = hp.get("lr", 0.1) * context.get_global_batch_size() / 256
        self.opt = context.wrap_optimizer(torch.optim.SGD(self.model.parameters(), lr=lr, momentum=0.9,
                                                          weight_decay=hp.get("weight_decay", 5e-5)))

    def train_batch(self, batch, epoch_idx, batch_idx):
        x, y = batch
        loss = F.cross_entropy(self.model(x).float(), y)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss}

    def evaluate_batch(self, batch, batch_idx):
        x, y = batch
        logits = self.model(x).float()
        return {"validation_loss": F.cross_entropy(logits, y),
                "top1_error": (logits.argmax(1) != y).float().mean()}

    def _data(self, n):
        dev, bs = self.context.device, self.context.get_per_slot_batch_size()
        g = torch.Generator().manual_seed(self.context.distributed.rank)
        dt = torch.bfloat16 if dev.type == "cuda" else torch.float32
        batches = [(torch.randn(bs, 3, 224, 224, generator=g).to(dev, dt).contiguous(memory_format=torch.channels_last),
                    torch.randint(0, 1000, (bs,), generator=g).to(dev)) for _ in range(4)]
        return pytorch.DataLoader(pytorch.DeviceBatchDataset(batches, n), batch_size=None)

    def build_training_data_loader(self):
        return self._data(5000 * self.context.distributed.size)

    def build_validation_data_loader(self):
        return self._data(4 * self.context.distributed.size)
