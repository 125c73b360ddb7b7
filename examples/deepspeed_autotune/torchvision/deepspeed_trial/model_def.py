"""DeepSpeedTrial for DeepSpeed autotune (reference: examples/deepspeed_autotune/torchvision/
deepspeed_trial/model_def.py). The only dsat-specific line is ``dsat.get_ds_config_from_hparams``:
the trial builds its engine from ds_config.json with the search's overwrite merged in; in a dsat
profiling trial the config's ``autotuning`` section makes the native engine measure itself.

Models: torchvision's ResNet v1.5 as ``models/resnet.py`` (torchvision is not in the image; NHWC
bf16 on MI355X); data: random ImageNet-like images.

``python -m determined_clone_amd.pytorch.dsat asha deepspeed.yaml .``
"""
import torch
import torch.nn.functional as F

from determined_clone_amd import pytorch
from determined_clone_amd.models import resnet
from determined_clone_amd.pytorch import deepspeed as det_ds
from determined_clone_amd.pytorch import dsat

MODELS = {"resnet50": resnet.resnet50, "resnet_tiny": resnet.resnet18_bottleneck_tiny}


class RandomImages(torch.utils.data.Dataset):
    def __init__(self, n: int, size: int, num_classes: int) -> None:
        self.n, self.size, self.num_classes = n, size, num_classes

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i: int):
        g = torch.Generator().manual_seed(i)
        return (torch.randn(3, self.size, self.size, generator=g),
                torch.randint(0, self.num_classes, (), generator=g))


class TorchvisionTrial(det_ds.DeepSpeedTrial):
    def __init__(self, context: det_ds.DeepSpeedTrialContext) -> None:
        self.context = context
        self.hparams = context.get_hparams()
        ds_config = dsat.get_ds_config_from_hparams(self.hparams)
        model = MODELS[self.hparams["model_name"]](num_classes=int(self.hparams["num_classes"]))
        if torch.cuda.is_available():
            model = resnet.to_mi355x_layout(model)  # channels_last weights for the NHWC kernels
        engine, _, _, _ = det_ds.initialize(model=model, model_parameters=model.parameters(),
                                            config=ds_config)
        self.engine = context.wrap_model_engine(engine)
        self.dtype = torch.bfloat16 if engine.config.bf16 else torch.float32

    def _loss(self, it):
        x, y = next(it)
        x = x.to(self.engine.device, self.dtype)
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
        return F.cross_entropy(self.engine(x).float(), y.to(self.engine.device))

    def train_batch(self, iter_dataloader, epoch_idx, batch_idx):
        loss = self._loss(iter_dataloader)
        self.engine.backward(loss)
        self.engine.step()
        return {"loss": loss}

    def evaluate_batch(self, iter_dataloader, batch_idx):
        return {"val_loss": self._loss(iter_dataloader)}

    def _data(self, n: int) -> pytorch.DataLoader:
        ds = RandomImages(n, int(self.hparams["image_size"]), int(self.hparams["num_classes"]))
        return pytorch.DataLoader(ds, batch_size=self.context.train_micro_batch_size_per_gpu)

    def build_training_data_loader(self):
        return self._data(1 << 20)

    def build_validation_data_loader(self):
        return self._data(4 * self.context.train_micro_batch_size_per_gpu)
