"""Core API training loop for DeepSpeed autotune (reference: examples/deepspeed_autotune/
torchvision/core_api/script.py). dsat-specific: ``dsat.get_ds_config_from_hparams`` for the engine
config, and the engine's forward / backward / step inside ``dsat.dsat_reporting_context`` -- in a
dsat profiling trial the native engine measures the configured steps, writes its json and exits;
the context reports it for the searcher operation. Outside dsat this is an ordinary Core API loop
with metric reporting, checkpoints, resume and preemption.

``python -m determined_clone_amd.pytorch.dsat binary deepspeed.yaml .``
"""
import json
import logging
import os

import torch
import torch.nn.functional as F

import determined_clone_amd as det
from determined_clone_amd import core
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


def main(core_context: core.Context, hparams: dict) -> None:
    ds_config = dsat.get_ds_config_from_hparams(hparams)
    model = MODELS[hparams["model_name"]](num_classes=int(hparams["num_classes"]))
    if torch.cuda.is_available():
        model = resnet.to_mi355x_layout(model)
    engine, _, _, _ = det_ds.initialize(model=model, model_parameters=model.parameters(),
                                        config=ds_config)
    dtype = torch.bfloat16 if engine.config.bf16 else torch.float32
    mbs = engine.train_micro_batch_size_per_gpu()
    ds = RandomImages(1 << 20, int(hparams["image_size"]), int(hparams["num_classes"]))
    sampler = torch.utils.data.distributed.DistributedSampler(
        ds, num_replicas=core_context.distributed.size, rank=core_context.distributed.rank)
    loader = iter(torch.utils.data.DataLoader(ds, batch_size=mbs, sampler=sampler))

    steps_completed = 0
    info = det.get_cluster_info()
    if info is not None and info.latest_checkpoint is not None:
        with core_context.checkpoint.restore_path(info.latest_checkpoint) as path:
            engine.load_checkpoint(path)
            steps_completed = json.loads((path / "state.json").read_text())["steps_completed"]

    def step() -> torch.Tensor:
        x, y = next(loader)
        x = x.to(engine.device, dtype)
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
        loss = F.cross_entropy(engine(x).float(), y.to(engine.device))
        engine.backward(loss)
        engine.step()
        return loss

    for op in core_context.searcher.operations():
        # a dsat profiling trial ends inside this context (SystemExit after reporting)
        with dsat.dsat_reporting_context(core_context, op):
            losses = []
            while steps_completed < op.length:
                losses.append(step().item())
                steps_completed += 1
                if steps_completed % int(hparams.get("report_rate", 10)) == 0:
                    core_context.train.report_training_metrics(
                        steps_completed, {"loss": sum(losses) / len(losses)})
                    losses = []
                if steps_completed % int(hparams.get("checkpoint_rate", 50)) == 0 or \
                        steps_completed == op.length:
                    # every rank writes its ZeRO optimizer shard into the one checkpoint
                    with core_context.checkpoint.store_path({"steps_completed": steps_completed},
                                                            shard=True) as (path, _):
                        engine.save_checkpoint(path)
                        if core_context.distributed.rank == 0:
                            (path / "state.json").write_text(json.dumps({"steps_completed": steps_completed}))
                    if core_context.preempt.should_preempt():
                        return
            with torch.no_grad():
                x, y = next(loader)
                x = x.to(engine.device, dtype)
                if x.is_cuda:
                    x = x.contiguous(memory_format=torch.channels_last)
                val = F.cross_entropy(engine(x).float(), y.to(engine.device)).item()
            core_context.train.report_validation_metrics(steps_completed, {"val_loss": val})
            op.report_completed(val)


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format=det.LOG_FORMAT)
    info = det.get_cluster_info()
    hp = info.trial.hparams if info is not None else json.loads(os.environ.get("DSAT_HPARAMS", "{}"))
    distributed = core.DistributedContext.from_deepspeed() if "RANK" in os.environ else None
    with core.init(distributed=distributed) as core_context:
        main(core_context, hp)
