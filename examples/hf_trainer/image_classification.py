"""Hugging Face Trainer image classification + DetCallback (reference:
examples/hf_trainer_api/hf_image_classification/image_classification.py).

A randomly initialised ViT (no checkpoint download in this environment) is trained on a
synthetic 10-class image set whose classes are separable colour/texture patterns, with accuracy
computed by ``compute_metrics``. Metrics, checkpoints, searcher progress and preemption flow
through the Core API via ``DetCallback``; on MI355X the Trainer runs in bf16.
"""
from typing import Any, Dict, Optional

import numpy as np
import torch
import transformers

import determined_clone_amd as det
from determined_clone_amd import core
from determined_clone_amd.transformers import DetCallback


class SyntheticImages(torch.utils.data.Dataset):
    def __init__(self, n: int = 512, size: int = 32, classes: int = 10, seed: int = 0) -> None:
        g = torch.Generator().manual_seed(seed)
        # class = a colour (per-channel offset) plus a fixed texture; noise on top
        pg = torch.Generator().manual_seed(99)
        protos = 2 * torch.rand(classes, 3, 1, 1, generator=pg) + 0.5 * torch.rand(
            classes, 3, size, size, generator=pg)
        self.labels = torch.randint(0, classes, (n,), generator=g)
        self.pixels = protos[self.labels] + 0.1 * torch.randn(n, 3, size, size, generator=g)

    def __len__(self) -> int:
        return len(self.labels)

    def __getitem__(self, i: int) -> Dict[str, Any]:
        return {"pixel_values": self.pixels[i], "labels": self.labels[i]}


def compute_metrics(p: transformers.EvalPrediction) -> Dict[str, float]:
    return {"accuracy": float((np.argmax(p.predictions, axis=1) == p.label_ids).mean())}


def build_model(size: int = 32, classes: int = 10) -> transformers.PreTrainedModel:
    cfg = transformers.ViTConfig(image_size=size, patch_size=4, num_channels=3, hidden_size=128,
                                 num_hidden_layers=4, num_attention_heads=4,
                                 intermediate_size=256, num_labels=classes)
    return transformers.ViTForImageClassification(cfg)


def main(max_steps: Optional[int] = None, output_dir: str = "/tmp/hf_img_out",
         hparams: Optional[Dict[str, Any]] = None) -> Dict[str, float]:
    info = det.get_cluster_info()
    hp = hparams or (info.trial.hparams if info else {"learning_rate": 1e-3})
    if max_steps is None:  # on-cluster: the searcher's max_length (batches)
        max_steps = int(info.trial._config["searcher"]["max_length"]["batches"]) if info else 300
    eval_every = max(max_steps // 4, 1)
    args = transformers.TrainingArguments(
        output_dir=output_dir, max_steps=max_steps, per_device_train_batch_size=32,
        per_device_eval_batch_size=64, learning_rate=float(hp["learning_rate"]),
        eval_strategy="steps", eval_steps=eval_every, save_steps=eval_every,
        logging_steps=max(eval_every // 2, 1), report_to=[], remove_unused_columns=False,
        bf16=torch.cuda.is_available(), dataloader_num_workers=0)
    distributed = core.DistributedContext.from_torch_distributed() if args.world_size > 1 else None
    with core.init(distributed=distributed) as core_context:
        # DetCallback needs a trial (on-cluster or unmanaged); off-cluster it is left out.
        callbacks = [DetCallback(core_context, args)] if info is not None else []
        trainer = transformers.Trainer(model=build_model(), args=args,
                                       train_dataset=SyntheticImages(),
                                       eval_dataset=SyntheticImages(128, seed=1),
                                       compute_metrics=compute_metrics, callbacks=callbacks)
        trainer.train(resume_from_checkpoint=args.resume_from_checkpoint)
        return trainer.evaluate()


if __name__ == "__main__":
    main()
