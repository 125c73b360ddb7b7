"""Batch inference with ``torch_batch_process``: sharding, checkpoint/resume, preemption and the
output location are handled by the API; the user writes ``process_batch`` and the flush."""
import torch

from determined_clone_amd.pytorch import experimental
from model import SyntheticCifar, build_model


class Predictor(experimental.TorchBatchProcessor):
    def __init__(self, context: experimental.TorchBatchProcessorContext) -> None:
        self.context = context
        self.model = context.prepare_model_for_inference(build_model())
        self.rows = []

    def process_batch(self, batch, batch_idx: int) -> None:
        idx, x = batch
        with torch.no_grad():
            pred = self.model(self.context.to_device(x)).argmax(1).cpu()
        self.rows.append(torch.stack([idx, pred], 1))

    def on_checkpoint_start(self) -> None:
        with self.context.upload_path() as path:
            if self.rows:
                out = torch.cat(self.rows)
                torch.save(out, path / f"predictions_{int(out[-1, 0])}.pt")
        self.rows = []


if __name__ == "__main__":
    experimental.torch_batch_process(Predictor, SyntheticCifar(), batch_size=64, checkpoint_interval=2)
