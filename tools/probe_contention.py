"""Side-stream contention probe for the ResNet-50 bench step (VERDICT r5 "3x3 implicit GEMM runs
slower in the step than isolated").

Runs the bench's PyTorchTrial step (same model, batch, optimizer, Trainer path) in one of:
  --mode normal       the bench step (weight gradients on the side stream)
  --mode freeze_conv  convolution weights frozen: no convolution weight gradient anywhere, so the
                      main stream runs alone (every data gradient and BatchNorm still runs)
and prints one JSON line with the mean step time. ``DCA_WGRAD_STREAM=0`` with ``--mode normal``
gives the serial (no overlap) step. main-alone + side-alone vs overlapped step = contention cost.
Usage: ``python tools/probe_contention.py --mode freeze_conv [--steps 10 --warmup 4]``."""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="normal", choices=["normal", "freeze_conv"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--batch", type=int, default=1024)
    args = ap.parse_args()
    from determined_clone_amd.ops import miopen_db

    miopen_db.use_private_copy("probe")
    os.environ.setdefault("DCA_GEMM_TUNED", "1")
    import torch
    import torch.nn.functional as F

    from determined_clone_amd import pytorch
    from determined_clone_amd.models import resnet

    torch.backends.cudnn.benchmark = False
    times = []

    class Trial(pytorch.PyTorchTrial):
        def __init__(self, context):
            self.context = context
            model = resnet.to_mi355x_layout(resnet.resnet50())
            if args.mode == "freeze_conv":
                for p in model.parameters():
                    if p.dim() == 4:
                        p.requires_grad_(False)
            self.model = context.wrap_model(model)
            opt = torch.optim.SGD([p for p in self.model.parameters() if p.requires_grad], lr=0.4,
                                  momentum=0.9, weight_decay=5e-5)
            self.opt = context.wrap_optimizer(opt)

        def train_batch(self, batch, epoch_idx, batch_idx):
            torch.cuda.synchronize()
            t = time.perf_counter()
            images, labels = batch
            loss = F.cross_entropy(self.model(images).float(), labels)
            self.context.backward(loss)
            self.context.step_optimizer(self.opt)
            torch.cuda.synchronize()
            if batch_idx >= args.warmup:
                times.append((time.perf_counter() - t) * 1e3)
            return {"loss": loss}

        def evaluate_batch(self, batch, batch_idx):
            return {"val_loss": torch.zeros(())}

        def _data(self, n):
            g = torch.Generator(device="cpu").manual_seed(1234)
            out = []
            for _ in range(2):
                x = torch.randn(args.batch, 3, 224, 224, generator=g).to("cuda", torch.bfloat16)
                out.append((x.contiguous(memory_format=torch.channels_last),
                            torch.randint(0, 1000, (args.batch,), generator=g).cuda()))
            return pytorch.DataLoader(pytorch.DeviceBatchDataset(out, n), batch_size=None)

        def build_training_data_loader(self):
            return self._data(10000)

        def build_validation_data_loader(self):
            return self._data(1)

    total = args.steps + args.warmup
    hp = {"global_batch_size": args.batch}
    with pytorch.init(hparams=hp, exp_conf={"optimizations": {"aggregation_frequency": 1}}) as ctx:
        trainer = pytorch.Trainer(Trial(ctx), ctx)
        trainer.fit(max_length=pytorch.Batch(total), reporting_period=pytorch.Batch(total),
                    checkpoint_policy="none")
    ms = sum(times) / len(times)
    print(json.dumps({"mode": args.mode, "wgrad_stream": os.environ.get("DCA_WGRAD_STREAM", "1"),
                      "ms_per_step": round(ms, 3), "min_ms": round(min(times), 3),
                      "img_s": round(args.batch / ms * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
