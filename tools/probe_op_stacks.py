"""Which Python call sites launch a given ATen op during a ResNet-50 training step.

Runs a few forward/backward/optimizer steps of the bench model under ``torch.profiler`` with
Python stacks and prints, per distinct stack, how many times per step the op ran (e.g. the small
``FillFunctor<float>`` launches seen in the rocprof step breakdown). GPU only.

Usage: python tools/probe_op_stacks.py --op aten::fill_ --batch 256
"""
import argparse
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="aten::fill_")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()

    import torch
    import torch.nn.functional as F
    from torch.profiler import ProfilerActivity, profile

    from determined_clone_amd import pytorch
    from determined_clone_amd.models import resnet

    class T(pytorch.PyTorchTrial):
        def __init__(self, context):
            self.context = context
            self.model = context.wrap_model(resnet.to_mi355x_layout(resnet.resnet50()))
            self.opt = context.wrap_optimizer(torch.optim.SGD(self.model.parameters(), lr=0.1, momentum=0.9))
            self.n = 0
            self.prof = None

        def train_batch(self, batch, epoch_idx, batch_idx):
            if batch_idx == 3:
                torch.cuda.synchronize()
                self.prof = profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True)
                self.prof.__enter__()
            x, y = batch
            loss = F.cross_entropy(self.model(x).float(), y)
            self.context.backward(loss)
            self.context.step_optimizer(self.opt)
            if batch_idx == 3 + a.steps - 1:
                torch.cuda.synchronize()
                self.prof.__exit__(None, None, None)
                stacks = Counter()
                for ev in self.prof.events():
                    if ev.name == a.op:
                        st = [s for s in (ev.stack or []) if "determined_clone_amd" in s or "bench" in s
                              or "torch/autograd" in s or "torch/nn" in s][:6]
                        # enclosing ops (e.g. autograd::engine::evaluate_function: XBackward) and
                        # the filled tensor's shape: identifies callers without a Python frame
                        par, chain = ev.cpu_parent, []
                        while par is not None and len(chain) < 4:
                            chain.append(par.name)
                            par = par.cpu_parent
                        shp = str(ev.input_shapes[0]) if ev.input_shapes else "?"
                        stacks[" <- ".join(st or chain) + f"  shape={shp}"] += 1
                for st, c in stacks.most_common(30):
                    print(f"{c / a.steps:6.1f}/step  {st}", flush=True)
            return {"loss": loss}

        def evaluate_batch(self, batch, batch_idx):
            x, y = batch
            return {"val_loss": F.cross_entropy(self.model(x).float(), y)}

        def build_training_data_loader(self):
            dev = self.context.device
            x = torch.randn(a.batch, 3, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            y = torch.randint(0, 1000, (a.batch,), device=dev)
            return pytorch.DataLoader(pytorch.DeviceBatchDataset([(x, y)], 100), batch_size=None)

        def build_validation_data_loader(self):
            return self.build_training_data_loader()

    with pytorch.init(hparams={"global_batch_size": a.batch}) as ctx:
        trial = T(ctx)
        pytorch.Trainer(trial, ctx).fit(max_length=pytorch.Batch(3 + a.steps), checkpoint_policy="none",
                                        reporting_period=pytorch.Batch(3 + a.steps))


if __name__ == "__main__":
    main()
