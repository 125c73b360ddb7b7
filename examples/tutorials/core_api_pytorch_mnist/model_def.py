"""Core API + plain PyTorch MNIST (reference: examples/tutorials/core_api_pytorch_mnist,
model_def{,_metrics,_checkpoints,_adaptive,_distributed}.py folded into one script).

No Trial class: an ordinary PyTorch training loop that
  * reports training / validation metrics          (core_context.train)
  * checkpoints every epoch and resumes from the latest checkpoint, pausing on preemption
                                                   (core_context.checkpoint / core_context.preempt)
  * follows the searcher's operations (epochs) so adaptive_asha can stop or extend it
                                                   (core_context.searcher)
  * trains data-parallel under the torch_distributed launcher: each rank reads its shard and
    gradients are all-reduced over RCCL (gloo on CPU slots) before every step
                                                   (core_context.distributed)
Off-cluster (``python model_def.py``) it runs with default hyperparameters and a dummy context.
Data: IDX files under ./data if present, else offline synthetic MNIST-shaped data.
"""
import logging
import os
import pathlib
from typing import Any, Dict, Optional, Tuple

import torch
import torch.nn.functional as F

import determined_clone_amd as det
from determined_clone_amd import core
from determined_clone_amd.models import mnist
from determined_clone_amd.parallel.ddp import allreduce_loose_grads, broadcast_module_state

DEFAULT_HPARAMS = {"global_batch_size": 64, "learning_rate": 1.0, "n_filters1": 32,
                   "n_filters2": 64, "dropout1": 0.25, "dropout2": 0.5, "synthetic_size": 6000,
                   "epochs": 2}


def _loader(dataset: Any, batch: int, dist: core.DistributedContext, shuffle: bool) -> Any:
    sampler = torch.utils.data.DistributedSampler(dataset, num_replicas=dist.size, rank=dist.rank,
                                                  shuffle=shuffle, seed=0)
    return torch.utils.data.DataLoader(dataset, batch_size=batch, sampler=sampler)


def load_state(path: pathlib.Path, trial_id: int, model: torch.nn.Module,
               opt: torch.optim.Optimizer) -> int:
    """Restore model/optimizer; returns the epochs already completed. A checkpoint from another
    trial (``continue`` / fork) restores weights but restarts the epoch count."""
    state = torch.load(path / "checkpoint.pt", map_location="cpu", weights_only=True)
    model.load_state_dict(state["model"])
    opt.load_state_dict(state["optimizer"])
    epochs, ckpt_trial = (int(v) for v in (path / "state").read_text().split(","))
    return epochs if ckpt_trial == trial_id else 0


def train_epoch(model: torch.nn.Module, loader: Any, opt: torch.optim.Optimizer, device: Any,
                core_context: core.Context, epoch: int, log_every: int = 20) -> None:
    dist = core_context.distributed
    model.train()
    loader.sampler.set_epoch(epoch)
    for i, (x, y) in enumerate(loader):
        x, y = x.to(device), y.to(device)
        opt.zero_grad(set_to_none=False)
        loss = F.nll_loss(model(x), y)
        loss.backward()
        if dist.size > 1:
            allreduce_loose_grads([p for p in model.parameters() if p.grad is not None])
        opt.step()
        if (i + 1) % log_every == 0:
            losses = dist.gather(float(loss))
            if dist.rank == 0:
                core_context.train.report_training_metrics(
                    steps_completed=epoch * len(loader) + i + 1,
                    metrics={"train_loss": sum(losses) / len(losses)})


def evaluate(model: torch.nn.Module, loader: Any, device: Any,
             dist: core.DistributedContext) -> Tuple[float, float]:
    model.eval()
    loss_sum, correct, n = 0.0, 0, 0
    with torch.no_grad():
        for x, y in loader:
            x, y = x.to(device), y.to(device)
            out = model(x)
            loss_sum += float(F.nll_loss(out, y, reduction="sum"))
            correct += int((out.argmax(1) == y).sum())
            n += len(y)
    parts = dist.allgather((loss_sum, correct, n))
    total = sum(p[2] for p in parts)
    return sum(p[0] for p in parts) / total, sum(p[1] for p in parts) / total


def main(core_context: core.Context, hparams: Dict[str, Any], trial_id: int = 0,
         latest_checkpoint: Optional[str] = None, data_dir: Optional[str] = "data") -> float:
    dist = core_context.distributed
    if torch.cuda.is_available():
        device = torch.device("cuda", dist.local_rank)
        torch.cuda.set_device(device)
    else:
        device = torch.device("cpu")
    torch.manual_seed(1)
    model = mnist.build_model(hparams).to(device)
    opt = torch.optim.Adadelta(model.parameters(), lr=float(hparams["learning_rate"]))
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.7)
    epochs_done = 0
    if latest_checkpoint is not None:
        with core_context.checkpoint.restore_path(latest_checkpoint) as path:
            epochs_done = load_state(pathlib.Path(path), trial_id, model, opt)
    if dist.size > 1:
        broadcast_module_state(model)

    per_rank = int(hparams["global_batch_size"]) // dist.size
    n = int(hparams.get("synthetic_size", 6000))
    train_loader = _loader(mnist.get_dataset(data_dir, True, synthetic_size=n), per_rank, dist, True)
    test_loader = _loader(mnist.get_dataset(data_dir, False, synthetic_size=max(n // 6, 100)),
                          per_rank, dist, False)

    test_loss = float("nan")
    epoch = epochs_done
    for op in core_context.searcher.operations():
        while epoch < op.length:
            train_epoch(model, train_loader, opt, device, core_context, epoch)
            epoch += 1
            sched.step()
            steps = epoch * len(train_loader)
            test_loss, acc = evaluate(model, test_loader, device, dist)
            if dist.rank == 0:
                core_context.train.report_validation_metrics(
                    steps_completed=steps, metrics={"test_loss": test_loss, "accuracy": acc})
                op.report_progress(epoch)
                with core_context.checkpoint.store_path({"steps_completed": steps}) as (path, _):
                    torch.save({"model": model.state_dict(), "optimizer": opt.state_dict()},
                               pathlib.Path(path) / "checkpoint.pt")
                    (pathlib.Path(path) / "state").write_text(f"{epoch},{trial_id}")
            if core_context.preempt.should_preempt():
                return test_loss
        if dist.rank == 0:
            op.report_completed(test_loss)
    return test_loss


def run() -> None:
    info = det.get_cluster_info()
    distributed = (core.DistributedContext.from_torch_distributed()
                   if int(os.environ.get("WORLD_SIZE", "1")) > 1 else None)
    with core.init(distributed=distributed) as core_context:
        if info is None:  # off-cluster: the dummy searcher runs ``epochs`` epochs
            hp = dict(DEFAULT_HPARAMS)
            core_context.searcher._length = int(hp["epochs"])  # noqa: SLF001
            main(core_context, hp)
        else:
            main(core_context, {**DEFAULT_HPARAMS, **info.trial.hparams}, info.trial.trial_id,
                 info.latest_checkpoint)


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format=det.LOG_FORMAT)
    run()
