"""The same batch inference written against the Core API directly: the script shards the
dataset by rank itself, keeps its own resume state in checkpoints, reports progress, checks for
preemption and gathers per-rank counts -- everything ``torch_batch_process`` does for you."""
import json
import os
import pathlib

import torch

import determined_clone_amd as det
from determined_clone_amd import core
from model import SyntheticCifar, build_model

BATCH, CKPT_EVERY = 64, 2


def run(ctx: core.Context, op) -> bool:
    """Process this rank's shard; False when preempted (a later run resumes)."""
    rank, size = ctx.distributed.rank, ctx.distributed.size
    info = det.get_cluster_info()
    done_batches = 0
    if info is not None and info.latest_checkpoint:  # resume after the last checkpointed batch
        with ctx.checkpoint.restore_path(info.latest_checkpoint) as path:
            done_batches = json.loads((pathlib.Path(path) / "state.json").read_text())["batches"]
    ds = SyntheticCifar()
    mine = list(range(rank, len(ds), size))  # this rank's shard
    batches = [mine[i:i + BATCH] for i in range(0, len(mine), BATCH)]
    dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    model = build_model().to(dev).eval()
    out_dir = pathlib.Path(os.environ.get("PREDICTIONS_DIR", "/tmp/core_api_predictions"))
    out_dir.mkdir(parents=True, exist_ok=True)
    rows = []
    for b in range(done_batches, len(batches)):
        idx = torch.tensor(batches[b])
        x = torch.stack([ds[i][1] for i in batches[b]]).to(dev)
        with torch.no_grad():
            rows.append(torch.stack([idx, model(x).argmax(1).cpu()], 1))
        if (b + 1) % CKPT_EVERY == 0 or b + 1 == len(batches):
            torch.save(torch.cat(rows), out_dir / f"rank{rank}_upto{b + 1}.pt")
            rows = []
            ctx.distributed.allgather(None)  # every rank reached the same point
            if rank == 0:
                with ctx.checkpoint.store_path({"steps_completed": b + 1}) as (path, _):
                    (pathlib.Path(path) / "state.json").write_text(json.dumps({"batches": b + 1}))
                op.report_progress(op.length * (b + 1) / len(batches))
            if ctx.preempt.should_preempt():
                return False
    counts = ctx.distributed.gather(len(mine))
    if rank == 0:
        ctx.train.report_validation_metrics(steps_completed=len(batches), metrics={"predicted": sum(counts)})
        op.report_completed(sum(counts))
    return True


def main(ctx: core.Context) -> None:
    for op in ctx.searcher.operations():
        if not run(ctx, op):
            return


if __name__ == "__main__":
    dist = core.DistributedContext.from_torch_distributed() if int(os.environ.get("WORLD_SIZE", "1")) > 1 else None
    with core.init(distributed=dist) as ctx:
        main(ctx)
