"""Diagnose data-parallel gradient agreement on one GPU (two gloo ranks on cuda:0).

Prints, per parameter, the relative difference between
  * acc   : one process, both half-batch losses (each /2) backpropagated into the same .grad
  * ref   : (g_half0 + g_half1) / 2 computed from two separate backward passes
  * local : each rank's own half-batch gradient (no sync) vs the single-process g_half<rank>
  * ddp   : the rank's gradient after the bucketed all-reduce (x grad_multiplier) vs ref
"""
import os
import socket
import sys
import tempfile

import torch
import torch.multiprocessing as mp
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HALF = 4


def _model():
    from determined_clone_amd.models import resnet

    torch.manual_seed(0)
    return resnet.to_mi355x_layout(resnet.resnet18_bottleneck_tiny(num_classes=10))


def _data(dev):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2 * HALF, 3, 64, 64, generator=g).to(dev, torch.bfloat16)
    y = torch.randint(0, 10, (2 * HALF,), generator=g).to(dev)
    return x, y


def _half(x, y, h):
    return x[h * HALF:(h + 1) * HALF].contiguous(memory_format=torch.channels_last), y[h * HALF:(h + 1) * HALF]


def _grads(model):
    return {n: p.grad.detach().float().cpu().clone() for n, p in model.named_parameters()}


def _worker(rank, world, port, out):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": "0", "LOCAL_WORLD_SIZE": "1"})
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from determined_clone_amd import core, pytorch

    dist_ctx = core.DistributedContext.from_torch_distributed()
    with pytorch.init(hparams={}, distributed=dist_ctx, exp_conf={"optimizations": {}}) as ctx:
        model = ctx.wrap_model(_model())
        opt = ctx.wrap_optimizer(torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9))
        x, y = _data(ctx.device)
        xb, yb = _half(x, y, rank)
        ctx._current_batch_idx = 0
        with ctx._no_sync():
            F.cross_entropy(model(xb).float(), yb).backward()
        local = _grads(model)
        opt.zero_grad()
        ctx.backward(F.cross_entropy(model(xb).float(), yb))
        sync = list(ctx._syncs.values())[0]
        launched_in_backward = sum(1 for b in sync.buckets if b.launched)
        sync.finish()
        torch.cuda.synchronize()
        ddp = {n: g * opt.grad_multiplier for n, g in _grads(model).items()}
        torch.save({"local": local, "ddp": ddp, "launched": launched_in_backward,
                    "nbuckets": len(sync.buckets), "mult": opt.grad_multiplier},
                   os.path.join(out, f"r{rank}.pt"))
    torch.distributed.destroy_process_group()


def _rel(a, b):
    return ((a - b).norm() / max(b.norm().item(), 1e-12)).item()


def main():
    from determined_clone_amd.ops import optim as fopt

    dev = torch.device("cuda:0")
    with tempfile.TemporaryDirectory() as d:
        s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
        mp.spawn(_worker, args=(2, port, d), nprocs=2, join=True)
        outs = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(2)]
    model = _model().to(dev)
    opt = fopt.FusedSGD(model.parameters(), lr=0.05, momentum=0.9)
    x, y = _data(dev)
    gh = []
    for h in range(2):
        opt.zero_grad()
        xb, yb = _half(x, y, h)
        F.cross_entropy(model(xb).float(), yb).backward()
        gh.append(_grads(model))
    opt.zero_grad()
    for h in range(2):
        xb, yb = _half(x, y, h)
        (F.cross_entropy(model(xb).float(), yb) / 2).backward()
    acc = _grads(model)
    ref = {n: (gh[0][n] + gh[1][n]) / 2 for n in acc}
    for r in range(2):
        print(f"rank{r}: buckets launched during backward {outs[r]['launched']}/{outs[r]['nbuckets']} mult={outs[r]['mult']}")
    print(f"{'param':40s} {'dtype':>6s} {'acc-ref':>9s} {'loc0':>9s} {'loc1':>9s} {'ddp0':>9s} {'ddp1':>9s}")
    for n, p in model.named_parameters():
        print(f"{n:40s} {str(p.dtype)[6:]:>6s} {_rel(acc[n], ref[n]):9.2e} "
              f"{_rel(outs[0]['local'][n], gh[0][n]):9.2e} {_rel(outs[1]['local'][n], gh[1][n]):9.2e} "
              f"{_rel(outs[0]['ddp'][n], ref[n]):9.2e} {_rel(outs[1]['ddp'][n], ref[n]):9.2e}")


if __name__ == "__main__":
    main()
