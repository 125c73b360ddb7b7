"""Multi-process data-parallel correctness on CPU (gloo, world_size 2)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank: int, world: int, port: int) -> None:
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world)})
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)


def _model() -> torch.nn.Module:
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))


def _data(n=8):
    g = torch.Generator().manual_seed(42)
    return torch.randn(n, 16, generator=g), torch.randn(n, 4, generator=g)


def _worker_sync(rank: int, world: int, port: int, fused: bool, agg: int, out_dir: str,
                 keep_original: bool = False, lazy: bool = False) -> None:
    _init(rank, world, port)
    if lazy:  # RCCL-like async collectives: data moves only at wait()
        from tests import lazy_collectives

        lazy_collectives.install()
    from determined_clone_amd import core, pytorch

    dist_ctx = core.DistributedContext.from_torch_distributed()
    with pytorch.init(hparams={}, distributed=dist_ctx, aggregation_frequency=agg,
                      exp_conf={"optimizations": {}}) as ctx:
        model = ctx.wrap_model(_model())
        orig = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
        sched = None
        if keep_original:
            # user code that ignores wrap_optimizer's return value and schedules the original
            ctx.wrap_optimizer(orig, fused=fused)
            opt = orig
            sched = torch.optim.lr_scheduler.StepLR(orig, step_size=1, gamma=0.5)
        else:
            opt = ctx.wrap_optimizer(orig, fused=fused)
        x, y = _data(8 * agg)
        b = 8 // world  # per-rank share of each 8-record global micro batch
        for step in range(3):
            for micro in range(agg):
                ctx._current_batch_idx = step * agg + micro
                lo = micro * 8 + rank * b
                xb, yb = x[lo:lo + b], y[lo:lo + b]
                loss = torch.nn.functional.mse_loss(model(xb), yb)
                ctx.backward(loss)
                ctx.step_optimizer(opt)
            if sched is not None:
                sched.step()
        torch.save({k: v.detach().clone() for k, v in model.state_dict().items()},
                   os.path.join(out_dir, f"r{rank}.pt"))
    torch.distributed.destroy_process_group()


def _reference(agg: int, scheduled: bool = False):
    model = _model()
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5) if scheduled else None
    x, y = _data(8 * agg)
    for step in range(3):
        opt.zero_grad()
        for micro in range(agg):
            xb, yb = x[micro * 8:(micro + 1) * 8], y[micro * 8:(micro + 1) * 8]
            (torch.nn.functional.mse_loss(model(xb), yb) / agg).backward()
        opt.step()
        if sched is not None:
            sched.step()
    return model.state_dict()


@pytest.mark.parametrize("world,fused,agg,lazy", [(2, False, 1, False), (2, True, 1, False), (2, True, 2, False),
                                                  (2, False, 2, False), (4, True, 1, False), (8, True, 2, False),
                                                  (8, False, 1, False), (2, True, 1, True), (4, True, 2, True),
                                                  (2, False, 1, True)])
def test_data_parallel_matches_single_process(world, fused, agg, lazy):
    """Bucketed all-reduce DDP at 2 ranks and at the driver's 4 / 8-rank layouts (VERDICT r5 #5;
    676 parameters: not a multiple of 8), every rank bit-identical, equal to one process on the
    full batch. ``lazy``: the bucket all-reduces complete only when waited for (RCCL semantics,
    tests/lazy_collectives.py), so a read before the wait would show."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker_sync, args=(world, _free_port(), fused, agg, d, False, lazy),
                           nprocs=world, start_method="spawn")
        ref = _reference(agg)
        outs = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
        for k in ref:
            for o in outs[1:]:
                torch.testing.assert_close(outs[0][k], o[k], atol=0, rtol=0)
            torch.testing.assert_close(outs[0][k], ref[k], atol=1e-5, rtol=1e-5)


def test_data_parallel_original_optimizer_object_drives_fused_replacement():
    # wrap_optimizer swaps torch SGD for the fused flat-buffer SGD; stepping (and LR-scheduling)
    # the ORIGINAL object must still all-reduce gradients and train the replacement
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker_sync, args=(world, _free_port(), True, 1, d, True),
                           nprocs=world, start_method="spawn")
        ref = _reference(1, scheduled=True)
        r0 = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "r1.pt"), weights_only=True)
        for k in ref:
            torch.testing.assert_close(r0[k], r1[k], atol=0, rtol=0)
            torch.testing.assert_close(r0[k], ref[k], atol=1e-5, rtol=1e-5)


def test_step_optimizer_refuses_unwrapped_optimizer_when_distributed():
    from determined_clone_amd import errors
    from determined_clone_amd.pytorch._context import PyTorchTrialContext

    ctx = PyTorchTrialContext.__new__(PyTorchTrialContext)
    ctx._aggregation_frequency = 1
    ctx._managed_training = False
    ctx._optimizer_alias = {}
    ctx.optimizers = []

    class _D:
        size = 2

    ctx.distributed = _D()
    opt = torch.optim.SGD(_model().parameters(), lr=0.1)
    with pytest.raises(errors.InvalidExperimentException, match="wrap_optimizer"):
        ctx.step_optimizer(opt)


def _worker_core(rank: int, world: int, port: int, out_dir: str) -> None:
    _init(rank, world, port)
    from determined_clone_amd import core

    d = core.DistributedContext.from_torch_distributed()
    assert d.allgather(rank) == [0, 1]
    g = d.gather(rank * 10)
    assert (g == [0, 10]) if rank == 0 else g is None
    assert d.broadcast("chief" if rank == 0 else None) == "chief"
    assert d.allgather_local(rank) == [0, 1]
    open(os.path.join(out_dir, f"ok{rank}"), "w").close()
    torch.distributed.destroy_process_group()


def test_core_distributed_context_collectives():
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker_core, args=(2, _free_port(), d), nprocs=2, start_method="spawn")
        assert os.path.exists(os.path.join(d, "ok0")) and os.path.exists(os.path.join(d, "ok1"))


def _worker_dist_after_close(rank: int, world: int, port: int, out_dir: str) -> None:
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world)})
    from determined_clone_amd import core

    # from_torch_distributed() initialises the default group itself here
    with core.init(distributed=core.DistributedContext.from_torch_distributed()) as ctx:
        assert ctx.distributed.allgather(rank) == list(range(world))
    # user code keeps using torch.distributed after the Core API context closed
    t = torch.tensor([rank + 1.0])
    torch.distributed.all_reduce(t)
    torch.distributed.barrier()
    assert t.item() == sum(range(1, world + 1))
    open(os.path.join(out_dir, f"ok{rank}"), "w").close()
    torch.distributed.destroy_process_group()


def test_default_group_survives_core_context_close():
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker_dist_after_close, args=(2, port, d), nprocs=2, join=True)
        assert sorted(os.listdir(d)) == ["ok0", "ok1"]


def _worker_exit_after_close(rank: int, world: int, port: int, out_dir: str) -> None:
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world)})
    from determined_clone_amd import core

    with core.init(distributed=core.DistributedContext.from_torch_distributed()) as ctx:
        assert ctx.distributed.allgather(rank) == list(range(world))
        assert ctx.distributed.allgather_local(rank) == list(range(world))
    open(os.path.join(out_dir, f"ok{rank}"), "w").close()
    # no destroy_process_group(): the process exits straight after close() with the default
    # group still up, and must not abort in a group destructor


def test_exit_straight_after_core_context_close_is_clean():
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.start_processes(_worker_exit_after_close, args=(2, _free_port(), d), nprocs=2,
                                 start_method="spawn", join=False)
        while not ctx.join():
            pass
        assert [p.exitcode for p in ctx.processes] == [0, 0]
        assert sorted(os.listdir(d)) == ["ok0", "ok1"]
