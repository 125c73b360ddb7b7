"""ZeRO-1/2 partitioned optimizer correctness on CPU (gloo, world_size 2) against the
non-partitioned fused optimizer on the full batch."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from determined_clone_amd.ops import optim as fopt
from determined_clone_amd.parallel import zero


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model() -> torch.nn.Module:
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(16, 40), torch.nn.Tanh(), torch.nn.Linear(40, 24),
                               torch.nn.Tanh(), torch.nn.Linear(24, 4))


def _groups(m):
    decay = [p for n, p in m.named_parameters() if n.endswith("weight")]
    nodecay = [p for n, p in m.named_parameters() if n.endswith("bias")]
    return [{"params": decay, "weight_decay": 0.1}, {"params": nodecay, "weight_decay": 0.0}]


def _data():
    g = torch.Generator().manual_seed(7)
    return torch.randn(16, 16, generator=g), torch.randn(16, 4, generator=g)


STEPS = 4


def _count_collectives():
    """Wrap the tensor collectives so the test can assert which ones ran (the production RCCL
    branch: in-place reduce_scatter_tensor / all_gather_into_tensor, not the list fallbacks)."""
    dist = torch.distributed
    calls = {"reduce_scatter_tensor": 0, "all_gather_into_tensor": 0, "all_gather": 0}
    for name in calls:
        fn = getattr(dist, name)

        def wrapped(*a, __fn=fn, __name=name, **k):
            calls[__name] += 1
            return __fn(*a, **k)
        setattr(dist, name, wrapped)
    return calls


def _worker(rank, world, port, stage, kind, max_norm, bucket_mb, out_dir, defer=False, lazy=False):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    if lazy:  # RCCL-like async collectives: data moves only at wait()
        from tests import lazy_collectives

        lazy_collectives.install()
    calls = _count_collectives()
    m = _model()
    cls = zero.zero_optimizer_for(kind)
    opt = cls(_groups(m), lr=0.05, stage=stage, bucket_mb=bucket_mb, first_bucket_mb=bucket_mb / 4)
    if defer:
        opt.attach_module(m)  # the engines' mode: gathers overlap the next forward
    x, y = _data()
    per = x.shape[0] // world
    for _ in range(STEPS):
        opt.zero_grad()
        xb, yb = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
        torch.nn.functional.mse_loss(m(xb), yb).backward()
        opt.finish_grad_sync()
        if max_norm:
            opt.prepare_grads(max_norm=max_norm)
        opt.step()
    if defer:
        assert opt._gather_pending and opt._gather_hook is not None  # still in flight after step()
    torch.save({"params": {k: v.detach().clone() for k, v in m.state_dict().items()},
                "opt": opt.state_dict(), "calls": calls,
                "pending_after_save": len(opt._gather_pending)}, os.path.join(out_dir, f"r{rank}.pt"))
    torch.distributed.destroy_process_group()


def _reference(kind, max_norm):
    m = _model()
    if kind == "sgd":
        opt = fopt.FusedSGD(_groups(m), lr=0.05, momentum=0.0)
    else:
        opt = fopt.FusedAdam(_groups(m), lr=0.05, adamw=(kind == "adamw"))
    x, y = _data()
    for _ in range(STEPS):
        opt.zero_grad()
        torch.nn.functional.mse_loss(m(x), y).backward()
        if max_norm:
            opt.prepare_grads(max_norm=max_norm)
        opt.step()
    return m, opt


@pytest.mark.parametrize("world,stage,kind,max_norm,bucket_mb,defer,lazy", [
    (2, 1, "adam", 0.0, 64.0, False, False),
    (2, 2, "adam", 0.0, 0.002, True, False),   # many small buckets: hooks fire bucket by bucket
    (2, 2, "adamw", 0.05, 0.002, False, False),  # global-norm clipping across shards
    (2, 2, "sgd", 0.0, 0.001, True, False),
    # the driver's 8-GPU layout: 1764 parameters (not a multiple of 8, so the
    # last shard is padded), 500-float buckets (boundaries inside the 640- and 960-element weights),
    # 8 deferred gathers in flight, clipping over 8 shards
    (4, 2, "adamw", 0.05, 0.002, True, False),
    (8, 1, "adam", 0.0, 64.0, False, False),
    (8, 2, "adamw", 0.05, 0.002, True, False),
    # RCCL-like lazy collectives (tests/lazy_collectives.py): a reduce-scatter / gather output read
    # before its wait would show here
    (2, 2, "adamw", 0.05, 0.002, True, True),
    (4, 1, "adam", 0.0, 0.002, True, True),
])
def test_zero_matches_full_batch(world, stage, kind, max_norm, bucket_mb, defer, lazy):
    assert sum(p.numel() for p in _model().parameters()) % 8 != 0  # padded last shard at world 8
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), stage, kind, max_norm, bucket_mb, d, defer, lazy),
                 nprocs=world, join=True)
        ref, ref_opt = _reference(kind, max_norm)
        outs = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    for k, v in ref.state_dict().items():
        for o in outs:
            torch.testing.assert_close(o["params"][k], v, atol=1e-5, rtol=1e-5)
    for o in outs:
        # gloo on host tensors runs the same in-place collectives as RCCL (parallel/_caps.py)
        assert o["calls"]["all_gather_into_tensor"] > 0 and o["calls"]["all_gather"] == 0, o["calls"]
        assert (o["calls"]["reduce_scatter_tensor"] > 0) == (stage >= 2), o["calls"]
        assert o["pending_after_save"] == 0
    # re-partition: both shards loaded into a single-rank ZeRO optimizer reproduce the
    # full optimizer state of the reference
    if kind != "sgd":
        m1 = _model()
        z1 = zero.zero_optimizer_for(kind)(_groups(m1), lr=0.05, stage=2)
        z1.load_shard_state_dicts([o["opt"] for o in outs])
        full = z1.consolidated_state_dict()
        rsd = ref_opt.state_dict()
        for idx, st in rsd["state"].items():
            torch.testing.assert_close(full["state"][idx]["exp_avg"], st["exp_avg"], atol=1e-6, rtol=1e-5)
            torch.testing.assert_close(full["state"][idx]["exp_avg_sq"], st["exp_avg_sq"], atol=1e-8, rtol=1e-5)


def test_single_rank_zero_equals_fused():
    m1, m2 = _model(), _model()
    z = zero.ZeroAdam(_groups(m1), lr=0.01, stage=2)
    f = fopt.FusedAdam(_groups(m2), lr=0.01)
    x, y = _data()
    for _ in range(3):
        for m, o in ((m1, z), (m2, f)):
            o.zero_grad()
            torch.nn.functional.mse_loss(m(x), y).backward()
            o.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b)
    # own-shard state dict round trip
    sd = z.state_dict()
    m3 = _model()
    z3 = zero.ZeroAdam(_groups(m3), lr=0.01, stage=2)
    z3.load_state_dict(sd)
    assert z3._step == 3
    torch.testing.assert_close(z3.flat[torch.float32].state["exp_avg"], z.flat[torch.float32].state["exp_avg"])


def test_lamb_rejected():
    with pytest.raises(ValueError):
        zero.zero_optimizer_for("lamb")


def _rs_len(world):
    return 3 + 5 * world + 7  # room for the offset-3 bucket plus an untouched tail


def _rs_worker(rank, world, port, out_dir):
    """In-place bucket reduce-scatter exactly as ZeroShardMixin._launch issues it: the output is
    the rank's own chunk of the bucket, a view into the reduced input."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from determined_clone_amd.parallel import _caps

    assert _caps.tensor_collectives(None, torch.device("cpu"))
    chunk = 5
    res = {}
    for start in (0, 3):  # a bucket at offset 0 and one further into the flat buffer
        flat = torch.arange(_rs_len(world), dtype=torch.float32) + 1000 * rank
        full = flat[start:start + world * chunk]
        out = full[rank * chunk:(rank + 1) * chunk]
        before = flat.clone()
        torch.distributed.reduce_scatter_tensor(out, full, op=torch.distributed.ReduceOp.SUM,
                                                async_op=True).wait()
        res[start] = (flat.clone(), before)
    t = torch.tensor([float(rank + 1)])
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.AVG)
    res["avg"] = t
    torch.save(res, os.path.join(out_dir, f"rs{rank}.pt"))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_inplace_reduce_scatter_offsets_per_bucket(world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rs_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        outs = [torch.load(os.path.join(d, f"rs{r}.pt"), weights_only=True) for r in range(world)]
    chunk = 5
    for r, o in enumerate(outs):
        for start in (0, 3):
            after, before = o[start]
            lo, hi = start + r * chunk, start + (r + 1) * chunk
            # own chunk == sum over ranks of that chunk; everything else untouched
            want = sum(outs[q][start][1][lo:hi] for q in range(world))
            torch.testing.assert_close(after[lo:hi], want)
            mask = torch.ones(_rs_len(world), dtype=torch.bool)
            mask[lo:hi] = False
            torch.testing.assert_close(after[mask], before[mask])
            # output = input + rank * chunk: the value at chunk offset i is the sum of element
            # (start + r*chunk + i) over ranks
            base = torch.arange(_rs_len(world), dtype=torch.float32)[lo:hi]
            torch.testing.assert_close(after[lo:hi], world * base + 1000 * sum(range(world)))
        torch.testing.assert_close(o["avg"], torch.tensor([(world + 1) / 2]))


class _Functional(torch.nn.Module):
    """Uses a child's weight functionally (the child's own forward never runs, so its forward
    pre-hook -- where deferred gathers are normally waited for -- never fires)."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.a = torch.nn.Linear(16, 40)
        self.b = torch.nn.Linear(40, 4)

    def forward(self, x):
        return torch.nn.functional.linear(torch.tanh(self.a(x)), self.b.weight, self.b.bias)


def _lazy_worker(rank, world, port, out_dir):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from tests import lazy_collectives

    lazy_collectives.install()  # RCCL-like: gathers / reduce-scatters move data only at wait()
    dist = torch.distributed
    m = _Functional()
    opt = zero.zero_optimizer_for("adam")(_groups(m), lr=0.05, stage=2, bucket_mb=0.002,
                                          first_bucket_mb=0.0005)
    opt.attach_module(m)
    x, y = _data()
    per = x.shape[0] // world
    deferred = []
    for _ in range(STEPS):
        # the contract for parameters read outside their module's forward: wait_params() first
        # (DeepSpeed engine zero_grad / the trial controller's evaluation entry do this)
        deferred.append(len(opt._gather_pending))
        opt.wait_params()
        opt.zero_grad()
        xb, yb = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
        torch.nn.functional.mse_loss(m(xb), yb).backward()
        opt.finish_grad_sync()
        opt.step()
    opt.wait_params()
    torch.save({"params": {k: v.detach().clone() for k, v in m.state_dict().items()},
                "deferred": deferred}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_deferred_param_gather_with_functional_weight_use():
    """with overlap_param_gather the post-step all-gathers stay in flight (lazily, as on
    RCCL) and only a module's own forward pre-hook waits for them; a parent that reads a child's
    weight functionally must call wait_params() first. With that contract the 2-rank ZeRO-2 run
    equals the full-batch reference, and the gathers really were deferred after every step."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_lazy_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        outs = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    ref = _Functional()
    opt = fopt.FusedAdam(_groups(ref), lr=0.05)
    x, y = _data()
    for _ in range(STEPS):
        opt.zero_grad()
        torch.nn.functional.mse_loss(ref(x), y).backward()
        opt.step()
    for o in outs:
        assert o["deferred"][0] == 0 and all(n > 0 for n in o["deferred"][1:]), o["deferred"]
        for k, v in ref.state_dict().items():
            torch.testing.assert_close(o["params"][k], v, atol=1e-5, rtol=1e-5)
