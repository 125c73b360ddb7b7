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


def _worker(rank, world, port, stage, kind, max_norm, bucket_mb, out_dir):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    m = _model()
    cls = zero.zero_optimizer_for(kind)
    opt = cls(_groups(m), lr=0.05, stage=stage, bucket_mb=bucket_mb, first_bucket_mb=bucket_mb / 4)
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
    torch.save({"params": {k: v.detach().clone() for k, v in m.state_dict().items()},
                "opt": opt.state_dict()}, os.path.join(out_dir, f"r{rank}.pt"))
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


@pytest.mark.parametrize("stage,kind,max_norm,bucket_mb", [
    (1, "adam", 0.0, 64.0),
    (2, "adam", 0.0, 0.002),   # many small buckets: hooks fire bucket by bucket
    (2, "adamw", 0.05, 0.002),  # global-norm clipping across shards
    (2, "sgd", 0.0, 0.001),
])
def test_zero_matches_full_batch(stage, kind, max_norm, bucket_mb):
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), stage, kind, max_norm, bucket_mb, d),
                 nprocs=world, join=True)
        ref, ref_opt = _reference(kind, max_norm)
        outs = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    for k, v in ref.state_dict().items():
        for o in outs:
            torch.testing.assert_close(o["params"][k], v, atol=1e-5, rtol=1e-5)
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
