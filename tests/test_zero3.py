"""ZeRO stage 3 (parallel/zero3.py via the DeepSpeed-style engine) on CPU.

Parameters partitioned per module unit, gathered on use, gradients reduce-scattered per unit:
training must equal the unpartitioned (stage 0) engine -- single process, and 2 gloo ranks vs one
process on the full batch -- including gradient accumulation, clipping (shard norms all-reduced)
and per-group weight decay; checkpoints hold consolidated weights that reload into stage 0 or
stage 3. Reference: DeepSpeed ``zero_optimization.stage: 3`` configs
(`examples/hf_trainer_api/hf_language_modeling/ds_configs/ds_config_stage_3.json`)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from determined_clone_amd.models import gpt2
from determined_clone_amd.pytorch import deepspeed as det_ds

CFG = {
    "train_micro_batch_size_per_gpu": 4,
    "gradient_accumulation_steps": 2,
    "optimizer": {"type": "AdamW", "params": {"lr": 3e-3, "weight_decay": 0.05}},
    "gradient_clipping": 0.1,
}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(step: int, micro: int, n: int = 4):
    g = torch.Generator().manual_seed(100 * step + micro)
    t = torch.randint(0, 512, (n, 33), generator=g)
    return t[:, :-1], t[:, 1:]


def _engine(stage: int, micro: int = 4, grouped: bool = True):
    torch.manual_seed(0)
    model = gpt2.gpt2("tiny", n_layer=2)
    params = model.parameters()
    if grouped:  # no weight decay on biases / norms (DeepSpeed-style param groups)
        decay = [p for n, p in model.named_parameters() if p.dim() >= 2]
        no_decay = [p for n, p in model.named_parameters() if p.dim() < 2]
        params = [{"params": decay}, {"params": no_decay, "weight_decay": 0.0}]
    cfg = dict(CFG, zero_optimization={"stage": stage}, train_micro_batch_size_per_gpu=micro)
    eng, _, _, _ = det_ds.initialize(model=model, model_parameters=params, config=cfg)
    return eng


def _train(eng, steps=3, rank=0, world=1, gb=4):
    n = gb // world
    losses = []
    for step in range(steps):
        for micro in range(2):
            x, y = _data(step, micro, gb)
            x, y = x[rank * n:(rank + 1) * n], y[rank * n:(rank + 1) * n]
            _, loss = eng(x, y)
            eng.backward(loss)
            eng.step()
            losses.append(float(loss.detach()))
    return losses


def test_stage3_single_process_matches_stage0():
    ref = _engine(0)
    ref_losses = _train(ref)
    eng = _engine(3)
    losses = _train(eng)
    assert losses == pytest.approx(ref_losses, rel=1e-5)
    want = ref.module_state_dict()
    got = eng.module_state_dict()
    for k, v in want.items():
        torch.testing.assert_close(got[k], v, rtol=1e-5, atol=1e-6, msg=k)
    # block units are released between steps (only shards persist)
    z3 = eng._z3
    assert any(not u.root for u in z3.units)
    assert all(u.full.untyped_storage().size() == 0 for u in z3.units)
    # eval under no_grad gathers and releases too
    with torch.no_grad():
        _, l_eval = eng(*_data(9, 0))
    with torch.no_grad():
        _, l_ref = ref(*_data(9, 0))
    torch.testing.assert_close(l_eval, l_ref, rtol=1e-5, atol=1e-6)
    assert all(u.full.untyped_storage().size() == 0 for u in z3.units)


def _worker(rank: int, world: int, port: int, out: str, gb: int = 4, lazy: bool = False) -> None:
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    if lazy:  # RCCL-like async collectives: data moves only at wait() (tests/lazy_collectives.py)
        from tests import lazy_collectives

        lazy_collectives.install()
    eng = _engine(3, micro=gb // world)
    shard = sum(u.shard_numel for u in eng._z3.units)
    full = sum(u.padded for u in eng._z3.units)
    assert shard * world == full
    losses = _train(eng, rank=rank, world=world, gb=gb)
    eng.save_checkpoint(out, tag="t")
    sd = eng.module_state_dict()
    # resume from the checkpoint in a fresh stage-3 engine and take one more step
    eng2 = _engine(3, micro=gb // world)
    eng2.load_checkpoint(out, tag="t")
    sd2 = eng2.module_state_dict()
    for k in sd:
        assert torch.equal(sd[k], sd2[k]), k
    more = _train(eng, steps=1, rank=rank, world=world, gb=gb)
    more2 = _train(eng2, steps=1, rank=rank, world=world, gb=gb)
    assert more2 == more
    sd_more = eng2.module_state_dict()
    if rank == 0:
        torch.save({"sd": sd, "losses": losses, "sd_more": sd_more, "more": more},
                   os.path.join(out, "final.pt"))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world,lazy", [(2, False), (8, False), (2, True), (4, True)])
def test_stage3_multi_rank_matches_single_process(tmp_path, world, lazy):
    """2 ranks, and the driver's 8-rank layout (per-unit shards padded to 8, 8
    reduce-scatters / all-gathers per unit) against one process on the full batch; ``lazy``: the
    per-unit gathers and reduce-scatters complete only when waited for (RCCL semantics)."""
    gb = 4 if world == 2 else 8
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), gb, lazy), nprocs=world, join=True)
    res = torch.load(tmp_path / "final.pt", weights_only=True)
    ref = _engine(0, micro=gb)
    _train(ref, gb=gb)
    for k, v in ref.module_state_dict().items():
        torch.testing.assert_close(res["sd"][k], v, rtol=1e-4, atol=2e-5, msg=k)
    # resume the 2-rank checkpoint on ONE rank: the optimizer shards are re-partitioned (not
    # reset), so the next step equals the 2-rank resumed run's next step
    eng1 = _engine(3, micro=gb)
    eng1.load_checkpoint(tmp_path, tag="t")
    _train(eng1, steps=1, gb=gb)  # full batch on one rank == the per-rank slices
    for k, v in res["sd_more"].items():
        torch.testing.assert_close(eng1.module_state_dict()[k], v, rtol=1e-4, atol=2e-5, msg=k)
    # consolidated checkpoint weights load into an unpartitioned engine
    eng0 = _engine(0, micro=gb)
    eng0.load_checkpoint(tmp_path, tag="t", load_optimizer_states=False)
    for k, v in ref.module_state_dict().items():
        torch.testing.assert_close(eng0.module_state_dict()[k], v, rtol=1e-4, atol=2e-5, msg=k)


@pytest.mark.gpu
def test_stage3_bf16_gpu_matches_stage0():
    """GPU path: bf16 GPT with the fused HIP kernels accumulating straight into the gathered
    units' gradient views; fused AdamW on the shards."""
    def build(stage):
        torch.manual_seed(0)
        model = gpt2.gpt2("tiny", n_layer=2)
        # SGD: Adam turns bf16 rounding noise on exactly-zero-gradient parameters (the key bias
        # of softmax attention) into O(lr) updates, hiding real differences
        cfg = dict(CFG, zero_optimization={"stage": stage}, bf16={"enabled": True},
                   optimizer={"type": "SGD", "params": {"lr": 0.05, "momentum": 0.9}})
        return det_ds.initialize(model=model, config=cfg)[0]

    ref, eng = build(0), build(3)
    assert eng.device.type == "cuda"
    init = {k: v.float().cpu() for k, v in ref.module_state_dict().items()}
    for e in (ref, eng):
        for step in range(3):
            for micro in range(2):
                x, y = _data(step, micro)
                _, loss = e(x.cuda(), y.cuda())
                e.backward(loss)
                e.step()
    want, got = ref.module_state_dict(), eng.module_state_dict()
    for k in want:
        upd = (want[k].float().cpu() - init[k]).norm().item()
        err = (got[k].float().cpu() - want[k].float().cpu()).norm().item()
        assert err <= 0.05 * upd + 1e-3, f"{k}: {err:.3e} vs update {upd:.3e}"
    assert all(u.full.untyped_storage().size() == 0 for u in eng._z3.units)


def test_stage3_deepspeed_trial_checkpoint_resume(tmp_path):
    """DeepSpeedTrial on a stage-3 engine: train 4, checkpoint, resume to 6 == uninterrupted 6."""
    from determined_clone_amd import pytorch
    from determined_clone_amd.common.storage import SharedFSStorageManager
    from tests.test_deepspeed_trial import GPTTrial

    hp = {"ds": {"zero_optimization": {"stage": 3}}}

    def fit(d, n, latest=None):
        with det_ds.init(hparams=hp, exp_conf={}) as ctx:
            ctx._core.checkpoint._storage_manager = SharedFSStorageManager(str(d))
            t = GPTTrial(ctx)
            det_ds.Trainer(t, ctx).fit(max_length=pytorch.Batch(n), latest_checkpoint=latest,
                                       checkpoint_policy="none", checkpoint_period=pytorch.Batch(4))
            return t.engine

    fit(tmp_path / "a", 4)
    (ck,) = os.listdir(tmp_path / "a")
    resumed = fit(tmp_path / "a", 6, latest=ck)
    straight = fit(tmp_path / "b", 6)
    assert resumed._z3 is not None and resumed.global_steps == 6
    want = straight.module_state_dict()
    for k, v in resumed.module_state_dict().items():
        torch.testing.assert_close(v, want[k], msg=k)


def test_stage3_refuses_lamb():
    # a ZeRO-3 shard spans several parameters: LAMB's per-tensor trust ratio would be computed over
    # unrelated slices and change with world size, so stage 3 refuses it (as stages 1/2 do)
    torch.manual_seed(0)
    model = gpt2.gpt2("tiny", n_layer=1)
    cfg = dict(CFG, optimizer={"type": "Lamb", "params": {"lr": 1e-3}},
               zero_optimization={"stage": 3})
    with pytest.raises(ValueError, match="LAMB"):
        det_ds.initialize(model=model, model_parameters=model.parameters(), config=cfg)
