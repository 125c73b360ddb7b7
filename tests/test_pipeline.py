"""Pipeline parallelism (parallel/pipeline.py + deepspeed/_pipe.py) on CPU with gloo.

A GPT (tied embedding / LM head) split into 2 or 4 stages, optionally x2 data parallel, trained
with the 1F1B schedule must match the same layers trained in ONE process with all micro-batches
(same per-layer seeds): losses, every layer's parameters, gradient clipping across stages with
the tied weight counted once, ZeRO-1 inside a stage, activation checkpointing; a per-layer
checkpoint written by the 2-stage run reloads into the 1-stage module. Reference behaviour:
DeepSpeed PipelineEngine as driven by `harness/determined/pytorch/deepspeed/_deepspeed_trial.py`
(``use_pipeline_parallel``) and `examples/deepspeed/gpt_neox` (``pipe_parallel_size: 2``)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from determined_clone_amd.models import gpt2
from determined_clone_amd.parallel import pipeline

M = 4  # micro-batches per train_batch
MB = 2  # micro-batch size
SEQ = 16
STEPS = 3


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg():
    return gpt2.config_for("tiny", n_layer=4, max_seq_len=SEQ, vocab_size=256)


def _ds_config(gas: int, zero: int = 0, clip: float = 0.05):
    return {"train_micro_batch_size_per_gpu": MB, "gradient_accumulation_steps": gas,
            "optimizer": {"type": "AdamW", "params": {"lr": 3e-3, "weight_decay": 0.01}},
            "gradient_clipping": clip, "zero_optimization": {"stage": zero}}


def _micro_batches(step: int, n: int):
    g = torch.Generator().manual_seed(1000 + step)
    out = []
    for _ in range(n):
        t = torch.randint(0, 256, (MB, SEQ + 1), generator=g)
        out.append((t[:, :-1], t[:, 1:]))
    return out


def _module(stages: int, ckpt: int = 0):
    return pipeline.PipelineModule(gpt2.pipeline_specs(_cfg()), num_stages=stages,
                                   loss_fn=gpt2.pipeline_loss, seed_layers=True,
                                   activation_checkpoint_interval=ckpt)


def _worker(rank: int, world: int, port: int, stages: int, zero: int, ckpt: int, out: str) -> None:
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from determined_clone_amd.pytorch import deepspeed as det_ds

    mod = _module(stages, ckpt)
    engine, _, _, _ = det_ds.initialize(model=mod, config=_ds_config(M, zero))
    assert isinstance(engine, det_ds.PipelineEngine)
    dp, D = engine.grid.data_parallel_id, engine.grid.data_parallel_size
    losses = []
    for step in range(STEPS):
        mine = _micro_batches(step, M * D)[dp * M:(dp + 1) * M]
        it = iter(mine) if (engine.is_first or engine.is_last) else None
        losses.append(float(engine.train_batch(it)))
    ev = float(engine.eval_batch(iter(_micro_batches(99, M)) if (engine.is_first or engine.is_last)
                                 else None))
    engine.save_checkpoint(os.path.join(out, "ckpt"))
    torch.save({"losses": losses, "eval": ev, "layers": mod.layer_state_dicts(),
                "tied_head": [i for i, s in enumerate(mod.specs)
                              if isinstance(s, pipeline.TiedLayerSpec)][-1]},
               os.path.join(out, f"r{rank}.pt"))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def _reference(D: int):
    from determined_clone_amd.pytorch import deepspeed as det_ds

    mod = _module(1)
    engine, _, _, _ = det_ds.initialize(model=mod, config=_ds_config(M * D))
    losses = [float(engine.train_batch(iter(_micro_batches(step, M * D)))) for step in range(STEPS)]
    ev = float(engine.eval_batch(iter(_micro_batches(99, M)), num_micro_batches=M))
    return mod, losses, ev


@pytest.mark.parametrize("world,stages,zero,ckpt", [(2, 2, 0, 0), (4, 2, 1, 2), (4, 4, 0, 0)])
def test_pipeline_matches_single_process(tmp_path, world, stages, zero, ckpt):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, stages, zero, ckpt, str(tmp_path)), nprocs=world, join=True)
    D = world // stages
    ref_mod, ref_losses, ref_eval = _reference(D)
    ref_layers = ref_mod.layer_state_dicts()
    seen = set()
    for r in range(world):
        res = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert res["losses"] == pytest.approx(ref_losses, rel=1e-4, abs=1e-5)
        if D == 1:  # eval averages over data-parallel ranks, each with its own micro-batches
            assert res["eval"] == pytest.approx(ref_eval, rel=1e-4)
        for idx, sd in res["layers"].items():
            keys = ["wte.weight"] if idx == res["tied_head"] else sd.keys()
            for k in keys:
                torch.testing.assert_close(sd[k], ref_layers[idx][k], rtol=2e-4, atol=2e-5,
                                           msg=f"layer {idx} {k}")
            seen.add(idx)
    assert seen == set(range(len(ref_mod.specs)))
    assert ref_losses[-1] < ref_losses[0]

    # the 2/4-stage per-layer checkpoint reloads into a 1-stage module
    from determined_clone_amd.pytorch import deepspeed as det_ds

    mod = _module(1)
    engine, _, _, _ = det_ds.initialize(model=mod, config=_ds_config(M * D))
    engine.load_checkpoint(tmp_path / "ckpt")
    assert engine.global_steps == STEPS
    for idx, sd in mod.layer_state_dicts().items():
        for k, v in sd.items():
            if idx == len(mod.specs) - 1 and k != "wte.weight":
                continue
            torch.testing.assert_close(v, ref_layers[idx][k], rtol=2e-4, atol=2e-5)


def test_partitioning():
    assert pipeline.partition_uniform(7, 3) == [0, 3, 5, 7]
    assert pipeline.partition_balanced([1, 1, 1, 1], 2) == [0, 2, 4]
    assert pipeline.partition_balanced([10, 1, 1, 1, 1, 10], 3) == [0, 1, 5, 6]
    specs = gpt2.pipeline_specs(_cfg())
    mod = pipeline.PipelineModule(specs, num_stages=1, loss_fn=gpt2.pipeline_loss)
    assert mod.parts == [0, len(specs)]
    m3 = pipeline.PipelineModule.__new__(pipeline.PipelineModule)
    torch.nn.Module.__init__(m3)
    m3.specs, m3.num_stages = specs, 3
    parts = m3._partition("parameters")
    # blocks (~200k params) dominate this small vocabulary's embedding / tied head (~35k):
    # embed+block | block+block | block+ln+head
    assert parts == [0, 2, 4, len(specs)]
    m3.num_stages = 2
    assert m3._partition("type:BlockPipe") == [0, 3, len(specs)]  # 2 blocks per stage
    assert m3._partition("uniform") == [0, 4, len(specs)]
    with pytest.raises(ValueError):
        pipeline.PipelineModule([torch.nn.Linear(2, 2)], num_stages=2)


def test_single_stage_module_matches_gpt():
    """The pipe layer list computes exactly GPT.forward's loss (same weights)."""
    cfg = _cfg()
    ref = gpt2.GPT(cfg)
    mod = pipeline.PipelineModule(gpt2.pipeline_specs(cfg), num_stages=1, loss_fn=gpt2.pipeline_loss)
    sd = ref.state_dict()
    n = cfg.n_layer
    mod.tied_modules["embed"].wte.weight.data.copy_(sd["wte.weight"])
    mod.tied_modules["embed"].wpe.weight.data.copy_(sd["wpe.weight"])
    for i in range(n):
        blk = {k[len(f"blocks.{i}."):]: v for k, v in sd.items() if k.startswith(f"blocks.{i}.")}
        getattr(mod, str(1 + i)).load_state_dict(blk)
    getattr(mod, str(1 + n)).ln_f.load_state_dict({"weight": sd["ln_f.weight"], "bias": sd["ln_f.bias"]})
    x, y = _micro_batches(0, 1)[0]
    _, want = ref(x, y)
    got = mod.loss_fn(mod(x), y)
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6)


# ---------------------------------------------------------------------------------- DeepSpeedTrial
class _Tokens(torch.utils.data.Dataset):
    def __init__(self, n: int) -> None:
        self.x = torch.randint(0, 256, (n, SEQ + 1), generator=torch.Generator().manual_seed(n))

    def __len__(self) -> int:
        return len(self.x)

    def __getitem__(self, i: int):
        return self.x[i, :-1], self.x[i, 1:]


def _trial_cls():
    from determined_clone_amd import pytorch
    from determined_clone_amd.pytorch import deepspeed as det_ds

    class PipeTrial(det_ds.DeepSpeedTrial):
        def __init__(self, context):
            self.context = context
            engine, _, _, _ = det_ds.initialize(model=_module(2), config=_ds_config(M))
            self.engine = context.wrap_model_engine(engine)

        def train_batch(self, it, epoch_idx, batch_idx):
            return {"loss": self.engine.train_batch(it)}

        def evaluate_batch(self, it, batch_idx):
            return {"val_loss": self.engine.eval_batch(it)}

        def build_training_data_loader(self):
            return pytorch.DataLoader(_Tokens(64), batch_size=self.context.train_micro_batch_size_per_gpu)

        def build_validation_data_loader(self):
            return pytorch.DataLoader(_Tokens(12), batch_size=MB)

    return PipeTrial


def _trial_worker(rank: int, world: int, port: int, out: str) -> None:
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world)})
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from determined_clone_amd import core, pytorch
    from determined_clone_amd.common.storage import SharedFSStorageManager
    from determined_clone_amd.pytorch import deepspeed as det_ds

    dist_ctx = core.DistributedContext.from_torch_distributed()
    with det_ds.init(hparams={}, exp_conf={}, distributed=dist_ctx) as ctx:
        ctx._core.checkpoint._storage_manager = SharedFSStorageManager(os.path.join(out, "ckpt"))
        trial = _trial_cls()(ctx)
        assert ctx.use_pipeline_parallel and ctx._mpu.data_parallel_world_size == 1
        assert ctx._mpu.should_build_data_loader  # 2 stages: both ends read data
        ctrl = det_ds.Trainer(trial, ctx).fit(max_length=pytorch.Batch(4), checkpoint_policy="none",
                                              validation_period=pytorch.Batch(2),
                                              checkpoint_period=pytorch.Batch(4))
        torch.save({"batches": ctrl.state.batches_trained, "last_val": ctrl.state.last_val,
                    "steps": trial.engine.global_steps, "micro": trial.engine.micro_steps,
                    "nval": ctrl.num_validation_batches},
                   os.path.join(out, f"t{rank}.pt"))
    torch.distributed.barrier()
    (ck,) = os.listdir(os.path.join(out, "ckpt"))
    with det_ds.init(hparams={}, exp_conf={}, distributed=dist_ctx) as ctx:  # resume 4 -> 6
        ctx._core.checkpoint._storage_manager = SharedFSStorageManager(os.path.join(out, "ckpt"))
        trial = _trial_cls()(ctx)
        ctrl = det_ds.Trainer(trial, ctx).fit(max_length=pytorch.Batch(6), latest_checkpoint=ck,
                                              checkpoint_policy="none")
        assert ctrl.state.batches_trained == 6 and trial.engine.global_steps == 6
    torch.distributed.destroy_process_group()


def test_deepspeed_trial_with_pipeline_engine(tmp_path):
    mp.spawn(_trial_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        res = torch.load(tmp_path / f"t{r}.pt", weights_only=True)
        assert res == {"batches": 4, "last_val": 4, "steps": 4, "micro": 4 * M, "nval": 12 // MB // M}
    n_layers = len(gpt2.pipeline_specs(_cfg()))
    for ck in os.listdir(tmp_path / "ckpt"):  # step 4, and step 6 written by the resumed run
        files = set(os.listdir(tmp_path / "ckpt" / ck / "model0"))
        assert {f"layer_{i:02d}-model_states.pt" for i in range(n_layers)} <= files
        assert "mp_rank_00_model_states.pt" in files
