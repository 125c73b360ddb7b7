"""DeepSpeedTrial + native ZeRO engine on CPU (local mode, and gloo world_size 2)."""
import json
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from determined_clone_amd.common.storage import SharedFSStorageManager
from determined_clone_amd.models import gpt2
from determined_clone_amd.pytorch import deepspeed as det_ds
from determined_clone_amd import pytorch


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class TokenDataset(torch.utils.data.Dataset):
    def __init__(self, n=64, seq=32, vocab=512):
        g = torch.Generator().manual_seed(0)
        self.x = torch.randint(0, vocab, (n, seq + 1), generator=g)

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return self.x[i, :-1], self.x[i, 1:]


DS_CONFIG = {
    "train_micro_batch_size_per_gpu": 4,
    "gradient_accumulation_steps": 2,
    "optimizer": {"type": "Adam", "params": {"lr": 3e-3, "weight_decay": 0.01}},
    "scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0, "warmup_max_lr": 3e-3,
                                                   "warmup_num_steps": 4}},
    "gradient_clipping": 1.0,
    "zero_optimization": {"stage": 0},
}


class GPTTrial(det_ds.DeepSpeedTrial):
    def __init__(self, context):
        self.context = context
        torch.manual_seed(0)
        model = gpt2.gpt2("tiny", n_layer=1)
        cfg = det_ds.overwrite_deepspeed_config(DS_CONFIG, context.get_hparams().get("ds", {}))
        engine, _, _, _ = det_ds.initialize(model=model, config=cfg)
        self.engine = context.wrap_model_engine(engine)

    def train_batch(self, it, epoch_idx, batch_idx):
        x, y = self.context.to_device(next(it))
        _, loss = self.engine(x, y)
        self.engine.backward(loss)
        self.engine.step()
        return {"loss": loss}

    def evaluate_batch(self, it, batch_idx):
        x, y = self.context.to_device(next(it))
        _, loss = self.engine(x, y)
        return {"val_loss": loss}

    def build_training_data_loader(self):
        return pytorch.DataLoader(TokenDataset(), batch_size=self.context.train_micro_batch_size_per_gpu)

    def build_validation_data_loader(self):
        return pytorch.DataLoader(TokenDataset(16), batch_size=4)


def _fit(tmp_path, hparams, **kw):
    with det_ds.init(hparams=hparams, exp_conf={}) as ctx:
        ctx._core.checkpoint._storage_manager = SharedFSStorageManager(str(tmp_path / "ckpt"))
        trial = GPTTrial(ctx)
        ctrl = det_ds.Trainer(trial, ctx).fit(**kw)
        return trial, ctrl


def test_local_deepspeed_trial_trains_validates_checkpoints(tmp_path):
    trial, ctrl = _fit(tmp_path, {}, max_length=pytorch.Batch(6), checkpoint_policy="none",
                       validation_period=pytorch.Batch(3), checkpoint_period=pytorch.Batch(6))
    eng = trial.engine
    assert eng.global_steps == 6 and eng.micro_steps == 12
    assert ctrl.state.batches_trained == 6 and ctrl.state.last_val == 6
    ckpts = os.listdir(tmp_path / "ckpt")
    assert len(ckpts) == 1
    d = tmp_path / "ckpt" / ckpts[0]
    assert (d / "det_state_dict_rank0.pth").exists()
    assert (d / "model0" / "mp_rank_00_model_states.pt").exists()
    assert json.loads((d / "load_data.json").read_text())["trial_type"] == "DeepSpeedTrial"
    # resume 6 -> 8 equals an uninterrupted run to 8
    with det_ds.init(hparams={}, exp_conf={}) as ctx:
        ctx._core.checkpoint._storage_manager = SharedFSStorageManager(str(tmp_path / "ckpt"))
        t2 = GPTTrial(ctx)
        c2 = det_ds.Trainer(t2, ctx).fit(max_length=pytorch.Batch(8), latest_checkpoint=ckpts[0],
                                         checkpoint_policy="none")
        assert c2.state.batches_trained == 8
        assert t2.engine.global_steps == 8
        assert t2.engine.lr_scheduler.last_batch_iteration == 8
    t3, _ = _fit(tmp_path / "u", {}, max_length=pytorch.Batch(8), checkpoint_policy="none")
    for k, v in t3.engine.module.state_dict().items():
        torch.testing.assert_close(t2.engine.module.state_dict()[k], v, msg=k)


def test_zero_stage2_local_matches_stage0(tmp_path):
    t0, _ = _fit(tmp_path / "a", {"ds": {"zero_optimization": {"stage": 0}}}, max_length=pytorch.Batch(4))
    t2, _ = _fit(tmp_path / "b", {"ds": {"zero_optimization": {"stage": 2}}}, max_length=pytorch.Batch(4))
    for (k, a), (_, b) in zip(t0.engine.module.state_dict().items(), t2.engine.module.state_dict().items()):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5, msg=k)


def test_config_batch_inference_and_errors():
    c = det_ds.DeepSpeedConfig({"train_batch_size": 32, "train_micro_batch_size_per_gpu": 4}, 2)
    assert c.grad_accum == 4
    c = det_ds.DeepSpeedConfig({"train_batch_size": 32, "gradient_accumulation_steps": 2}, 4)
    assert c.micro_batch == 4
    with pytest.raises(ValueError):
        det_ds.DeepSpeedConfig({"train_batch_size": 30, "train_micro_batch_size_per_gpu": 4,
                                "gradient_accumulation_steps": 2}, 2)
    assert det_ds.DeepSpeedConfig({"train_batch_size": 8, "zero_optimization": {"stage": 3}}, 1).zero_stage == 3
    with pytest.raises(ValueError):
        det_ds.DeepSpeedConfig({"train_batch_size": 8, "zero_optimization": {"stage": 4}}, 1)


def test_warmup_schedulers():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1.0)
    s = det_ds.WarmupDecayLR(opt, total_num_steps=10, warmup_max_lr=1.0, warmup_num_steps=4,
                             warmup_type="linear")
    lrs = []
    for _ in range(10):
        lrs.append(opt.param_groups[0]["lr"])
        s.step()
    assert lrs[0] == 0.0 and abs(lrs[2] - 0.5) < 1e-9 and abs(lrs[4] - 1.0) < 1e-9
    assert lrs[-1] < lrs[5]


# ------------------------------------------------------------------ multi-process engine equivalence
def _engine_worker(rank, world, port, stage, out, overlap=False, gmb=4):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = gpt2.gpt2("tiny", n_layer=1)
    mb = gmb // world
    cfg = dict(DS_CONFIG, zero_optimization={"stage": stage, "overlap_param_gather": overlap},
               train_micro_batch_size_per_gpu=mb)
    eng, _, _, _ = det_ds.initialize(model=model, config=cfg)
    ds = TokenDataset(64)
    for step in range(3):
        for micro in range(2):
            base = (step * 2 + micro) * gmb
            idx = list(range(base + rank * mb, base + rank * mb + mb))
            x = torch.stack([ds[i][0] for i in idx])
            y = torch.stack([ds[i][1] for i in idx])
            _, loss = eng(x, y)
            eng.backward(loss)
            eng.step()
    eng.save_checkpoint(out, tag="t")
    if rank == 0:
        torch.save(eng.module.state_dict(), os.path.join(out, "final.pt"))
    torch.distributed.destroy_process_group()


def _single_reference(out, gmb=4):
    torch.manual_seed(0)
    model = gpt2.gpt2("tiny", n_layer=1)
    cfg = dict(DS_CONFIG, train_micro_batch_size_per_gpu=gmb)
    eng, _, _, _ = det_ds.initialize(model=model, config=cfg)
    ds = TokenDataset(64)
    for step in range(3):
        for micro in range(2):
            base = (step * 2 + micro) * gmb
            x = torch.stack([ds[i][0] for i in range(base, base + gmb)])
            y = torch.stack([ds[i][1] for i in range(base, base + gmb)])
            _, loss = eng(x, y)
            eng.backward(loss)
            eng.step()
    return eng


@pytest.mark.parametrize("world,stage,overlap", [(2, 1, False), (2, 2, False), (2, 2, True), (8, 2, True)])
def test_engine_zero_multi_rank_matches_single_process(world, stage, overlap):
    """overlap=True: the post-step parameter all-gathers stay in flight into the next forward
    (zero_optimization.overlap_param_gather) and are waited for module by module; world 8 is the
    driver's GPT-2 ZeRO-2 layout (8 pending gathers, shards padded to 8)."""
    gmb = 4 if world == 2 else 8
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_engine_worker, args=(world, _free_port(), stage, d, overlap, gmb), nprocs=world, join=True)
        final = torch.load(os.path.join(d, "final.pt"), weights_only=True)
        ref = _single_reference(d + "/ref", gmb)
        for k, v in ref.module.state_dict().items():
            torch.testing.assert_close(final[k], v, atol=2e-5, rtol=1e-4, msg=k)
        # re-shard: a single-process stage-2 engine loads the 2-rank checkpoint
        torch.manual_seed(1)
        eng1, _, _, _ = det_ds.initialize(model=gpt2.gpt2("tiny", n_layer=1),
                                          config=dict(DS_CONFIG, zero_optimization={"stage": 2},
                                                      train_micro_batch_size_per_gpu=8))
        eng1.load_checkpoint(d, tag="t")
        assert eng1.global_steps == 3
        for k, v in ref.module.state_dict().items():
            torch.testing.assert_close(eng1.module.state_dict()[k], v, atol=2e-5, rtol=1e-4)
        full = eng1.optimizer.consolidated_state_dict()
        rsd = ref.optimizer.state_dict()
        for i, st in rsd["state"].items():
            torch.testing.assert_close(full["state"][i]["exp_avg"], st["exp_avg"], atol=1e-6, rtol=1e-3)


@pytest.mark.gpu
def test_engine_grads_readable_right_after_backward_gpu():
    """Weight gradients run on a side stream (ops/_grad.py); ``engine.backward`` joins it, so a
    reader of ``.grad`` between ``backward`` and ``step`` (custom clipping, logging) sees the
    finished gradient: same values as with the side stream off (``DCA_WGRAD_STREAM=0``)."""
    from determined_clone_amd.ops import _grad

    def grads(side: bool):
        old = _grad.SIDE_STREAM
        _grad.SIDE_STREAM = side
        try:
            torch.manual_seed(0)
            model = gpt2.cast_for_mi355x(gpt2.gpt2("tiny", n_layer=2, max_seq_len=256)).cuda()
            cfg = dict(DS_CONFIG, gradient_accumulation_steps=1, gradient_clipping=0.0)
            eng, _, _, _ = det_ds.initialize(model=model, config=cfg)
            g = torch.Generator(device="cpu").manual_seed(1)
            x = torch.randint(0, 512, (4, 256), generator=g).cuda()
            _, loss = eng(x, x)
            eng.backward(loss)
            # read on the current stream immediately (no synchronize in between)
            out = [p.grad.float().clone() for p in eng.module.parameters() if p.grad is not None]
            assert not _grad.pending()
            torch.cuda.synchronize()
            return out
        finally:
            _grad.SIDE_STREAM = old

    ref, got = grads(False), grads(True)
    assert len(ref) == len(got) and len(ref) > 0
    for a, b in zip(ref, got):
        torch.testing.assert_close(b, a, rtol=1e-3, atol=1e-5)
