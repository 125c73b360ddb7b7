"""Tensor parallelism (parallel/tensor.py, models/gpt2_tp.py) against the dense model on CPU/gloo:
TP=2 loss and gradients equal the dense model's (sharded grads = slices of the dense grads),
the TP-aware clip norm equals the dense norm, full_state_dict round-trips, and a DeepSpeed engine
with a ``pipe x data x model`` mpu trains dp2 x tp2 like dense dp2 (reference:
examples/deepspeed/gpt_neox/zero1.yaml model_parallel_size: 2)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from determined_clone_amd.models import gpt2
from determined_clone_amd.models.gpt2_tp import TPGPT
from determined_clone_amd.parallel import tensor as tp


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, fn, *args):
    port = _port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_entry, args=(world, port, d, fn, args), nprocs=world, join=True)


def _entry(rank, world, port, d, fn, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if torch.cuda.is_available():
        torch.cuda.set_device(0)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world, d, *args)
    finally:
        dist.destroy_process_group()


def _cfg(pos="learned"):
    return gpt2.config_for("tiny", n_layer=2, n_head=4, d_model=256, vocab_size=500,
                           max_seq_len=32, pos_emb=pos)


def _parity(rank, world, d, pos):
    torch.manual_seed(0)
    cfg = _cfg(pos)
    full = gpt2.GPT(cfg)
    grid = tp.ModelParallelGrid(model_parallel_size=world)
    m = TPGPT(cfg, grid.get_model_parallel_group()).load_from(full)
    g = torch.Generator().manual_seed(1)
    idx = torch.randint(0, cfg.vocab_size, (2, 32), generator=g)
    tgt = torch.randint(0, cfg.vocab_size, (2, 32), generator=g)
    tgt[0, :5] = -100
    _, ref = full(idx, tgt)
    ref.backward()
    _, loss = m(idx, tgt)
    loss.backward()
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-5)
    # sharded / replicated gradients vs the dense gradients
    b, fb = m.blocks[1], full.blocks[1]
    rows = b.attn.qkv_rows()
    torch.testing.assert_close(b.attn.qkv.weight.grad, fb.attn.qkv.weight.grad[rows], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(b.attn.proj.weight.grad, fb.attn.proj.weight.grad[:, b.attn.proj.col_index()],
                               rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(b.mlp.fc.bias.grad, fb.mlp.fc.bias.grad[b.mlp.fc.row_index()], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(b.mlp.proj.bias.grad, fb.mlp.proj.bias.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(b.ln2.weight.grad, fb.ln2.weight.grad, rtol=1e-4, atol=1e-6)
    s, n = m.wte.start, m.wte.per
    torch.testing.assert_close(m.wte.weight.grad, full.wte.weight.grad[s:s + n], rtol=1e-4, atol=1e-6)
    # TP-aware clip norm == dense norm
    from determined_clone_amd.ops import optim as fopt

    opt = fopt.FusedAdamW(m.parameters(), lr=1e-3)
    tp.tp_norm_setup(opt, list(m.parameters()), grid.get_model_parallel_group())
    opt.space.ensure_views()
    opt.prepare_grads(max_norm=1.0)
    dense = torch.sqrt(sum(p.grad.double().pow(2).sum() for p in full.parameters()))
    assert abs(float(opt.last_grad_norm) - float(dense)) < 1e-4 * float(dense)
    # gathered dense state dict
    sd = m.full_state_dict()
    for k, v in full.state_dict().items():
        torch.testing.assert_close(sd[k], v, msg=k)


@pytest.mark.parametrize("pos", ["learned", "rotary"])
def test_tp2_matches_dense(pos):
    _run(2, _parity, pos)


def _engine(rank, world, d):
    """dp2 x tp2 through the DeepSpeed engine (ZeRO-1, clipping) == dense dp2 (same data split)."""
    from determined_clone_amd.pytorch import deepspeed as det_ds

    torch.manual_seed(0)
    cfg = _cfg()
    full = gpt2.GPT(cfg)
    grid = tp.ModelParallelGrid(model_parallel_size=2)
    m = TPGPT(cfg, grid.get_model_parallel_group()).load_from(full)
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_clipping": 0.05,
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.1}},
          "zero_optimization": {"stage": 1}}
    eng, _, _, _ = det_ds.initialize(model=m, config=ds, mpu=grid)
    g = torch.Generator().manual_seed(7)
    data = [(torch.randint(0, cfg.vocab_size, (2, 32), generator=g),
             torch.randint(0, cfg.vocab_size, (2, 32), generator=g)) for _ in range(2)]
    norms_tp = []
    for _ in range(3):
        idx, tgt = data[grid.get_data_parallel_rank()]  # TP ranks see the same micro batch
        _, loss = eng(idx, tgt)
        eng.backward(loss)
        eng.step()
        norms_tp.append(float(eng._last_grad_norm))
    sd = m.full_state_dict()
    if rank == 0:
        torch.save(sd, os.path.join(d, "tp.pt"))
    # checkpoint round trip: one model-states file per TP rank, ZeRO shards per (dp, tp) rank
    eng.save_checkpoint(os.path.join(d, "ckpt"))
    dist.barrier()
    assert sorted(f for f in os.listdir(os.path.join(d, "ckpt", "global_step3")) if "model_states" in f) == \
        ["mp_rank_00_model_states.pt", "mp_rank_01_model_states.pt"]
    m2 = TPGPT(cfg, grid.get_model_parallel_group())
    eng3, _, _, _ = det_ds.initialize(model=m2, config=ds, mpu=grid)
    eng3.load_checkpoint(os.path.join(d, "ckpt"))
    for k, v in m2.full_state_dict().items():
        torch.testing.assert_close(v, sd[k], rtol=0, atol=0, msg=k)
    dist.barrier()
    # dense dp2 reference on ranks {0, 2} (dp ids 0 and 1 of model-parallel rank 0)
    ref_group = dist.new_group([0, 2])
    if grid.get_model_parallel_rank() == 0:
        torch.manual_seed(0)
        dense = gpt2.GPT(cfg)
        eng2, _, _, _ = det_ds.initialize(model=dense, config=ds, group=ref_group)
        norms = []
        for _ in range(3):
            idx, tgt = data[grid.get_data_parallel_rank()]
            _, loss = eng2(idx, tgt)
            eng2.backward(loss)
            eng2.step()
            norms.append(float(eng2._last_grad_norm))
        if rank == 0:
            got = torch.load(os.path.join(d, "tp.pt"), weights_only=True)
            for k, v in dense.state_dict().items():
                # Adam normalises each update (~lr = 1e-2 per step): fp32 reduction-order noise
                # on near-zero gradients shows up at ~1e-4; a wrong average / clip would be ~1e-2
                torch.testing.assert_close(got[k], v, rtol=0, atol=5e-4, msg=k)
            torch.testing.assert_close(torch.tensor(norms), torch.tensor(norms_tp), rtol=1e-4, atol=0)
    dist.barrier()


def test_engine_dp2_tp2_matches_dense_dp2():
    _run(4, _engine)


# ---------------------------------------------------------------------------- GPU: bf16 HIP path
def _gpu_tp(rank, world, d):
    """Two TP ranks on cuda:0 (gloo stages CUDA tensors through the host; RCCL needs one device
    per rank): bf16 TP loss / sharded gradients vs the dense bf16 model on the HIP kernels (fused
    linear, local-head MFMA flash attention, bias-GELU, fused LayerNorm)."""
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfg = gpt2.config_for("tiny", n_layer=2, n_head=4, d_model=256, vocab_size=1000, max_seq_len=128)
    full = gpt2.cast_for_mi355x(gpt2.GPT(cfg)).to(dev)
    grid = tp.ModelParallelGrid(model_parallel_size=world)
    m = gpt2.cast_for_mi355x(TPGPT(cfg, grid.get_model_parallel_group())).to(dev).load_from(full)
    g = torch.Generator().manual_seed(1)
    idx = torch.randint(0, cfg.vocab_size, (2, 128), generator=g).to(dev)
    _, ref = full(idx, idx)
    ref.backward()
    _, loss = m(idx, idx)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - ref.item()) < 2e-2 * abs(ref.item()), (loss.item(), ref.item())
    b, fb = m.blocks[0], full.blocks[0]
    for got, want in ((b.attn.qkv.weight.grad, fb.attn.qkv.weight.grad[b.attn.qkv_rows().to(dev)]),
                      (b.mlp.proj.weight.grad, fb.mlp.proj.weight.grad[:, b.mlp.proj.col_index().to(dev)]),
                      (b.ln1.weight.grad, fb.ln1.weight.grad)):
        err = (got.float() - want.float()).norm().item()
        assert err <= 5e-2 * want.float().norm().item() + 1e-6, err


@pytest.mark.gpu
def test_tp2_bf16_hip_path_matches_dense():
    _run(2, _gpu_tp)


# ---------------------------------------------------------------------------- pipe x tensor
def _pipe_tp(rank, world, d):
    """pipe 2 x model 2 (the reference gpt_neox zero1.yaml layout): the 1F1B pipeline of
    tensor-parallel stages reproduces the dense model's loss and clip norm, and checkpoints per
    (stage, TP rank)."""
    from determined_clone_amd.models import gpt2_tp
    from determined_clone_amd.pytorch import deepspeed as det_ds

    torch.manual_seed(0)
    cfg = _cfg()
    full = gpt2.GPT(cfg)
    grid = tp.ModelParallelGrid(model_parallel_size=2, pipe_parallel_size=2)
    mod = det_ds.PipelineModule(gpt2_tp.pipeline_specs_tp(cfg, grid.mp_group), num_stages=2,
                                loss_fn=gpt2_tp.PipelineLossTP(cfg, grid.mp_group), grid=grid)
    gpt2_tp.load_pipeline_from(mod, full)
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2,
          "gradient_clipping": 1e-3, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
          "zero_optimization": {"stage": 1}}
    eng, _, _, _ = det_ds.initialize(model=mod, config=ds)
    g = torch.Generator().manual_seed(5)
    micro = [(torch.randint(0, cfg.vocab_size, (2, 32), generator=g),
              torch.randint(0, cfg.vocab_size, (2, 32), generator=g)) for _ in range(2)]
    loss = eng.train_batch(iter(micro))
    ref = sum(full(x, y)[1] for x, y in micro) / 2
    ref.backward()
    torch.testing.assert_close(loss.float(), ref.detach(), rtol=1e-5, atol=1e-5)
    dense_norm = float(torch.sqrt(sum(p.grad.double().pow(2).sum() for p in full.parameters())))
    assert abs(float(eng._last_grad_norm) - dense_norm) < 1e-4 * dense_norm, (float(eng._last_grad_norm), dense_norm)
    eng.save_checkpoint(os.path.join(d, "ck"))
    dist.barrier()
    names = sorted(os.listdir(os.path.join(d, "ck", "global_step1")))
    assert "layer_00-model_00-model_states.pt" in names and "layer_00-model_01-model_states.pt" in names
    assert "pipe_stage_01_dp_00_mp_01_optim_states.pt" in names


def test_pipe2_tp2_matches_dense():
    _run(4, _pipe_tp)


def _z3_refused(rank, world, d):
    from determined_clone_amd.pytorch import deepspeed as det_ds

    grid = tp.ModelParallelGrid(model_parallel_size=2)
    m = TPGPT(_cfg(), grid.get_model_parallel_group())
    with pytest.raises(ValueError, match="ZeRO stages 0-2"):
        det_ds.initialize(model=m, mpu=grid, config={
            "train_micro_batch_size_per_gpu": 1, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
            "zero_optimization": {"stage": 3}})


def test_tp_refuses_zero3():
    _run(2, _z3_refused)
