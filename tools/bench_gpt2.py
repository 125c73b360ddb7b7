"""GPT-2-medium DeepSpeedTrial ZeRO-2 training throughput (tokens/sec) on MI355X.

BASELINE.json config "GPT-2-medium DeepSpeedTrial ZeRO-2 on 8xMI355X (native ZeRO partition on
RCCL)". Times the real DeepSpeedTrial path: ``det_ds.Trainer.fit`` -> DeepSpeedTrialController ->
``train_batch(iterator)`` -> engine forward / backward (bucketed reduce-scatter overlapped with
backward) / step (fused HIP AdamW on the owned shard + all-gather). GPT-2-medium (24 x 1024, 16
heads, 50304 padded vocab, 355M params), seq 1024, bf16 weights/activations with fp32 master and
moments, random-init weights, synthetic tokens resident in HBM. Weak scaling.

Usage: python tools/bench_gpt2.py [--micro 32 --gas 1 --steps 20 --warmup 5 --stage 2]
(torch.distributed.run for N>1). Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DCA_GEMM_TUNED", "1")  # replay the shipped tuned GEMMs (ops/gemm_tuning.py)

import torch  # noqa: E402

from determined_clone_amd import pytorch  # noqa: E402
from determined_clone_amd.models import gpt2  # noqa: E402
from determined_clone_amd.pytorch import deepspeed as det_ds  # noqa: E402


class GPT2BenchTrial(det_ds.DeepSpeedTrial):
    def __init__(self, context):
        self.context = context
        hp = context.get_hparams()
        self.warmup, self.steps = int(hp["warmup"]), int(hp["steps"])
        self.seq = int(hp["seq"])
        torch.manual_seed(0)
        self.model = gpt2.gpt2(hp["model"], max_seq_len=self.seq)
        ds_config = {
            "train_micro_batch_size_per_gpu": int(hp["micro"]),
            "gradient_accumulation_steps": int(hp["gas"]),
            "optimizer": {"type": "AdamW", "params": {"lr": 1.5e-4, "betas": [0.9, 0.95],
                                                       "eps": 1e-8, "weight_decay": 0.1}},
            "scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0,
                                                          "warmup_max_lr": 1.5e-4,
                                                          "warmup_num_steps": 100}},
            "gradient_clipping": 1.0,
            "bf16": {"enabled": True},
            "zero_optimization": {"stage": int(hp["stage"]), "overlap_comm": True,
                                  "overlap_param_gather": True,
                                  "reduce_bucket_size": int(hp.get("bucket_elems", 5e7))},
        }
        engine, _, _, _ = det_ds.initialize(model=self.model, config=ds_config)
        self.engine = context.wrap_model_engine(engine)
        self.t0 = self.t1 = None

    def _mark(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if self.context.distributed.size > 1:
            torch.distributed.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        return time.perf_counter()

    def train_batch(self, it, epoch_idx, batch_idx):
        if batch_idx == self.warmup and self.t0 is None:
            self.t0 = self._mark()
        x, y = next(it)
        _, loss = self.engine(x, y)
        self.engine.backward(loss)
        self.engine.step()
        if batch_idx == self.warmup + self.steps - 1 and \
                self.engine.micro_steps % self.engine.gradient_accumulation_steps() == 0:
            self.t1 = self._mark()
        return {"loss": loss}

    def evaluate_batch(self, it, batch_idx):
        x, y = next(it)
        _, loss = self.engine(x, y)
        return {"val_loss": loss}

    def _data(self, n, length=100000):
        dev = self.context.device
        g = torch.Generator().manual_seed(1 + self.context.distributed.rank)
        V = self.model.cfg.vocab_size
        mb = self.context.train_micro_batch_size_per_gpu
        batches = []
        for _ in range(n):
            t = torch.randint(0, V, (mb, self.seq + 1), generator=g).to(dev)
            batches.append((t[:, :-1].contiguous(), t[:, 1:].contiguous()))
        return pytorch.DataLoader(pytorch.DeviceBatchDataset(batches, length * self.context.distributed.size),
                                  batch_size=None)

    def build_training_data_loader(self):
        return self._data(4)

    def build_validation_data_loader(self):
        return self._data(1, length=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--micro", type=int, default=32,
                    help="micro batch per GPU (32: +8.5%% over 16, profiles/round2_gpt2_micro_batch_ab.txt)")
    ap.add_argument("--gas", type=int, default=1)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--stage", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    from determined_clone_amd.launch import ranks

    if ranks.needs_launch(a.gpus):  # --gpus N without a launcher: start the N ranks as a child
        raise SystemExit(ranks.run_as_ranks(__file__, sys.argv[1:], a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        raise SystemExit(f"bench_gpt2.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    hp = {"model": a.model, "micro": a.micro, "gas": a.gas, "seq": a.seq, "stage": a.stage,
          "warmup": a.warmup, "steps": a.steps}
    with det_ds.init(hparams=hp, exp_conf={}) as ctx:
        trial = GPT2BenchTrial(ctx)
        total = a.warmup + a.steps
        det_ds.Trainer(trial, ctx).fit(max_length=pytorch.Batch(total),
                                       reporting_period=pytorch.Batch(total), checkpoint_policy="none")
        if trial.t1 is None:
            trial.t1 = trial._mark()
        ms = (trial.t1 - trial.t0) / a.steps * 1000.0
        backend, pg_size = "none", 1
        if ctx.distributed.size > 1:
            ms = max(ctx.distributed.allgather(ms))
            backend, pg_size = str(torch.distributed.get_backend()), torch.distributed.get_world_size()
        wdt = next(p.dtype for p in trial.model.parameters())
        dtype = {torch.bfloat16: "bf16", torch.float16: "fp16", torch.float32: "fp32"}.get(wdt, str(wdt))
        where = "resident in HBM" if torch.cuda.is_available() else "in host memory (CPU run)"
        tokens = a.micro * a.gas * a.seq * world
        tps = tokens / (ms / 1000.0)
        fpt = trial.model.flops_per_token(a.seq)
        if ctx.distributed.rank == 0:
            print(json.dumps({
                "metric": f"tokens/sec {a.model} DeepSpeedTrial ZeRO-{a.stage}", "value": round(tps, 1),
                "unit": "tokens/sec", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": dtype,
                "data": f"synthetic (random tokens {where}, random-init weights)",
                "world_size": pg_size, "backend": backend,
                "tflops_per_gpu": round(tps * fpt / world / 1e12, 1),
                "config": {"model": a.model, "global_batch": a.micro * a.gas * world, "seq_len": a.seq,
                           "parallelism": f"zero{a.stage}-dp{world}", "micro_batch": a.micro,
                           "grad_accum": a.gas, "params": sum(p.numel() for p in trial.model.parameters())},
            }), flush=True)


if __name__ == "__main__":
    main()
