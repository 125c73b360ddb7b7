"""Headline benchmark: ResNet-50 PyTorchTrial training throughput (images/sec) on MI355X.

BASELINE.json metric: "images/sec ResNet-50 PyTorchTrial at 1/2/4/8 MI355X". The step that is
timed is the real PyTorchTrial path of this framework: ``pytorch.Trainer.fit`` ->
``_PyTorchTrialController`` -> ``trial.train_batch`` (forward, ``context.backward`` with bucketed
RCCL all-reduce overlapped with backward, ``context.step_optimizer`` with the fused HIP SGD) on
ResNet-50 v1.5 (random init, 25.6M params), bf16 NHWC activations, fp32 master weights, synthetic
224x224 ImageNet-shaped data resident in HBM. Weak scaling: 1024 images per GPU per step.

Usage: ``python bench.py [--gpus N --steps K --warmup W]``. With ``--gpus N > 1`` and no launcher
around it, the process starts ``torch.distributed.run --nproc-per-node N`` itself as a CHILD (never
an exec; before any GPU call) and forwards rank 0's JSON line -- the same layout the reference's
``launch/torch_distributed.py`` builds for a multi-slot trial. Under an external launcher
(RANK/LOCAL_RANK/WORLD_SIZE in the env) each process is one rank. Rank 0 prints one JSON line,
which also records the process-group size torch.distributed actually formed (``world_size``) and
its backend (``nccl`` is RCCL on ROCm).
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "images/sec ResNet-50 PyTorchTrial"
BASELINE_VALUE = None  # BASELINE.json "published" is empty


def _args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1024,
                    help="images per GPU per step (288 GB HBM: 1024 is 6%% faster than 512 and 13%% "
                         "faster than 256, profiles/round2_resnet50_batch_ab.txt, round2_resnet50_bs1024_ab.txt)")
    return ap.parse_args(argv)


def _rank_miopen_dirs() -> None:
    """Each rank gets its own writable copy of the shipped MIOpen find/perf DB and kernel cache
    (ops/miopen_db.py): the shipped files are never written, and no two ranks share one sqlite DB.
    The library GEMMs replay the shipped TunableOp results (ops/gemm_tuning.py: +5% on this step,
    profiles/round3_resnet50_gemm_tuning_ab.txt)."""
    from determined_clone_amd.ops import miopen_db

    miopen_db.use_private_copy(f"bench_rank{os.environ.get('LOCAL_RANK', '0')}")
    os.environ.setdefault("DCA_GEMM_TUNED", "1")


def _gpu_state() -> dict:
    """sclk level in use, power draw / cap and junction temperature of the visible amdgpu cards
    (sysfs; for the stderr diagnostics: a throttled or power-capped device shows here)."""
    import glob

    out = {}
    for dev in sorted(glob.glob("/sys/class/drm/card[0-9]*/device"))[:8]:
        def rd(name: str) -> str:
            try:
                with open(os.path.join(dev, name)) as f:
                    return f.read().strip()
            except OSError:
                return ""
        sclk = next((ln.split(":", 1)[1].strip().rstrip("*").strip() for ln in rd("pp_dpm_sclk").splitlines()
                     if ln.endswith("*")), "")
        hw = sorted(glob.glob(os.path.join(dev, "hwmon", "hwmon*")))
        def hwrd(name: str) -> str:
            try:
                with open(os.path.join(hw[0], name)) as f:
                    return f.read().strip()
            except (OSError, IndexError):
                return ""
        pw = hwrd("power1_average") or hwrd("power1_input")
        if not sclk and not pw:
            continue  # not an amdgpu device with power management
        card = os.path.basename(os.path.dirname(dev))
        out[card] = {"sclk": sclk, "power_w": round(int(pw) / 1e6, 1) if pw.isdigit() else None,
                     "cap_w": round(int(hwrd("power1_cap")) / 1e6, 1) if hwrd("power1_cap").isdigit() else None,
                     "temp_c": round(int(hwrd("temp1_input")) / 1e3, 1) if hwrd("temp1_input").isdigit() else None}
    return out


def _run_rank(args: argparse.Namespace) -> None:
    _rank_miopen_dirs()
    import torch
    import torch.nn.functional as F

    from determined_clone_amd import pytorch
    from determined_clone_amd.models import resnet

    class ResNet50BenchTrial(pytorch.PyTorchTrial):
        def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
            self.context = context
            hp = context.get_hparams()
            self.per_slot = context.get_per_slot_batch_size()
            self.warmup = int(hp["warmup"])
            self.steps = int(hp["steps"])
            model = resnet.to_mi355x_layout(resnet.resnet50())
            self.model = context.wrap_model(model)
            lr = 0.1 * context.get_global_batch_size() / 256
            opt = torch.optim.SGD(self.model.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5)
            self.opt = context.wrap_optimizer(opt)
            self.t0 = self.t1 = None
            self.events = []
            self.mid_state = {}

        def _mark(self) -> float:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            if self.context.distributed.size > 1:
                import torch.distributed as dist

                dist.barrier()
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            return time.perf_counter()

        def train_batch(self, batch, epoch_idx: int, batch_idx: int):
            if batch_idx == self.warmup:
                self.t0 = self._mark()
            if torch.cuda.is_available() and batch_idx >= self.warmup:
                # per-step GPU timestamps (no synchronisation) for the stderr diagnostics
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                self.events.append(ev)
            images, labels = batch
            logits = self.model(images)
            loss = F.cross_entropy(logits.float(), labels)
            self.context.backward(loss)
            self.context.step_optimizer(self.opt)
            if batch_idx == self.warmup + self.steps // 2 and torch.cuda.is_available():
                self.mid_state = _gpu_state()  # clocks / power WHILE the timed steps run (sysfs)
            if batch_idx == self.warmup + self.steps - 1:
                if torch.cuda.is_available():
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record()
                    self.events.append(ev)
                self.t1 = self._mark()
            return {"loss": loss}

        def evaluate_batch(self, batch, batch_idx: int):
            images, labels = batch
            logits = self.model(images)
            return {"val_loss": F.cross_entropy(logits.float(), labels)}

        def _data(self, n_batches: int, length: int) -> pytorch.DataLoader:
            dev = self.context.device
            g = torch.Generator(device="cpu").manual_seed(1234 + self.context.distributed.rank)
            batches = []
            for _ in range(n_batches):
                x = torch.randn(self.per_slot, 3, 224, 224, generator=g).to(dev, torch.bfloat16)
                x = x.contiguous(memory_format=torch.channels_last)
                y = torch.randint(0, 1000, (self.per_slot,), generator=g).to(dev)
                batches.append((x, y))
            # batch_size=None: each item already is a per-slot batch resident in device memory.
            ds = pytorch.DeviceBatchDataset(batches, length * self.context.distributed.size)
            return pytorch.DataLoader(ds, batch_size=None)

        def build_training_data_loader(self):
            return self._data(4, 10000)

        def build_validation_data_loader(self):
            return self._data(1, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if torch.cuda.is_available():
        # this rank's GPU first: a bare torch.cuda call would open a context on device 0 in every rank
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
        # A process that just ended on this GPU may still be returning its ~200 GB of HBM: starting
        # the bs-1024 step in the remainder makes the caching allocator free and re-map blocks every
        # step (alloc retries). Wait (bounded) for the device's memory to come back first.
        free0, total = torch.cuda.mem_get_info()
        t_wait = time.time()
        wait_s = float(os.environ.get("DCA_BENCH_MEM_WAIT_S", "60"))
        while free0 < 0.8 * total and time.time() - t_wait < wait_s:
            time.sleep(2)
            free0, total = torch.cuda.mem_get_info()
        print(json.dumps({"device_free_gb_at_start": round(free0 / 2**30, 1),
                          "device_total_gb": round(total / 2**30, 1),
                          "waited_s": round(time.time() - t_wait, 1)}), file=sys.stderr, flush=True)
        # MIOpen immediate mode (benchmark=False) picks each conv's solver from the shipped find /
        # perf DB (ops/tuned/miopen) without timing candidates: same kernels and step time as
        # per-process miopenFind, but a 12 s instead of a 4 min process at bs 1024
        # (profiles/round2_miopen_immediate_mode_ab.txt); DCA_CONV_BENCHMARK=1 runs the find
        torch.backends.cudnn.benchmark = os.environ.get("DCA_CONV_BENCHMARK", "0") == "1"
    hparams = {"global_batch_size": args.batch * world, "warmup": args.warmup, "steps": args.steps}
    # the timed step runs eagerly: train_batch's per-step timestamps must run on every step (a
    # HIP-graph replay skips the Python body); the step is GPU-bound at bs 1024 anyway
    exp_conf = {"optimizations": {"aggregation_frequency": 1, "average_training_metrics": True}}
    with pytorch.init(hparams=hparams, exp_conf=exp_conf) as ctx:
        trial = ResNet50BenchTrial(ctx)
        trainer = pytorch.Trainer(trial, ctx)
        total = args.warmup + args.steps
        trainer.fit(max_length=pytorch.Batch(total), reporting_period=pytorch.Batch(total),
                    checkpoint_policy="none")
        dt = trial.t1 - trial.t0
        ms = dt / args.steps * 1000.0
        backend, pg_size = "none", 1
        if ctx.distributed.size > 1:
            import torch.distributed as dist

            ms = max(ctx.distributed.allgather(ms))
            backend, pg_size = str(dist.get_backend()), dist.get_world_size()
        imgs = args.batch * world * args.steps / (ms * args.steps / 1000.0)
        on_gpu = trial.context.device.type == "cuda"
        if on_gpu:
            ev = trial.events
            step_ms = [round(a.elapsed_time(b), 2) for a, b in zip(ev[:-1], ev[1:])]
            ms_stats = torch.cuda.memory_stats()
            print(json.dumps({"rank": ctx.distributed.rank, "gpu_state_mid": trial.mid_state,
                              "gpu_state_end": _gpu_state()}), file=sys.stderr)
            print(json.dumps({"rank": ctx.distributed.rank, "step_ms": step_ms,
                              "max_reserved_gb": round(torch.cuda.max_memory_reserved() / 2**30, 1),
                              "alloc_retries": ms_stats.get("num_alloc_retries", 0),
                              "device_free_gb": round(torch.cuda.mem_get_info()[0] / 2**30, 1)}),
                  file=sys.stderr, flush=True)
        if ctx.distributed.rank == 0:
            # labels describe what actually ran
            conv_dtype = next(p.dtype for p in trial.model.parameters() if p.dim() == 4)
            dtype = {torch.bfloat16: "bf16", torch.float16: "fp16", torch.float32: "fp32"}.get(conv_dtype, str(conv_dtype))
            opt_name = type(trial.opt).__name__
            where = "resident in HBM" if on_gpu else "in host memory (no GPU: CPU run)"
            out = {
                "metric": METRIC, "value": round(imgs, 1), "unit": "images/sec",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None if BASELINE_VALUE is None else round(imgs / BASELINE_VALUE, 3),
                "dtype": dtype,
                "data": f"synthetic (random 224x224x3 images + labels {where}, random-init weights)",
                "device": torch.cuda.get_device_name() if on_gpu else "cpu",
                "world_size": pg_size, "backend": backend,
                # slow-mode evidence (profiles/round4_bench_slow_mode.txt): allocator retries mean the
                # step ran short of device memory (another process's HBM not yet returned)
                "diagnostics": {"alloc_retries": int(ms_stats.get("num_alloc_retries", 0)) if on_gpu else 0,
                                "device_free_gb_at_start": round(free0 / 2**30, 1) if on_gpu else None,
                                "max_reserved_gb": round(torch.cuda.max_memory_reserved() / 2**30, 1) if on_gpu else None,
                                "max_allocated_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1) if on_gpu else None,
                                # candidates timed by the convolution chooser in this process
                                # (0: every decision came from ops/tuned/conv_choices_gfx950.json)
                                "conv_chooser_timings": _conv_timings()},
                "config": {"model": "resnet50", "global_batch": args.batch * world, "seq_len": None,
                           "image_size": 224, "parallelism": f"dp{world}",
                           "trial": "PyTorchTrial", "optimizer": f"SGD momentum ({opt_name})",
                           "slots_per_trial": world},
            }
            print(json.dumps(out), flush=True)


def _conv_timings() -> int:
    from determined_clone_amd.ops import conv as conv_ops

    return int(conv_ops.TIMINGS)


def main() -> None:
    args = _args()
    from determined_clone_amd.launch import ranks

    if ranks.needs_launch(args.gpus):
        # no launcher around us: become the launcher (child process, before any GPU call)
        raise SystemExit(ranks.run_as_ranks(__file__, sys.argv[1:], args.gpus))
    _run_rank(args)


if __name__ == "__main__":
    main()
