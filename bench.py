"""Headline benchmark: ResNet-50 PyTorchTrial training throughput (images/sec) on MI355X.

BASELINE.json metric: "images/sec ResNet-50 PyTorchTrial at 1/2/4/8 MI355X". The step that is
timed is the real PyTorchTrial path of this framework: ``pytorch.Trainer.fit`` ->
``_PyTorchTrialController`` -> ``trial.train_batch`` (forward, ``context.backward`` with bucketed
RCCL all-reduce overlapped with backward, ``context.step_optimizer`` with the fused HIP SGD) on
ResNet-50 v1.5 (random init, 25.6M params), bf16 NHWC activations, fp32 master weights, synthetic
224x224 ImageNet-shaped data resident in HBM. Weak scaling: 1024 images per GPU per step.

Usage: ``python bench.py [--gpus N --steps K --warmup W]``; for N>1 launch under
``torch.distributed.run`` (one rank per GPU, RANK/LOCAL_RANK/WORLD_SIZE from the env).
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
# MIOpen's find/perf databases and kernel cache ship in-tree (ops/miopen_db.py): a fresh box
# neither tunes nor compiles the convolutions. The library GEMMs replay the shipped TunableOp
# results (ops/gemm_tuning.py: +5% on this step, profiles/round3_resnet50_gemm_tuning_ab.txt).
_MIOPEN = os.path.join(HERE, "determined_clone_amd", "ops", "tuned", "miopen")
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(_MIOPEN, "db"))
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(_MIOPEN, "cache"))
os.environ.setdefault("DCA_GEMM_TUNED", "1")

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from determined_clone_amd import pytorch  # noqa: E402
from determined_clone_amd.models import resnet  # noqa: E402

METRIC = "images/sec ResNet-50 PyTorchTrial"
BASELINE_VALUE = None  # BASELINE.json "published" is empty


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
        # batch_size=None: each item already is a per-slot batch resident in HBM.
        ds = pytorch.DeviceBatchDataset(batches, length * self.context.distributed.size)
        return pytorch.DataLoader(ds, batch_size=None)

    def build_training_data_loader(self):
        return self._data(4, 10000)

    def build_validation_data_loader(self):
        return self._data(1, 1)


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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1024,
                    help="images per GPU per step (288 GB HBM: 1024 is 6%% faster than 512 and 13%% "
                         "faster than 256, profiles/round2_resnet50_batch_ab.txt, round2_resnet50_bs1024_ab.txt)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    if torch.cuda.is_available():
        # this rank's GPU first: a bare torch.cuda call would open a context on device 0 in every rank
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
        # A process that just ended on this GPU may still be returning its ~200 GB of HBM: starting
        # the bs-1024 step in the remainder makes the caching allocator free and re-map blocks every
        # step (alloc retries). Wait (bounded) for the device's memory to come back first.
        free0, total = torch.cuda.mem_get_info()
        t_wait = time.time()
        while free0 < 0.8 * total and time.time() - t_wait < 60:
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
    # the timed step runs eagerly: optimizations.hip_graph is refused for MIOpen convolutions
    # (pytorch/_graph.py), and train_batch's timestamps must run on every step
    exp_conf = {"optimizations": {"aggregation_frequency": 1, "average_training_metrics": True}}
    with pytorch.init(hparams=hparams, exp_conf=exp_conf) as ctx:
        trial = ResNet50BenchTrial(ctx)
        trainer = pytorch.Trainer(trial, ctx)
        total = args.warmup + args.steps
        trainer.fit(max_length=pytorch.Batch(total), reporting_period=pytorch.Batch(total),
                    checkpoint_policy="none")
        dt = trial.t1 - trial.t0
        ms = dt / args.steps * 1000.0
        if ctx.distributed.size > 1:
            ms = max(ctx.distributed.allgather(ms))
        imgs = args.batch * world * args.steps / (ms * args.steps / 1000.0)
        if torch.cuda.is_available():
            ev = trial.events
            step_ms = [round(a.elapsed_time(b), 2) for a, b in zip(ev[:-1], ev[1:])]
            ms_stats = torch.cuda.memory_stats()
            print(json.dumps({"rank": ctx.distributed.rank, "gpu_state_end": _gpu_state()}), file=sys.stderr)
            print(json.dumps({"rank": ctx.distributed.rank, "step_ms": step_ms,
                              "max_reserved_gb": round(torch.cuda.max_memory_reserved() / 2**30, 1),
                              "alloc_retries": ms_stats.get("num_alloc_retries", 0),
                              "device_free_gb": round(torch.cuda.mem_get_info()[0] / 2**30, 1)}),
                  file=sys.stderr, flush=True)
        if ctx.distributed.rank == 0:
            out = {
                "metric": METRIC, "value": round(imgs, 1), "unit": "images/sec",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None if BASELINE_VALUE is None else round(imgs / BASELINE_VALUE, 3),
                "dtype": "bf16", "data": "synthetic (random 224x224x3 images + labels resident in HBM, random-init weights)",
                "config": {"model": "resnet50", "global_batch": args.batch * world, "seq_len": None,
                           "image_size": 224, "parallelism": f"dp{world}",
                           "trial": "PyTorchTrial", "optimizer": "SGD momentum (fused HIP)",
                           "slots_per_trial": world},
            }
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
