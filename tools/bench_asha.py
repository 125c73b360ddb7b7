"""ASHA search throughput: completed trials per hour of the CIFAR-10 adaptive_asha search.

BASELINE.json's second metric ("ASHA trials/hr") on the config "CIFAR-10 adaptive_asha HP search,
16 concurrent trials gang-scheduled across 8 MI355X". This runs the real platform end to end, all
in one process tree on this node: an in-process master (searcher + native scheduler) and an agent
that exposes every MI355X as ``--slots-per-gpu`` slots; the master schedules
``max_concurrent_trials`` CIFAR-10 trials (``examples/cifar10_asha/model_def.py``: bf16 NHWC CNN,
fused BN+ReLU HIP kernel, fused SGD) as separate trial processes; adaptive ASHA promotes / stops
them. The value is COMPLETED trials / wall-clock hours from experiment creation to the searcher's
shutdown (trial process start-up, validation and checkpointing included).

Defaults are the example's search (examples/cifar10_asha/adaptive.yaml): 50,000 records x 8
epochs, 64 trials, 16 concurrent, batch 128, on ``--gpus N`` GPUs of this node (each GPU exposed as
ceil(16 / N) slots so the 16 concurrent trials are gang-scheduled onto them). Data: synthetic
CIFAR-shaped, class-conditional with position jitter and 10 % label noise (models/cifar.py), so the
validation errors spread and ASHA really prunes. The JSON also reports the share of allocation
time spent in trial start-up (process spawn to the first training batch, from the trials'
DET_STARTUP_TRACE marks) and the spread of final validation errors.

Usage: ``python tools/bench_asha.py [--gpus N] [--max-trials 64 --max-concurrent 16]``;
prints one JSON line.
"""
import argparse
import base64
import json
import os
import shutil
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import yaml  # noqa: E402
from typing import Dict, List, Tuple  # noqa: E402

from determined_clone_amd.agent import Agent  # noqa: E402
from determined_clone_amd.common.api import Session  # noqa: E402
from determined_clone_amd.master import Master, MasterServer  # noqa: E402
from determined_clone_amd.util import tar_directory  # noqa: E402


def search_config(args: argparse.Namespace) -> dict:
    with open(os.path.join(ROOT, "examples", "cifar10_asha", "adaptive.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["name"] = "bench_asha"
    cfg["records_per_epoch"] = args.records_per_epoch
    # PyTorchTrial epochs follow the training loader's length: shrink the synthetic dataset.
    cfg["hyperparameters"]["train_records"] = args.records_per_epoch
    cfg["hyperparameters"]["val_records"] = max(args.batch, args.records_per_epoch // 5)
    cfg["searcher"].update(max_trials=args.max_trials, max_concurrent_trials=args.max_concurrent,
                           max_length={"epochs": args.epochs})
    cfg["hyperparameters"]["global_batch_size"] = args.batch
    cfg["checkpoint_storage"] = {"save_trial_latest": 1, "save_trial_best": 0, "save_experiment_best": 1}
    cfg["max_restarts"] = 0
    if args.hip_graph is not None:  # A/B of the trials' HIP-graph-captured training step
        cfg.setdefault("optimizations", {})["hip_graph"] = bool(args.hip_graph)
    return cfg


def _print_trace(s: Session, trials: list) -> None:
    """Mean seconds-since-process-start of each start-up mark (exec/harness.py DET_STARTUP_TRACE)
    over the trials, plus the mean allocation wall time."""
    import re
    import statistics

    marks: dict = {}
    for t in trials:
        for line in s.get(f"/api/v1/trials/{t['id']}/logs")["logs"]:
            m = re.search(r"startup: (.+) at \+([0-9.]+)s", line["log"])
            if m:
                marks.setdefault(m.group(1), []).append(float(m.group(2)))
    for k, v in sorted(marks.items(), key=lambda kv: statistics.mean(kv[1])):
        print(f"[bench_asha] startup '{k}': mean +{statistics.mean(v):.3f}s over {len(v)} trials",
              file=sys.stderr, flush=True)


def _startup_share(m, s: Session, trials: list) -> dict:
    """Start-up seconds (spawn -> first training batch, one mark per trial process) summed over
    every allocation, over the summed allocation wall time."""
    import re

    marks = []
    for t in trials:
        for line in s.get(f"/api/v1/trials/{t['id']}/logs")["logs"]:
            mm = re.search(r"startup: first train batch at \+([0-9.]+)s", line["log"])
            if mm:
                marks.append(float(mm.group(1)))
    rows = m.db.all("SELECT start_time, end_time FROM allocations")
    alloc_s = sum(max(0.0, (r["end_time"] or time.time()) - (r["start_time"] or 0.0)) for r in rows)
    return {"share": round(sum(marks) / alloc_s, 4) if alloc_s else None,
            "mean_s": round(sum(marks) / len(marks), 3) if marks else None, "allocations": len(rows)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=0, help="GPUs of this node to use (0 = all)")
    ap.add_argument("--slots-per-gpu", type=int, default=0,
                    help="slots per GPU (0 = ceil(max_concurrent / gpus))")
    ap.add_argument("--max-trials", type=int, default=64)
    ap.add_argument("--max-concurrent", type=int, default=16)
    ap.add_argument("--epochs", type=int, default=8)
    ap.add_argument("--records-per-epoch", type=int, default=50000)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--timeout", type=float, default=3000.0)
    ap.add_argument("--cpu", action="store_true", help="artificial CPU slots (plumbing check)")
    ap.add_argument("--fake-gpus", type=int, default=0,
                    help="CPU rehearsal of the 8-GPU layout: the agent reports N ROCm devices "
                         "(--slots-per-gpu each) while the trials run on the CPU")
    ap.add_argument("--hip-graph", type=int, default=None, choices=(0, 1),
                    help="override the example's optimizations.hip_graph (A/B)")
    ap.add_argument("--trace", action="store_true",
                    help="also print mean start-up phase times to stderr")
    args = ap.parse_args()

    tmp = tempfile.mkdtemp(prefix="det-asha-bench-")
    m = Master(os.path.join(tmp, "m.db"),
               checkpoint_storage={"type": "shared_fs", "host_path": os.path.join(tmp, "ckpt")})
    srv = MasterServer(m, "127.0.0.1", 0).start()
    from determined_clone_amd.agent import agent as agent_mod

    if args.fake_gpus:
        fake = [{"id": i, "uuid": f"fake-gpu-{i}", "type": "rocm", "brand": "AMD", "gfx_target": "gfx950"}
                for i in range(args.fake_gpus)]
        agent_mod._detect_physical = lambda artificial_slots=0: [dict(d) for d in fake]
    phys = [d for d in agent_mod._detect_physical() if d["type"] == "rocm"]
    n_gpus = min(args.gpus, len(phys)) if args.gpus and phys else len(phys)
    spg = args.slots_per_gpu or max(1, -(-args.max_concurrent // max(1, n_gpus)))
    use_cpu_slots = args.cpu and not args.fake_gpus
    agent = Agent(m.master_url, "agent-0", artificial_slots=args.max_concurrent if use_cpu_slots else 0,
                  workdir=os.path.join(tmp, "agent"), slots_per_gpu=spg,
                  max_gpus=n_gpus if not use_cpu_slots else 0)
    # allocation timeline: (time, +1/-1, allocation, physical devices) -> concurrency overall / per GPU
    timeline: List[Tuple[float, int, str, Tuple[int, ...]]] = []
    devices_of: Dict[str, Tuple[int, ...]] = {}
    orig_start, orig_event = agent._start, agent._event

    def _start(spec):
        from determined_clone_amd.agent import runtime as rt

        devs = tuple(sorted({int(d.get("device_index", d["id"])) for d in rt.assigned_devices(spec, agent.devices)}))
        devices_of[spec["allocation_id"]] = devs
        timeline.append((time.time(), 1, spec["allocation_id"], devs))
        return orig_start(spec)

    def _event(alloc, state, exit_code=None):
        if state == "TERMINATED" and alloc in devices_of:
            timeline.append((time.time(), -1, alloc, devices_of.pop(alloc)))
        return orig_event(alloc, state, exit_code)

    agent._start, agent._event = _start, _event
    agent.start_background()
    s = Session(m.master_url)
    s.token = s.post("/api/v1/auth/login", {"username": "admin", "password": ""})["token"]
    try:
        cfg = search_config(args)
        env = cfg.setdefault("environment", {}).setdefault("environment_variables", [])
        env.append("DET_STARTUP_TRACE=1")  # per-trial start-up marks (start-up share below)
        if os.environ.get("DET_STARTUP_PROFILE"):
            env.append("DET_STARTUP_PROFILE=1")
        body = {"config": cfg, "model_definition": base64.b64encode(
            tar_directory(os.path.join(ROOT, "examples", "cifar10_asha"))).decode()}
        t0 = time.time()
        eid = s.post("/api/v1/experiments", body)["experiment"]["id"]
        state, last_print = "", 0.0
        while time.time() - t0 < args.timeout:
            state = s.get(f"/api/v1/experiments/{eid}")["experiment"]["state"]
            if state in ("COMPLETED", "CANCELED", "ERROR"):
                break
            if time.time() - last_print > 30:
                trials = s.get(f"/api/v1/experiments/{eid}/trials")["trials"]
                done = sum(t["state"] == "COMPLETED" for t in trials)
                print(f"[bench_asha] t={time.time() - t0:.0f}s trials={len(trials)} completed={done}",
                      file=sys.stderr, flush=True)
                last_print = time.time()
            time.sleep(0.5)
        wall = time.time() - t0
        trials = s.get(f"/api/v1/experiments/{eid}/trials")["trials"]
        done = [t for t in trials if t["state"] == "COMPLETED"]
        steps = sum(int(t.get("steps_completed") or 0) for t in done)
        vals = sorted(t["best_validation"] for t in done if t.get("best_validation") is not None)
        best = vals[0] if vals else None
        startup = _startup_share(m, s, trials)
        conc, per_dev, peak, peak_dev = 0, {}, 0, 0
        for _t, d, _a, devs in sorted(timeline, key=lambda e: (e[0], e[1])):
            conc += d
            peak = max(peak, conc)
            for g in devs:
                per_dev[g] = per_dev.get(g, 0) + d
                peak_dev = max(peak_dev, per_dev[g])
        if args.trace:
            _print_trace(s, trials)
        if state != "COMPLETED":
            errs = [t["id"] for t in trials if t["state"] == "ERROR"]
            print(f"[bench_asha] experiment ended {state!r}; errored trials {errs}", file=sys.stderr)
            for tid in (errs or [t["id"] for t in trials if t["state"] == "RUNNING"])[:1]:
                for line in s.get(f"/api/v1/trials/{tid}/logs")["logs"][-40:]:
                    print("   ", line["log"], file=sys.stderr)
        print(json.dumps({
            "metric": "ASHA trials/hr", "value": round(len(done) / (wall / 3600.0), 1),
            "unit": "trials/hr", "n_gpus": n_gpus, "higher_is_better": True,
            "experiment_state": state, "trials_completed": len(done), "trials_created": len(trials),
            "batches_trained": steps, "wall_s": round(wall, 1), "best_validation_error": best,
            "validation_error_quartiles": [round(vals[int(q * (len(vals) - 1))], 4) for q in (0, .25, .5, .75, 1)]
            if vals else None,
            "startup_share": startup["share"], "startup_mean_s": startup["mean_s"],
            "allocations": startup["allocations"],
            "max_concurrent_trials": peak, "max_trials_per_gpu": peak_dev,
            "gpus_used": len({g for e in timeline for g in e[3]}),
            "dtype": "bf16" if not args.cpu else "fp32", "data": "synthetic CIFAR-10-shaped",
            "config": {"model": "cifar10_cnn", "searcher": "adaptive_asha", "max_trials": args.max_trials,
                       "max_concurrent_trials": args.max_concurrent, "slots_per_gpu": spg,
                       "max_length_epochs": args.epochs, "records_per_epoch": args.records_per_epoch,
                       "global_batch": args.batch}}), flush=True)
    finally:
        agent.stop()
        srv.stop()
        time.sleep(1.0)
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
