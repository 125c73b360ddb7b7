"""bench.py driver contract on CPU: 2 ranks under torch.distributed.run (gloo), rank 0 prints ONE
JSON line whose value is the whole-job aggregate of the max-over-ranks step time."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_prints_one_aggregate_json_line():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "2"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in r
    assert r["n_gpus"] == 2 and r["steps"] == 2 and r["warmup"] == 1
    assert r["scaling"] == "weak" and r["higher_is_better"] is True
    assert r["config"]["model"] == "resnet50" and r["config"]["global_batch"] == 4
    assert r["config"]["parallelism"] == "dp2"
    # whole-job images/s from the slowest rank's step time
    assert abs(r["value"] - 4 / (r["ms_per_step"] / 1000.0)) / r["value"] < 0.01


def test_bench_gpus_flag_launches_ranks_itself():
    """``python bench.py --gpus 2`` with NO launcher around it (the driver's BENCH command shape)
    starts the two ranks itself and reports what torch.distributed formed."""
    env = dict(os.environ, OMP_NUM_THREADS="2")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--batch", "2"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["world_size"] == 2
    assert r["config"]["parallelism"] == "dp2" and r["config"]["global_batch"] == 4
    assert r["backend"] == "gloo"  # CPU here; "nccl" (RCCL) on the GPU box
    assert r["device"] == "cpu" and "host memory" in r["data"]


def _rank_errors(stderr: str) -> str:
    """The ranks' own tracebacks (the launcher's summary at the end only says which were killed)."""
    i = stderr.find("Traceback (most recent call last)")
    return stderr[i:i + 4000] if i >= 0 else stderr[:3000]


def _one_json_line(out):
    assert out.returncode == 0, _rank_errors(out.stderr) + "\n...\n" + out.stderr[-1500:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def _run_ranks(cmd):
    """Run an 8-rank self-launch once more if the first attempt died: two full-suite runs in this
    container each lost one 8-rank launch (a different test each time) while every standalone and
    partial-suite repetition passed, i.e. an environmental start-up failure (all 8 CPU-bound ranks
    plus the launcher on 8 cores). The first failure is reported as a warning with the ranks'
    tracebacks, so a real fault still shows; a second failure fails the test."""
    import warnings

    out = subprocess.run(cmd, cwd=ROOT, env=_clean_env(), capture_output=True, text=True, timeout=900)
    if out.returncode != 0:
        warnings.warn("8-rank launch failed once, retrying: " + _rank_errors(out.stderr)[:2000])
        out = subprocess.run(cmd, cwd=ROOT, env=_clean_env(), capture_output=True, text=True,
                             timeout=900)
    return out


def _clean_env():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_bench_eight_ranks_world_size_eight():
    """the driver's 8-GPU launch shape (``bench.py --gpus 8``, no launcher) forms
    an 8-rank process group and reports the 8-rank aggregate (gloo on CPU, tiny batch)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1",
           "--warmup", "1", "--batch", "1"]
    r = _one_json_line(_run_ranks(cmd))
    assert r["n_gpus"] == 8 and r["world_size"] == 8 and r["backend"] == "gloo"
    assert r["config"]["parallelism"] == "dp8" and r["config"]["global_batch"] == 8
    assert abs(r["value"] - 8 / (r["ms_per_step"] / 1000.0)) / r["value"] < 0.01


def test_bench_gpt2_eight_ranks_zero2():
    """``tools/bench_gpt2.py --gpus 8``: the GPT-2 DeepSpeedTrial ZeRO-2 bench at 8 ranks (a tiny
    GPT on CPU; the MI355X run uses gpt2-medium)."""
    cmd = [sys.executable, os.path.join(ROOT, "tools", "bench_gpt2.py"), "--gpus", "8", "--model", "tiny",
           "--micro", "1", "--seq", "64", "--steps", "1", "--warmup", "1"]
    r = _one_json_line(_run_ranks(cmd))
    assert r["n_gpus"] == 8 and r["world_size"] == 8 and r["backend"] == "gloo"
    assert r["config"]["parallelism"] == "zero2-dp8" and r["config"]["global_batch"] == 8
