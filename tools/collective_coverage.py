"""Line coverage of the production collective calls in the CPU multi-rank tests.

``coverage`` is not installed in this image, so this runs the multi-rank workers of
``tests/test_zero.py``, ``tests/test_zero3.py``, ``tests/test_distributed.py`` and
``tests/test_deepspeed_trial.py`` (gloo, 2 ranks each) under a ``sys.settrace`` line tracer limited
to ``determined_clone_amd/parallel/*.py``, merges the executed lines of every rank, and reports, for
every line of those files that calls an in-place tensor collective (``reduce_scatter_tensor``,
``all_gather_into_tensor``) or uses ``ReduceOp.AVG``, whether some rank executed it -- the lines
the 8-GPU RCCL run takes.

Usage: python tools/collective_coverage.py [--world 8] [> profiles/round6_collective_coverage_w8.txt]
(``--world 8``: every worker at the driver's 8-rank layout.)
"""
import glob
import json
import os
import re
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PAR = os.path.join(ROOT, "determined_clone_amd", "parallel")
PATTERN = re.compile(r"reduce_scatter_tensor\(|all_gather_into_tensor\(|ReduceOp\.AVG")


def _traced(rank, fn_path, args, out_dir):
    """mp.spawn entry: run tests.<module>.<fn>(rank, *args) under a line tracer."""
    import importlib
    import threading

    executed = set()

    def tracer(frame, event, arg):
        fname = frame.f_code.co_filename
        if not fname.startswith(PAR):
            return None

        def local(f, ev, a):
            if ev == "line":
                executed.add((f.f_code.co_filename, f.f_lineno))
            return local
        executed.add((fname, frame.f_lineno))
        return local

    sys.settrace(tracer)
    threading.settrace(tracer)
    mod, fn = fn_path.rsplit(".", 1)
    try:
        getattr(importlib.import_module(mod), fn)(rank, *args)
    finally:
        sys.settrace(None)
        with open(os.path.join(out_dir, f"cov-{fn}-{rank}-{os.getpid()}.json"), "w") as f:
            json.dump(sorted(executed), f)


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main() -> None:
    import argparse

    import torch.multiprocessing as mp

    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2, choices=(2, 4, 8))
    w = ap.parse_args().world
    gb = 4 if w == 2 else 8  # global (micro) batch the per-rank slices are cut from
    runs = [
        ("tests.test_zero._worker", lambda d: (w, _free_port(), 1, "adam", 0.0, 64.0, d, False)),
        ("tests.test_zero._worker", lambda d: (w, _free_port(), 2, "adamw", 0.05, 0.002, d, False)),
        ("tests.test_zero._worker", lambda d: (w, _free_port(), 2, "sgd", 0.0, 0.001, d, True)),
        ("tests.test_zero3._worker", lambda d: (w, _free_port(), d, gb)),
        ("tests.test_distributed._worker_sync", lambda d: (w, _free_port(), True, 1, d)),
        ("tests.test_distributed._worker_sync", lambda d: (w, _free_port(), False, 2, d)),
        ("tests.test_deepspeed_trial._engine_worker", lambda d: (w, _free_port(), 2, d, True, gb)),
        ("tests.test_deepspeed_trial._engine_worker", lambda d: (w, _free_port(), 1, d, False, gb)),
    ]
    cov_dir = tempfile.mkdtemp(prefix="collcov-")
    for fn_path, mk in runs:
        with tempfile.TemporaryDirectory() as d:
            mp.spawn(_traced, args=(fn_path, mk(d), cov_dir), nprocs=w, join=True)
        print(f"ran {fn_path} x{w} ranks", flush=True)
    executed = set()
    for f in glob.glob(os.path.join(cov_dir, "*.json")):
        executed.update((a, b) for a, b in json.load(open(f)))
    print()
    print("in-place collective / AVG call sites in determined_clone_amd/parallel (executed by a gloo rank?)")
    hit = total = 0
    for path in sorted(glob.glob(os.path.join(PAR, "*.py"))):
        for ln, line in enumerate(open(path), 1):
            if PATTERN.search(line) and not line.lstrip().startswith(("#", '"', "*", "``")):
                total += 1
                ok = (path, ln) in executed
                hit += ok
                print(f"  {'EXECUTED' if ok else 'not run '}  {os.path.relpath(path, ROOT)}:{ln}  {line.strip()[:90]}")
    print(f"\n{hit}/{total} call sites executed")


if __name__ == "__main__":
    main()
