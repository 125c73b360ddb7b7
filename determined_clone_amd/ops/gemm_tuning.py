"""Tuned hipBLASLt / rocBLAS solutions for the framework's GEMMs (PyTorch TunableOp), shipped in-tree.

The library GEMMs of the hot paths -- GPT-2 linears (forward, data gradient, split-K weight
gradient), ResNet-50's pointwise convolutions run as GEMMs (ops/conv.py), the classifier -- go to
hipBLASLt through ``at::cuda::blas::gemm``, and hipBLASLt's heuristic picks the first solution of
its ranking, not the fastest one on MI355X for the shape (e.g. a 256x256x32 macro tile on the GPT-2
MLP GEMMs). TunableOp times every hipBLASLt and rocBLAS solution for each (transpose, M, N, K,
dtype) once and keeps the fastest; the results of a tuning run on MI355X are shipped in
``ops/tuned/gemm_gfx950.csv`` (the same idea as the shipped MIOpen find DB under ``tools/miopen``),
so training processes only REPLAY them: no tuning on the job's clock, and shapes that were not
tuned fall back to the default heuristic.

The CSV starts with TunableOp's validator lines (PyTorch / ROCm / hipBLASLt / rocBLAS versions, GPU
arch): on a different software stack TunableOp rejects the file and everything runs untuned.

* ``enable()`` -- replay the shipped results; called when the HIP extension loads on a GPU
  process, effective with ``DCA_GEMM_TUNED=1`` (set by the benchmarks and the ResNet-50 / GPT-2
  example configs). Opt-in because switching TunableOp on costs a process ~0.8 s at its first GEMMs
  (library / validator loading, tools/probe_trial_startup.py): worth it for a long training job,
  20% of a short ASHA trial.
* ``DCA_GEMM_TUNE=<file>`` -- tuning run: every new shape is timed and the results are written to
  ``<file>`` at exit; ``tools/tune_gemms.py`` merges such files into the shipped one.

Each process replays from its own temporary copy of the file (removed at exit), so no rank ever
opens the shipped file for writing.
"""
import os
import shutil
import tempfile
from typing import Dict, List, Optional

RESULTS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "gemm_gfx950.csv")
_state: Dict[str, Optional[str]] = {"path": None}


def enable(path: Optional[str] = None, tune: bool = False) -> bool:
    """Route library GEMMs through TunableOp: replay ``path`` (default: the shipped results) or,
    with ``tune``, time every solution of each new shape and write the results to ``path``.
    Returns whether TunableOp is on."""
    if _state["path"] is not None:
        return True
    if os.environ.get("DCA_GEMM_TUNE"):  # tuning run (tools/tune_gemms.py): write results there
        path, tune = os.environ["DCA_GEMM_TUNE"], True
    if os.environ.get("DCA_GEMM_TUNED", "0") != "1" and not tune:
        return False
    import torch

    if not torch.cuda.is_available() or not hasattr(torch.cuda, "tunable"):
        return False
    src = path or RESULTS
    if tune:
        target = src
    else:
        if not os.path.exists(src):
            return False
        fd, target = tempfile.mkstemp(prefix="dca_gemm_tuned_", suffix=".csv")
        os.close(fd)
        shutil.copyfile(src, target)
        # replay never writes the database back (results are written as tunings complete), so
        # the copy can go when the process ends
        import atexit

        atexit.register(lambda p=target: os.path.exists(p) and os.remove(p))
    import torch.cuda.tunable as tunable

    tunable.set_filename(target, False)
    tunable.tuning_enable(tune)
    if tune:
        # time each candidate on rotated operand copies (L2/MALL-cold, as in the training step)
        tunable.set_rotating_buffer_size(256)
        tunable.set_max_tuning_duration(8)
        tunable.set_max_tuning_iterations(30)
        # reject candidates whose output differs from the default solution's: without this check
        # TunableOp kept a hipBLASLt solution for tn_256_3211264_64 (ResNet-50 layer1 1x1 forward
        # at bs 1024) that was fastest because it computed wrong values
        # (tools/validate_tuned_gemms.py, profiles/round6_tuned_gemm_validation.txt)
        if hasattr(tunable, "set_numerical_check_tolerances"):
            tunable.set_numerical_check_tolerances(True, 0.05, 0.05)
        else:
            os.environ["PYTORCH_TUNABLEOP_NUMERICAL_CHECK"] = "1"
    tunable.enable(True)
    _state["path"] = target
    return True


def merge(results: List[str], out: str = RESULTS) -> int:
    """Union the tuned rows of ``results`` (TunableOp CSVs from one software stack) into ``out``;
    later files win for a repeated (op, params). Returns the number of tuned rows written."""
    validators: Dict[str, str] = {}
    rows: Dict[tuple, str] = {}
    for p in ([out] if os.path.exists(out) else []) + list(results):
        with open(p) as f:
            for line in f:
                line = line.rstrip("\n")
                if not line:
                    continue
                parts = line.split(",")
                if parts[0] == "Validator":
                    validators[parts[1]] = line
                elif len(parts) >= 3:
                    rows[(parts[0], parts[1])] = line
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        for k in sorted(validators):
            f.write(validators[k] + "\n")
        for k in sorted(rows):
            f.write(rows[k] + "\n")
    return len(rows)
