"""Merge TunableOp result files from tuning runs into the shipped ``ops/tuned/gemm_gfx950.csv``.

Tuning runs happen on an MI355X (tools/gpu/r3_tune.sh): each benchmark runs a few steps with
``DCA_GEMM_TUNE=<file>`` (ops/gemm_tuning.py), which times every hipBLASLt / rocBLAS solution of
each GEMM shape it meets and writes the winners to <file> at exit.
Usage: ``python tools/tune_gemms.py run1.csv [run2.csv ...]``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from determined_clone_amd.ops import gemm_tuning  # noqa: E402

if __name__ == "__main__":
    n = gemm_tuning.merge(sys.argv[1:])
    print(f"{n} tuned GEMM rows in {gemm_tuning.RESULTS}")
