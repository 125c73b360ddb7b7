"""A/B of the linear weight-gradient split-K factor (ops/transformer.py ``_WGRAD_SPLITS``) on the
GPT-2 bench: ``python tools/probe_wgrad_splits.py SPLITS [bench_gpt2 args...]``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from determined_clone_amd.ops import transformer as T  # noqa: E402

T._WGRAD_SPLITS = int(sys.argv[1])
sys.argv = [sys.argv[0]] + sys.argv[2:]
import bench_gpt2  # noqa: E402

bench_gpt2.main()
