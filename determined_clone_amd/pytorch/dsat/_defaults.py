"""Constants of DeepSpeed autotuning (reference: `harness/determined/pytorch/dsat/_defaults.py`)."""
USE_DSAT_MODE_KEY = "_use_dsat_mode"
OVERWRITE_KEY = "overwrite_deepspeed_args"
PROFILE_KEY = "_dsat_profile_steps"  # [start, end)
SEARCH_METHODS = ["binary", "random"]
SMALLER_IS_BETTER_METRICS = ["forward", "backward", "latency"]
LARGER_IS_BETTER_METRICS = ["throughput", "FLOPS_per_gpu"]
ARG_DEFAULTS = {
    "max_trials": 32,
    "max_concurrent_trials": 4,
    "zero_stages": [1, 2, 3],
    "start_profile_step": 3,
    "end_profile_step": 5,
    "metric": "throughput",
    "random_seed": 42,
    "max_mbs": 1024,
}
