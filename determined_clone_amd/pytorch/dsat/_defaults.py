"""Constants of DeepSpeed autotuning (reference: `harness/determined/pytorch/dsat/_defaults.py`)."""
USE_DSAT_MODE_KEY = "_use_dsat_mode"
CONFIG_KEY = "deepspeed_config"          # hparam naming the DS json, relative to the model dir
OVERWRITE_KEY = "overwrite_deepspeed_args"
PROFILE_KEY = "_dsat_profile_steps"  # [start, end)
SEARCH_METHODS = ["binary", "random", "asha", "_test"]
SMALLER_IS_BETTER_METRICS = ["forward", "backward", "latency"]
LARGER_IS_BETTER_METRICS = ["throughput", "FLOPS_per_gpu"]
GAS_DEFAULT = 1

# files the engine's autotuning hook writes in the working directory before it ends the process
# with SystemExit (pytorch/deepspeed/_autotune.py); dsat_reporting_context / the DeepSpeedTrial
# controller read them back and report them to the searcher
MODEL_INFO_PROFILING_PATH = "model_info.json"
AUTOTUNING_RESULTS_PATH = "autotuning_metric.json"

# the first trial of a search measures the model (parameters, activation bytes per sample, device
# memory) at micro batch 1; the search sizes its micro-batch ranges from it
MODEL_INFO_PROFILE_DS_CONFIG = {
    "train_micro_batch_size_per_gpu": 1,
    "autotuning": {"enabled": True, "model_info_path": MODEL_INFO_PROFILING_PATH,
                   "model_info": {"profile": True}},
}

# ZeRO knobs sampled per random configuration, written as the increment over the previous stage.
# Bucket sizes (elements) are centred on what moves well over one xGMI hop: 8-256 Mi elements of
# bf16 (16-512 MiB) -- the all-reduce / reduce-scatter of one bucket is then several hundred us,
# far above the collective launch latency, while the tail bucket after the last layer stays short.
_BUCKETS = [n * 2 ** 20 for n in (8, 16, 32, 64, 128, 256)]
DEFAULT_ZERO_SEARCH_SPACE = {
    0: {},
    1: {"reduce_bucket_size": _BUCKETS, "allgather_bucket_size": _BUCKETS},
    2: {"overlap_comm": [True, False], "reduce_scatter": [True, False],
        "contiguous_gradients": [True, False]},
    3: {"allgather_partitions": [True, False]},
}

ARG_DEFAULTS = {
    "max_trials": 32,
    "max_concurrent_trials": 4,
    "zero_stages": [1, 2, 3],
    "start_profile_step": 3,
    "end_profile_step": 5,
    "metric": "throughput",
    "random_seed": 42,
    "max_mbs": 1024,
    # random
    "trials_per_random_config": 5,
    # binary / asha
    "search_range_factor": 1.0,
    # asha (arxiv:1810.05934: eta = divisor, s = asha_early_stopping)
    "divisor": 2,
    "min_binary_search_trials": 3,
    "max_rungs": 5,
    "asha_early_stopping": 0,
}
