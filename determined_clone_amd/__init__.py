"""determined_clone_amd — an MI355X-native deep-learning training platform with the capabilities of
Determined (Core API, PyTorchTrial/Trainer, DeepSpeed-style ZeRO, hyperparameter search, master /
agent / CLI), built on PyTorch-ROCm, hand-written HIP kernels for gfx950 and RCCL over xGMI."""
__version__ = "0.1.0"

from determined_clone_amd._info import (ClusterInfo, RendezvousInfo, ResourcesInfo, TrialInfo,
                                        get_cluster_info)
from determined_clone_amd._experiment_config import ExperimentConfig
from determined_clone_amd._import import import_from_path
from determined_clone_amd.errors import InvalidHP
from determined_clone_amd import errors, util

# Log format whose level prefix the master's log viewer filters on (reference: det.LOG_FORMAT).
LOG_FORMAT = "%(levelname)s: [%(process)s] %(name)s: %(message)s"


def __getattr__(name: str):
    # Lazy subpackages so `import determined_clone_amd` stays light (CLI, master).
    import importlib

    if name in ("core", "pytorch", "searcher", "experimental", "tensorboard", "profiler",
                "launch", "ops", "parallel", "models", "master", "agent", "cli", "config",
                "transformers", "exec", "native", "common"):
        return importlib.import_module(f"determined_clone_amd.{name}")
    raise AttributeError(name)
