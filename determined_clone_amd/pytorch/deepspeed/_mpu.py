"""Model-parallel unit descriptor (reference: `harness/determined/pytorch/deepspeed/_mpu.py`)."""
from dataclasses import dataclass
from typing import Any


@dataclass
class ModelParallelUnit:
    """Data-parallel topology and which ranks report metrics / build data loaders. Custom model
    parallel trials pass their own instance to ``DeepSpeedTrialContext.set_mpu``."""

    data_parallel_rank: int
    data_parallel_world_size: int
    should_report_metrics: bool
    should_build_data_loader: bool


def make_data_parallel_mpu(dist_context: Any) -> ModelParallelUnit:
    return ModelParallelUnit(data_parallel_rank=dist_context.get_rank(),
                             data_parallel_world_size=dist_context.get_size(),
                             should_report_metrics=True, should_build_data_loader=True)


def make_deepspeed_mpu(topology: Any) -> ModelParallelUnit:
    """From a pipeline/model-parallel grid object exposing DeepSpeed's topology accessors."""
    first = topology.get_pipe_parallel_rank() == 0
    last = topology.get_pipe_parallel_rank() == topology.get_pipe_parallel_world_size() - 1
    return ModelParallelUnit(
        data_parallel_rank=topology.get_data_parallel_rank(),
        data_parallel_world_size=topology.get_data_parallel_world_size(),
        should_report_metrics=True,
        # every tensor-parallel rank of the first / last stage reads the same batch itself
        # (instead of Megatron's broadcast from slice rank 0)
        should_build_data_loader=first or last)
