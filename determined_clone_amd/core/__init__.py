"""Core API (reference: `harness/determined/core/__init__.py`)."""
from determined_clone_amd.core._checkpoint import (CheckpointContext, DownloadMode,
                                                   DummyCheckpointContext, merge_metadata,
                                                   merge_resources)
from determined_clone_amd.core._distributed import DistributedContext, DummyDistributedContext
from determined_clone_amd.core._experimental import (DummyExperimentalCoreContext,
                                                     ExperimentalCoreContext)
from determined_clone_amd.core._heartbeat import _Heartbeat
from determined_clone_amd.core._preempt import DummyPreemptContext, PreemptContext, PreemptMode
from determined_clone_amd.core._searcher import (DummySearcherContext, DummySearcherOperation,
                                                 SearcherContext, SearcherMode, SearcherOperation,
                                                 Unit, _parse_searcher_units)
from determined_clone_amd.core._train import DummyTrainContext, EarlyExitReason, TrainContext
from determined_clone_amd.core._context import Context, TensorboardMode, _dummy_init, init
