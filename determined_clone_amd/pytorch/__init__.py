"""PyTorch training APIs (reference: `harness/determined/pytorch/__init__.py`)."""
from determined_clone_amd.pytorch._callback import PyTorchCallback
from determined_clone_amd.pytorch._data import (DataLoader, DeviceBatchDataset, DevicePrefetcher,
                                                SyntheticDataset, TorchData, adapt_batch_sampler,
                                                data_length, to_device)
from determined_clone_amd.pytorch._lr_scheduler import LRScheduler
from determined_clone_amd.pytorch._reducer import (MetricReducer, Reducer, _PyTorchReducerContext,
                                                   _simple_reduce_metrics)
from determined_clone_amd.pytorch._trial import Batch, Epoch, PyTorchTrial, TrainUnit
from determined_clone_amd.pytorch._context import ClipGradNorm, PyTorchTrialContext, clip_grad_norm
from determined_clone_amd.pytorch._controller import _PyTorchTrialController, load_state_dict_file
from determined_clone_amd.pytorch._trainer import Trainer, init
from determined_clone_amd.pytorch._load import load_trial_from_checkpoint_path
from determined_clone_amd.pytorch import samplers

PyTorchTrial.trial_context_class = PyTorchTrialContext
