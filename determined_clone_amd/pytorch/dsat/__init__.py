"""DeepSpeed autotuning for DeepSpeedTrials (reference: `harness/determined/pytorch/dsat`):
``python -m determined_clone_amd.pytorch.dsat {binary,random} config.yaml model_dir``."""
from determined_clone_amd.pytorch.dsat import _defaults
from determined_clone_amd.pytorch.dsat._search import DSATSearchMethod
