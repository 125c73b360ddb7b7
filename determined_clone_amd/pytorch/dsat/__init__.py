"""DeepSpeed autotuning for DeepSpeedTrials and Core API scripts (reference:
`harness/determined/pytorch/dsat`):
``python -m determined_clone_amd.pytorch.dsat {binary,random,asha} config.yaml model_dir``."""
from determined_clone_amd.pytorch.dsat import _defaults
from determined_clone_amd.pytorch.dsat._asha import ASHADSATSearchMethod
from determined_clone_amd.pytorch.dsat._search import DSATSearchMethod
from determined_clone_amd.pytorch.dsat._utils import (
    dsat_reporting_context,
    get_batch_config_from_mbs_gas_and_slots,
    get_ds_config_from_hparams,
    get_random_zero_optim_config,
    merge_dicts,
    report_json_results,
)
