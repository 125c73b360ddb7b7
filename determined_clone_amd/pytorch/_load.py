"""Rebuild a trained PyTorchTrial from a checkpoint directory (reference:
`harness/determined/pytorch/_load.py` load_trial_from_checkpoint_path)."""
import importlib
import json
import pathlib
import sys
from typing import Any, Dict, Optional

import torch

from determined_clone_amd import core


def load_trial_from_checkpoint_path(path: str, trial_class: Any = None,
                                    trial_kwargs: Optional[Dict[str, Any]] = None,
                                    torch_load_kwargs: Optional[Dict[str, Any]] = None) -> Any:
    from determined_clone_amd.pytorch._context import PyTorchTrialContext
    from determined_clone_amd.pytorch._controller import load_state_dict_file

    p = pathlib.Path(path)
    load_data = json.loads((p / "load_data.json").read_text()) if (p / "load_data.json").exists() else {}
    if trial_class is None:
        spec = load_data.get("trial_cls_spec")
        if not spec:
            raise ValueError("trial_class not given and checkpoint has no trial_cls_spec")
        code = p / "code"
        if code.exists() and str(code) not in sys.path:
            sys.path.insert(0, str(code))
        mod, _, qual = spec.partition(":")
        obj: Any = importlib.import_module(mod)
        for part in qual.split("."):
            obj = getattr(obj, part)
        trial_class = obj
    core_ctx = core._dummy_init()
    ctx = PyTorchTrialContext(core_context=core_ctx, trial_seed=0,
                              hparams=load_data.get("hparams") or {}, slots_per_trial=1,
                              num_gpus=1 if torch.cuda.is_available() else 0,
                              exp_conf=load_data.get("experiment_config"), managed_training=False)
    trial = trial_class(ctx, **(trial_kwargs or {}))
    ckpt = load_state_dict_file(str(p / "state_dict.pth"))
    sds = ckpt.get("models_state_dict") or [ckpt.get("model_state_dict")]
    for m, sd in zip(ctx.models, sds):
        m.load_state_dict(sd)
    for o, sd in zip(ctx.optimizers, ckpt.get("optimizers_state_dict", [])):
        o.load_state_dict(sd)
    return trial
