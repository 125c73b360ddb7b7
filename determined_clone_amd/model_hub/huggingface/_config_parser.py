"""Hyperparameter -> keyword-argument parsing for the transformers builders (reference:
``model_hub/model_hub/huggingface/_config_parser.py``).

Each ``*Kwargs`` class declares the keys it accepts and their defaults; keys listed in
``_OPTIONAL`` are emitted only when the hparams provide them (e.g. ``num_labels`` must not be
passed to ``AutoConfig`` unless the user set it)."""
import dataclasses
from typing import Any, Dict, Tuple, Type, Union

from determined_clone_amd.model_hub.utils import AttrDict

_UNSET = object()


class _Kwargs:
    """Base: construct from any mapping, ignoring unknown keys; ``as_dict`` drops unset optionals."""

    _OPTIONAL: Tuple[str, ...] = ()

    @classmethod
    def from_mapping(cls, args: Dict[str, Any]) -> "_Kwargs":
        names = {f.name for f in dataclasses.fields(cls)}
        obj = cls(**{k: v for k, v in args.items() if k in names})  # type: ignore[call-arg]
        return obj

    def as_dict(self) -> Dict[str, Any]:
        return {f.name: getattr(self, f.name) for f in dataclasses.fields(self)
                if getattr(self, f.name) is not _UNSET}


@dataclasses.dataclass
class DatasetKwargs(_Kwargs):
    """Either ``dataset_name`` (+ ``dataset_config_name``) or ``train_file``/``validation_file``."""

    dataset_name: Any = None
    dataset_config_name: Any = None
    validation_split_percentage: Any = None
    train_file: Any = None
    validation_file: Any = None


@dataclasses.dataclass
class ConfigKwargs(_Kwargs):
    pretrained_model_name_or_path: Any = None
    cache_dir: Any = None
    revision: Any = "main"
    use_auth_token: Any = False
    num_labels: Any = _UNSET
    finetuning_task: Any = _UNSET


@dataclasses.dataclass
class TokenizerKwargs(_Kwargs):
    pretrained_model_name_or_path: Any = None
    cache_dir: Any = None
    revision: Any = "main"
    use_auth_token: Any = False
    use_fast: Any = True
    do_lower_case: Any = _UNSET


@dataclasses.dataclass
class ModelKwargs(_Kwargs):
    pretrained_model_name_or_path: Any = None
    cache_dir: Any = None
    revision: Any = "main"
    use_auth_token: Any = False


@dataclasses.dataclass
class OptimizerKwargs(_Kwargs):
    """transformers.Trainer defaults; ``adafactor`` switches from AdamW to Adafactor."""

    weight_decay: Any = 0.0
    adafactor: Any = False
    learning_rate: Any = 5e-5
    max_grad_norm: Any = 1.0
    adam_beta1: Any = 0.9
    adam_beta2: Any = 0.999
    adam_epsilon: Any = 1e-8
    scale_parameter: Any = False
    relative_step: Any = False


@dataclasses.dataclass
class LRSchedulerKwargs(_Kwargs):
    num_training_steps: Any = None
    lr_scheduler_type: Any = "linear"
    num_warmup_steps: Any = 0


def parse_dict_to_dataclasses(dataclass_types: Tuple[Type[_Kwargs], ...],
                              args: Union[Dict[str, Any], AttrDict],
                              as_dict: bool = False) -> Tuple[Any, ...]:
    """Fill each dataclass from the keys of ``args`` it declares (one key may feed several)."""
    out = []
    for t in dataclass_types:
        obj = t.from_mapping(args)
        out.append(AttrDict(obj.as_dict()) if as_dict else obj)
    return tuple(out)


def default_parse_config_tokenizer_model_kwargs(
        hparams: Union[Dict[str, Any], AttrDict]) -> Tuple[AttrDict, AttrDict, AttrDict]:
    """Config / tokenizer / model kwargs; ``pretrained_model_name_or_path`` feeds all three and
    ``config_name`` / ``tokenizer_name`` / ``model_name`` override it per builder."""
    hp = hparams if isinstance(hparams, AttrDict) else AttrDict(hparams)
    cfg, tok, mdl = parse_dict_to_dataclasses((ConfigKwargs, TokenizerKwargs, ModelKwargs), hp, as_dict=True)
    for target, key in ((cfg, "config_name"), (tok, "tokenizer_name"), (mdl, "model_name")):
        if key in hp:
            target.pretrained_model_name_or_path = hp[key]
    if any(x.pretrained_model_name_or_path is None for x in (cfg, tok, mdl)):
        raise ValueError("set pretrained_model_name_or_path (or config_name, tokenizer_name and "
                         "model_name) in the hyperparameters")
    return cfg, tok, mdl


def default_parse_optimizer_lr_scheduler_kwargs(
        hparams: Union[Dict[str, Any], AttrDict]) -> Tuple[OptimizerKwargs, LRSchedulerKwargs]:
    opt, sched = parse_dict_to_dataclasses((OptimizerKwargs, LRSchedulerKwargs), hparams)
    return opt, sched
