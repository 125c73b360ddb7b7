"""Hugging Face transformers as a PyTorchTrial (reference: ``model_hub/model_hub/huggingface/
_trial.py``: build_using_auto, build_default_optimizer / lr scheduler, default_load_dataset,
BaseTransformerTrial).

On MI355X the default optimizer is ``torch.optim.AdamW`` (``context.wrap_optimizer`` swaps it for
the flat-buffer HIP AdamW), gradient clipping is the device-side fused clip of the optimizer step
(``pytorch.clip_grad_norm``), and ``use_bf16: true`` runs the forward under bf16 autocast."""
import inspect
import logging
from typing import Any, Dict, List, Optional, Tuple, Union

import torch

from determined_clone_amd import pytorch as det_torch
from determined_clone_amd.model_hub import utils
from determined_clone_amd.model_hub.huggingface import _config_parser as hf_parse

logger = logging.getLogger("determined_clone_amd.model_hub")

MODEL_MODES = {
    "base": "AutoModel",
    "pretraining": "AutoModelForPreTraining",
    "causal-lm": "AutoModelForCausalLM",
    "masked-lm": "AutoModelForMaskedLM",
    "seq2seq-lm": "AutoModelForSeq2SeqLM",
    "sequence-classification": "AutoModelForSequenceClassification",
    "multiple-choice": "AutoModelForMultipleChoice",
    "next-sentence": "AutoModelForNextSentencePrediction",
    "token-classification": "AutoModelForTokenClassification",
    "question-answering": "AutoModelForQuestionAnswering",
}


def build_using_auto(config_kwargs: Dict[str, Any], tokenizer_kwargs: Dict[str, Any], model_mode: str,
                     model_kwargs: Union[Dict[str, Any], hf_parse.ModelKwargs],
                     use_pretrained_weights: bool = True) -> Tuple[Any, Any, Any]:
    """(config, tokenizer, model) through transformers' Auto classes; ``use_pretrained_weights``
    False builds the architecture with random weights from the config."""
    import transformers

    if model_mode not in MODEL_MODES:
        raise ValueError(f"model_mode must be one of {sorted(MODEL_MODES)}, got {model_mode!r}")
    config = transformers.AutoConfig.from_pretrained(**dict(config_kwargs))
    tokenizer = transformers.AutoTokenizer.from_pretrained(**dict(tokenizer_kwargs))
    builder = getattr(transformers, MODEL_MODES[model_mode])
    mk = model_kwargs.as_dict() if isinstance(model_kwargs, hf_parse.ModelKwargs) else dict(model_kwargs)
    if use_pretrained_weights:
        mk["config"] = config
        model = builder.from_pretrained(**mk)
    else:
        model = builder.from_config(config)
    return config, tokenizer, model


def group_parameters_for_optimizer(model: torch.nn.Module, weight_decay: Optional[float] = 0.0,
                                   no_decay: Tuple[str, ...] = ("bias", "LayerNorm.weight")
                                   ) -> List[Dict[str, Any]]:
    """Two param groups: with ``weight_decay`` and (biases / LayerNorm weights) without."""
    decay, plain = [], []
    for n, p in model.named_parameters():
        (plain if any(nd in n for nd in no_decay) else decay).append(p)
    return [{"params": decay, "weight_decay": weight_decay or 0.0},
            {"params": plain, "weight_decay": 0.0}]


def build_default_optimizer(model: torch.nn.Module, optimizer_kwargs: hf_parse.OptimizerKwargs) -> torch.optim.Optimizer:
    groups = group_parameters_for_optimizer(model, optimizer_kwargs.weight_decay)
    if optimizer_kwargs.adafactor:
        from transformers.optimization import Adafactor

        return Adafactor(groups, lr=optimizer_kwargs.learning_rate,
                         scale_parameter=optimizer_kwargs.scale_parameter,
                         relative_step=optimizer_kwargs.relative_step)
    return torch.optim.AdamW(groups, lr=optimizer_kwargs.learning_rate,
                             betas=(optimizer_kwargs.adam_beta1, optimizer_kwargs.adam_beta2),
                             eps=optimizer_kwargs.adam_epsilon)


def build_default_lr_scheduler(optimizer: torch.optim.Optimizer,
                               scheduler_kwargs: hf_parse.LRSchedulerKwargs) -> Any:
    from transformers.optimization import get_scheduler

    return get_scheduler(scheduler_kwargs.lr_scheduler_type, optimizer,
                         num_warmup_steps=scheduler_kwargs.num_warmup_steps,
                         num_training_steps=scheduler_kwargs.num_training_steps)


def default_load_dataset(data_config_input: Union[Dict[str, Any], utils.AttrDict]) -> Any:
    """``datasets.load_dataset`` from a hub name (with a validation split carved out of train
    when the dataset has none) or from local ``train_file`` / ``validation_file``."""
    import datasets as hf_datasets

    (dc,) = hf_parse.parse_dict_to_dataclasses((hf_parse.DatasetKwargs,), data_config_input)
    if dc.dataset_name is not None:
        ds = hf_datasets.load_dataset(dc.dataset_name, dc.dataset_config_name)
        if "validation" not in ds.keys():
            pct = dc.validation_split_percentage
            if pct is None:
                raise ValueError("dataset has no validation split: set validation_split_percentage")
            ds["validation"] = hf_datasets.load_dataset(dc.dataset_name, dc.dataset_config_name,
                                                        split=f"train[:{pct}%]")
            ds["train"] = hf_datasets.load_dataset(dc.dataset_name, dc.dataset_config_name,
                                                   split=f"train[{pct}%:]")
        return ds
    if dc.train_file is None:
        raise ValueError("give dataset_name or train_file")
    files = {"train": dc.train_file}
    if dc.validation_file is not None:
        files["validation"] = dc.validation_file
    ext = dc.train_file.rsplit(".", 1)[-1]
    return hf_datasets.load_dataset("text" if ext == "txt" else ext, data_files=files)


def remove_unused_columns(model: torch.nn.Module, dataset: Any) -> None:
    """Keep only the dataset columns the model's ``forward`` accepts (plus label columns)."""
    accepted = set(inspect.signature(model.forward).parameters) | {"label", "label_ids"}
    cols = [c for c in dataset.column_names if c in accepted]
    dataset.set_format(type=dataset.format["type"], columns=cols)


class BaseTransformerTrial(det_torch.PyTorchTrial):
    """PyTorchTrial over a transformers model built from hyperparameters: implements
    ``__init__`` (config/tokenizer/model, optimizer, LR schedule, clipping) and ``train_batch``;
    subclasses provide the data loaders and ``evaluate_batch``.

    Required hparams: ``model_mode`` and ``use_apex_amp``; ``num_training_steps`` is derived from
    ``searcher.max_length`` when absent; ``use_pretrained_weights`` defaults to true."""

    def __init__(self, context: det_torch.PyTorchTrialContext) -> None:
        self.context = context
        if not hasattr(self, "hparams"):
            self.hparams = utils.AttrDict(context.get_hparams())
        if not hasattr(self, "data_config"):
            self.data_config = utils.AttrDict(context.get_data_config())
        if not hasattr(self, "exp_config"):
            self.exp_config = utils.AttrDict(context.get_experiment_config())
        self.check_hparams()
        self.config_kwargs, self.tokenizer_kwargs, self.model_kwargs = \
            hf_parse.default_parse_config_tokenizer_model_kwargs(self.hparams)
        opt_kwargs, sched_kwargs = hf_parse.default_parse_optimizer_lr_scheduler_kwargs(self.hparams)
        self.config, self.tokenizer, self.model = build_using_auto(
            self.config_kwargs, self.tokenizer_kwargs, self.hparams.model_mode, self.model_kwargs,
            use_pretrained_weights=self.hparams.use_pretrained_weights)
        self.model = self.context.wrap_model(self.model)
        self.optimizer = self.context.wrap_optimizer(build_default_optimizer(self.model, opt_kwargs))
        if self.hparams.use_apex_amp:
            self.model, self.optimizer = self.context.configure_apex_amp(models=self.model,
                                                                         optimizers=self.optimizer)
        elif self.hparams.get("use_bf16", False):
            self.context.experimental.use_amp(torch.bfloat16)
        self.lr_scheduler = self.context.wrap_lr_scheduler(
            build_default_lr_scheduler(self.optimizer, sched_kwargs),
            det_torch.LRScheduler.StepMode.STEP_EVERY_BATCH)
        self.grad_clip_fn = det_torch.clip_grad_norm(opt_kwargs.max_grad_norm) \
            if opt_kwargs.max_grad_norm and opt_kwargs.max_grad_norm > 0 else None

    def check_hparams(self) -> None:
        if not isinstance(self.hparams, utils.AttrDict):
            self.hparams = utils.AttrDict(self.hparams)
        if "num_training_steps" not in self.hparams:
            self.hparams.num_training_steps = utils.compute_num_training_steps(
                self.context.get_experiment_config(), self.context.get_global_batch_size())
        if "use_pretrained_weights" not in self.hparams:
            logger.warning("use_pretrained_weights not set: loading pretrained weights "
                           "(set it to false to train from scratch)")
            self.hparams.use_pretrained_weights = True
        for hp in ("use_apex_amp", "model_mode", "num_training_steps"):
            if hp not in self.hparams:
                raise ValueError(f"{hp} is a required hyperparameter for BaseTransformerTrial")

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Any:
        outputs = self.model(**batch)
        loss = outputs["loss"] if isinstance(outputs, dict) else outputs[0]
        self.context.backward(loss)
        self.context.step_optimizer(self.optimizer, self.grad_clip_fn)
        return loss
