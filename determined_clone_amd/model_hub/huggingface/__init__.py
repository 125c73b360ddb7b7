"""Hugging Face transformers integration (reference: ``model_hub/model_hub/huggingface``)."""
from determined_clone_amd.model_hub.huggingface._config_parser import (
    ConfigKwargs, DatasetKwargs, LRSchedulerKwargs, ModelKwargs, OptimizerKwargs, TokenizerKwargs,
    default_parse_config_tokenizer_model_kwargs, default_parse_optimizer_lr_scheduler_kwargs,
    parse_dict_to_dataclasses)
from determined_clone_amd.model_hub.huggingface._trial import (
    MODEL_MODES, BaseTransformerTrial, build_default_lr_scheduler, build_default_optimizer,
    build_using_auto, default_load_dataset, group_parameters_for_optimizer, remove_unused_columns)
