"""Hugging Face ``transformers.Trainer`` integration (reference:
`harness/determined/transformers/_hf_callback.py` DetCallback).

``DetCallback`` plugs a stock HF Trainer into the Core API:

* ``on_log`` routes HF log dicts to training (``loss``, ``learning_rate`` ...) or validation
  (``eval_*``) metrics, once per global step;
* progress is reported per step (searcher unit ``batches``) or per epoch (``epochs``); when the current
  searcher operation's length is reached the callback forces a log + evaluate + save, reports the
  searcher metric and moves to the next operation (or stops training);
* ``on_save`` uploads the step's ``checkpoint-<step>/`` directory (and tensorboard ``runs/``) as a
  sharded Determined checkpoint; on (re)start the latest Determined checkpoint is downloaded into
  ``output_dir`` and passed to the Trainer as ``resume_from_checkpoint``;
* a preemption signal triggers a save and then stops the process after upload.
"""
import json
import logging
import os
from typing import Any, Dict, List, Optional, Tuple

from transformers import TrainerCallback, TrainerControl, TrainerState, TrainingArguments
from transformers.trainer_utils import get_last_checkpoint

from determined_clone_amd import _info

logger = logging.getLogger("determined_clone_amd.transformers")

EVAL_PREFIX = "eval_"
TEST_PREFIX = "test_"
TRAIN_AVG_PREFIX = "train_"
TRAIN = "train_progress"


def metric_kind(logs: Dict[str, Any]) -> str:
    """Classify an HF log dict by its first key (eval_/test_/train_ summary/in-progress train)."""
    for k in logs:
        if k.startswith(EVAL_PREFIX):
            return EVAL_PREFIX
        if k.startswith(TEST_PREFIX):
            return TEST_PREFIX
        if k.startswith(TRAIN_AVG_PREFIX):
            return TRAIN_AVG_PREFIX
        return TRAIN
    return TRAIN


class DetCallback(TrainerCallback):
    def __init__(self, core_context: Any, args: TrainingArguments,
                 filter_metrics: Optional[List[str]] = None,
                 user_data: Optional[Dict[str, Any]] = None) -> None:
        super().__init__()
        self.core_context = core_context
        self.filter_metrics = filter_metrics
        self.user_data = user_data
        info = _info.get_cluster_info()
        if info is None or info.trial is None:
            raise RuntimeError("DetCallback must run as a Determined trial (no cluster info found)")
        self.info = info
        self._restore_latest(args)
        self.last_step = {"train": -1, "eval": -1}
        self.last_metrics: Dict[str, Any] = {}
        self.ops = self.core_context.searcher.operations()
        self.op = next(self.ops)
        self.pending_searcher_update = False
        scfg = info.trial._config["searcher"]
        self.searcher_metric = scfg.get("metric")
        if scfg["name"] == "custom":
            self.unit, self.max_length = "batches", self.op.length
        else:
            (self.unit, self.max_length), = scfg["max_length"].items()
            self._warn_if_mismatched(args)

    # ------------------------------------------------------------------ metrics
    def _filtered(self, logs: Dict[str, Any]) -> Dict[str, Any]:
        if not self.filter_metrics:
            return dict(logs)
        return {k: v for k, v in logs.items() if any(f in k for f in self.filter_metrics)}

    def on_log(self, args: TrainingArguments, state: TrainerState, control: TrainerControl,
               logs: Optional[Dict[str, Any]] = None, **kwargs: Any) -> None:
        if not logs:
            return
        kind = metric_kind(logs)
        metrics = self._filtered(logs)
        step = state.global_step
        if kind == TRAIN and self.last_step["train"] != step:
            if state.is_world_process_zero:
                self.core_context.train.report_training_metrics(steps_completed=step, metrics=metrics)
            self.last_step["train"] = step
        elif kind == EVAL_PREFIX and self.last_step["eval"] != step:
            if state.is_world_process_zero:
                self.core_context.train.report_validation_metrics(steps_completed=step, metrics=metrics)
            self.last_step["eval"] = step
        self.last_metrics.update(metrics)
        if self.pending_searcher_update:
            self._advance_searcher(state, control)
        elif self.core_context.preempt.should_preempt():
            control.should_save = True

    # ------------------------------------------------------------------ progress / searcher
    def on_step_end(self, args: TrainingArguments, state: TrainerState, control: TrainerControl,
                    **kwargs: Any) -> None:
        if state.epoch is None or self.unit != "batches":
            return
        if state.is_world_process_zero:
            self.op.report_progress(state.global_step)
        if state.global_step >= self.op.length:
            self._advance_searcher(state, control)

    def on_epoch_end(self, args: TrainingArguments, state: TrainerState, control: TrainerControl,
                     **kwargs: Any) -> None:
        if state.epoch is None or self.unit != "epochs":
            return
        if state.is_world_process_zero:
            self.op.report_progress(state.epoch)
        if state.epoch >= self.op.length:
            self._advance_searcher(state, control)

    def _advance_searcher(self, state: TrainerState, control: TrainerControl) -> None:
        step = state.global_step
        if not (self.last_step["train"] == step and self.last_step["eval"] == step):
            # ask the Trainer for fresh train + eval metrics and a checkpoint first
            control.should_log = control.should_evaluate = control.should_save = True
            self.pending_searcher_update = True
            return
        if state.is_world_process_zero:
            if self.searcher_metric in self.last_metrics:
                value = self.last_metrics[self.searcher_metric]
            else:
                logger.warning(f"searcher metric {self.searcher_metric!r} not among logged metrics "
                               f"{sorted(self.last_metrics)}; reporting trainer best_metric")
                value = state.best_metric
            self.op.report_completed(value)
        self.pending_searcher_update = False
        try:
            self.op = next(self.ops)
        except StopIteration:
            control.should_training_stop = True

    # ------------------------------------------------------------------ checkpoints
    def on_save(self, args: TrainingArguments, state: TrainerState, control: TrainerControl,
                **kwargs: Any) -> None:
        step_dir = f"checkpoint-{state.global_step}"
        if state.is_world_process_zero and self.user_data is not None:
            os.makedirs(os.path.join(args.output_dir, step_dir), exist_ok=True)
            with open(os.path.join(args.output_dir, step_dir, "my_data.json"), "w") as f:
                json.dump(self.user_data, f)
        md = {"steps_completed": state.global_step, "trial_id": self.info.trial.trial_id}
        self.core_context.checkpoint.upload(
            args.output_dir, metadata=md, shard=True,
            selector=lambda p: p.startswith((f"{step_dir}/", "runs/")))
        if self.core_context.preempt.should_preempt():
            raise SystemExit("preempted after checkpoint upload")

    def _restore_latest(self, args: TrainingArguments) -> None:
        latest = self.info.latest_checkpoint
        if latest is None:
            return
        if args.overwrite_output_dir:
            logger.info("overwrite_output_dir=True: not restoring the latest Determined checkpoint")
            return
        self.core_context.checkpoint.download(latest, args.output_dir)
        args.resume_from_checkpoint = get_last_checkpoint(args.output_dir)
        logger.info(f"resuming from {args.resume_from_checkpoint}")

    def _warn_if_mismatched(self, args: TrainingArguments) -> None:
        trainer_len: Tuple[str, float]
        trainer_len = ("epochs", args.num_train_epochs) if args.max_steps == -1 else ("batches", args.max_steps)
        if trainer_len != (self.unit, self.max_length):
            logger.warning(f"searcher max_length {self.unit}={self.max_length} differs from the HF "
                           f"Trainer's {trainer_len[0]}={trainer_len[1]}; use matching units "
                           "(--max_steps with batches, --num_train_epochs with epochs)")
