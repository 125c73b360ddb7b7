"""DetCallback drives a stock Hugging Face Trainer (tiny random GPT-2, CPU) through the Core API."""
import os

import pytest
import torch

transformers = pytest.importorskip("transformers")

from determined_clone_amd import _info, core  # noqa: E402
from determined_clone_amd.transformers import DetCallback, metric_kind  # noqa: E402


class Tokens(torch.utils.data.Dataset):
    def __init__(self, n=32, seq=16, vocab=64):
        g = torch.Generator().manual_seed(0)
        self.x = torch.randint(0, vocab, (n, seq), generator=g)

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return {"input_ids": self.x[i], "labels": self.x[i]}


def test_metric_kind():
    assert metric_kind({"eval_loss": 1}) == "eval_"
    assert metric_kind({"train_runtime": 1}) == "train_"
    assert metric_kind({"loss": 1}) == "train_progress"


def test_det_callback_reports_metrics_checkpoints_and_searcher(tmp_path):
    cfg = {"searcher": {"name": "single", "metric": "eval_loss", "max_length": {"batches": 6}}}
    info = _info.ClusterInfo("http://127.0.0.1:1", "c", "a", [0], "t", "al", "tok", "TRIAL",
                             trial_info=_info.TrialInfo(7, 1, 0, {}, cfg))
    _info._set_cluster_info(info)
    try:
        ctx = core._dummy_init(checkpoint_storage=str(tmp_path / "ckpts")).__enter__()
        ctx.searcher._length = 6
        seen = {"train": [], "val": [], "completed": []}
        ctx.train.report_training_metrics = lambda steps_completed, metrics, **k: seen["train"].append(steps_completed)
        ctx.train.report_validation_metrics = lambda steps_completed, metrics: seen["val"].append((steps_completed, metrics))
        model = transformers.GPT2LMHeadModel(transformers.GPT2Config(
            vocab_size=64, n_positions=16, n_embd=32, n_layer=1, n_head=2, bos_token_id=0, eos_token_id=0))
        args = transformers.TrainingArguments(
            output_dir=str(tmp_path / "out"), max_steps=6, per_device_train_batch_size=4,
            per_device_eval_batch_size=8, eval_strategy="steps", eval_steps=3, save_steps=3,
            logging_steps=1, report_to=[], use_cpu=True)
        cb = DetCallback(ctx, args, user_data={"note": "hi"})
        orig = cb.op.report_completed
        cb.op.report_completed = lambda m: (seen["completed"].append(m), orig(m))
        trainer = transformers.Trainer(model=model, args=args, train_dataset=Tokens(),
                                       eval_dataset=Tokens(8), callbacks=[cb])
        trainer.train()
    finally:
        _info._set_cluster_info(None)
    assert seen["train"][:3] == [1, 2, 3]
    assert [s for s, _ in seen["val"]] == [3, 6]
    assert seen["completed"] and seen["completed"][0] == seen["val"][-1][1]["eval_loss"]
    stored = os.listdir(tmp_path / "ckpts")
    assert stored, "no checkpoint uploaded"
    found = [os.path.join(r, f) for s in stored for r, _, fs in os.walk(tmp_path / "ckpts" / s) for f in fs]
    assert any(p.endswith("checkpoint-6/my_data.json") for p in found)
