"""Hugging Face Trainer + DetCallback (reference: examples/hf_trainer_api). A small randomly
initialised GPT-2 (no downloads) trained on synthetic tokens; metrics, checkpoints, searcher
progress and preemption go through the Core API."""
import torch
import transformers

import determined_clone_amd as det
from determined_clone_amd import core
from determined_clone_amd.transformers import DetCallback


class Tokens(torch.utils.data.Dataset):
    def __init__(self, n=2048, seq=128, vocab=1024):
        g = torch.Generator().manual_seed(0)
        self.x = torch.randint(0, vocab, (n, seq), generator=g)

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return {"input_ids": self.x[i], "labels": self.x[i]}


def main() -> None:
    info = det.get_cluster_info()
    hp = info.trial.hparams if info else {"learning_rate": 3e-4}
    model = transformers.GPT2LMHeadModel(transformers.GPT2Config(
        vocab_size=1024, n_positions=128, n_embd=256, n_layer=4, n_head=4, bos_token_id=0, eos_token_id=0))
    args = transformers.TrainingArguments(
        output_dir="/tmp/hf_out", max_steps=200, per_device_train_batch_size=16,
        learning_rate=float(hp["learning_rate"]), eval_strategy="steps", eval_steps=50,
        save_steps=50, logging_steps=10, report_to=[], bf16=torch.cuda.is_available())
    distributed = core.DistributedContext.from_torch_distributed() if args.world_size > 1 else None
    with core.init(distributed=distributed) as core_context:
        cb = DetCallback(core_context, args)
        trainer = transformers.Trainer(model=model, args=args, train_dataset=Tokens(),
                                       eval_dataset=Tokens(128), callbacks=[cb])
        trainer.train(resume_from_checkpoint=args.resume_from_checkpoint)


if __name__ == "__main__":
    main()
