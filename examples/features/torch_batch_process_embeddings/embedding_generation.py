"""Sharded embedding generation with ``torch_batch_process`` (reference:
examples/features/torch_batch_process_embeddings/bert_embedding_generation.py).

A randomly initialised BERT encoder (no checkpoint download in this environment) embeds a
synthetic tokenised corpus. Every rank processes its shard of the dataset, writes its embeddings
under the shared output checkpoint every ``checkpoint_interval`` batches, and a crashed or
preempted job resumes after the last completed batch. On MI355X the encoder runs in bf16.

Run: ``python embedding_generation.py`` (one process) or under
``python -m determined_clone_amd.launch.torch_distributed`` for one rank per GPU.
"""
from typing import Any, Dict

import torch
import transformers

from determined_clone_amd.pytorch import experimental


class SyntheticCorpus(torch.utils.data.Dataset):
    """Pre-tokenised documents of random length (padded to ``seq``)."""

    def __init__(self, n: int = 256, seq: int = 64, vocab: int = 4096, seed: int = 0) -> None:
        g = torch.Generator().manual_seed(seed)
        self.ids = torch.randint(1, vocab, (n, seq), generator=g)
        lens = torch.randint(seq // 4, seq + 1, (n,), generator=g)
        self.mask = (torch.arange(seq)[None, :] < lens[:, None]).long()
        self.ids = self.ids * self.mask

    def __len__(self) -> int:
        return len(self.ids)

    def __getitem__(self, i: int) -> Dict[str, Any]:
        return {"index": i, "input_ids": self.ids[i], "attention_mask": self.mask[i]}


def build_encoder(hidden: int = 128, layers: int = 2, vocab: int = 4096) -> torch.nn.Module:
    cfg = transformers.BertConfig(vocab_size=vocab, hidden_size=hidden, num_hidden_layers=layers,
                                  num_attention_heads=4, intermediate_size=4 * hidden)
    return transformers.BertModel(cfg)


class EmbeddingProcessor(experimental.TorchBatchProcessor):
    def __init__(self, context: experimental.TorchBatchProcessorContext) -> None:
        self.context = context
        model = build_encoder()
        if torch.cuda.is_available():
            # bf16 + the MFMA attention kernels; padded documents go through key-length masking
            from determined_clone_amd.transformers import use_flash_attention

            model = use_flash_attention(model.to(torch.bfloat16))
        self.model = context.prepare_model_for_inference(model)
        self.indices, self.embeddings = [], []
        self.last_index = 0

    def process_batch(self, batch: Dict[str, Any], batch_idx: int) -> None:
        ids = self.context.to_device(batch["input_ids"])
        mask = self.context.to_device(batch["attention_mask"])
        with torch.no_grad():
            h = self.model(input_ids=ids, attention_mask=mask).last_hidden_state
            m = mask.unsqueeze(-1).to(h.dtype)
            emb = (h * m).sum(1) / m.sum(1).clamp_min(1)  # masked mean pooling
        self.embeddings.append(emb.float().cpu())
        self.indices.append(batch["index"].cpu())
        self.last_index = batch_idx

    def on_checkpoint_start(self) -> None:
        """Flush the embeddings computed since the previous checkpoint into the output storage
        (every rank enters ``upload_path``: with several workers it is a collective)."""
        with self.context.upload_path() as path:
            if self.embeddings:
                torch.save({"index": torch.cat(self.indices),
                            "embedding": torch.cat(self.embeddings)},
                           path / f"embeddings_{self.last_index}.pt")
        self.indices, self.embeddings = [], []

    def on_finish(self) -> None:
        self.on_checkpoint_start()


def main(n_docs: int = 256, batch_size: int = 16, checkpoint_interval: int = 4) -> None:
    experimental.torch_batch_process(EmbeddingProcessor, SyntheticCorpus(n_docs),
                                     batch_size=batch_size,
                                     checkpoint_interval=checkpoint_interval)


if __name__ == "__main__":
    main()
