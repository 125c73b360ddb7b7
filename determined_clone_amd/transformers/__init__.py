"""Hugging Face Trainer integration (reference: `harness/determined/transformers`)."""
from determined_clone_amd.transformers._hf_callback import DetCallback, metric_kind
from determined_clone_amd.transformers._attention import mask_to_key_lengths, use_flash_attention
