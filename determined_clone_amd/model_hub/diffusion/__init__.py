"""Latent-diffusion fine-tuning and generation (reference:
`examples/diffusion/textual_inversion_stable_diffusion/detsd`)."""
from determined_clone_amd.model_hub.diffusion.textual_inversion import (  # noqa: F401
    TextualInversionDataset, TextualInversionPipeline, TextualInversionTrainer,
    load_learned_embeddings)
