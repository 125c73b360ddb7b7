"""Textual inversion fine-tuning on the cluster (reference:
`examples/diffusion/textual_inversion_stable_diffusion/finetune.py`)."""
import logging

from determined_clone_amd.model_hub.diffusion import TextualInversionTrainer

if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    TextualInversionTrainer.train_on_cluster()
