"""Image generation with learned concept embeddings (reference:
`examples/diffusion/textual_inversion_stable_diffusion/generate.py`)."""
import logging

from determined_clone_amd.model_hub.diffusion import TextualInversionPipeline

if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    TextualInversionPipeline.generate_on_cluster()
