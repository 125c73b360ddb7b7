"""Model hub: ready-made trials for model libraries (reference: ``model_hub/``). ``huggingface``
wraps transformers models as PyTorchTrials; the reference's ``mmdetection`` integration needs
mmcv/mmdet, which are not part of the MI355X image."""
from determined_clone_amd.model_hub import utils
