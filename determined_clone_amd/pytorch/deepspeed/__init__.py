"""DeepSpeedTrial API on the native MI355X ZeRO engine
(reference: `harness/determined/pytorch/deepspeed/__init__.py`)."""
from determined_clone_amd.pytorch.deepspeed._mpu import (ModelParallelUnit, make_data_parallel_mpu,
                                                         make_deepspeed_mpu)
from determined_clone_amd.pytorch.deepspeed._engine import (DeepSpeedConfig, DeepSpeedEngine,
                                                            WarmupCosineLR, WarmupDecayLR, WarmupLR,
                                                            initialize)
from determined_clone_amd.pytorch.deepspeed._trial import (DeepSpeedTrial, DeepSpeedTrialContext,
                                                           DeepSpeedTrialController, Trainer, init,
                                                           overwrite_deepspeed_config,
                                                           run_deepspeed_trial)
from determined_clone_amd.parallel.pipeline import (LayerSpec, PipelineGrid, PipelineModule,
                                                    TiedLayerSpec)
from determined_clone_amd.pytorch.deepspeed._pipe import PipelineEngine
