"""GPT-2 DeepSpeedTrial on the native ZeRO engine (reference: examples/deepspeed/gpt_neox/
gpt2_trial.py, which drives GPT-NeoX through DeepSpeed; here ``det_ds.initialize`` builds the
MI355X engine: ZeRO-1/2 over RCCL, fused HIP AdamW, MFMA flash attention, fused LN / GELU / CE).

``hyperparameters.pipe_parallel_size: N`` trains the same GPT as an N-stage pipeline
(``pipe.yaml``; the reference example's ``pipe_parallel_size: 2``);
``hyperparameters.model_parallel_size: M`` shards it Megatron-style over M adjacent ranks
(``tp.yaml``; the reference example's ``model_parallel_size: 2``): heads / MLP columns / vocab
split, gradients averaged over the data-parallel group only; both together (``pipe_tp.yaml``) is
the reference's ``zero1.yaml`` layout: a pipeline of tensor-parallel stages.

The DeepSpeed JSON config is ``ds_config.json`` overlaid with ``hyperparameters.overwrite_deepspeed_args``
(same convention as the reference's ``overwrite_deepspeed_config``). Synthetic token data."""
import json
import os

import torch

from determined_clone_amd import pytorch
from determined_clone_amd.models import gpt2
from determined_clone_amd.pytorch import deepspeed as det_ds


class TokenData(torch.utils.data.Dataset):
    def __init__(self, n: int, seq: int, vocab: int, seed: int) -> None:
        self.n, self.seq, self.vocab, self.seed = n, seq, vocab, seed

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i: int):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        t = torch.randint(0, self.vocab, (self.seq + 1,), generator=g)
        return t[:-1], t[1:]


class GPT2Trial(det_ds.DeepSpeedTrial):
    def __init__(self, context: det_ds.DeepSpeedTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.seq = int(hp.get("seq_len", 1024))
        cfg = gpt2.config_for(hp.get("model", "gpt2-medium"), max_seq_len=self.seq)
        base = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ds_config.json")))
        ds_config = det_ds.overwrite_deepspeed_config(base, hp.get("overwrite_deepspeed_args", {}))
        self.pipe = int(hp.get("pipe_parallel_size", 0))
        mp_size = int(hp.get("model_parallel_size", 1))
        grid = None
        if mp_size > 1 and self.pipe >= 1:
            # the reference's gpt_neox zero1.yaml layout: pipe_parallel_size x model_parallel_size
            from determined_clone_amd.models import gpt2_tp
            from determined_clone_amd.parallel.tensor import ModelParallelGrid

            g = ModelParallelGrid(model_parallel_size=mp_size, pipe_parallel_size=self.pipe)
            model = det_ds.PipelineModule(gpt2_tp.pipeline_specs_tp(cfg, g.mp_group),
                                          num_stages=self.pipe, grid=g,
                                          loss_fn=gpt2_tp.PipelineLossTP(cfg, g.mp_group),
                                          activation_checkpoint_interval=int(
                                              hp.get("activation_checkpoint_interval", 0)))
        elif mp_size > 1:
            from determined_clone_amd.models.gpt2_tp import TPGPT
            from determined_clone_amd.parallel.tensor import ModelParallelGrid

            grid = ModelParallelGrid(model_parallel_size=mp_size)
            model = TPGPT(cfg, grid.get_model_parallel_group())
        elif self.pipe >= 1:
            # GPT-NeoX style pipeline (reference gpt_neox/zero1.yaml: pipe_parallel_size 2):
            # embedding | blocks | final norm | tied LM head over `pipe` stages, 1F1B schedule
            model = det_ds.PipelineModule(gpt2.pipeline_specs(cfg), num_stages=self.pipe,
                                          loss_fn=gpt2.pipeline_loss, seed_layers=True,
                                          activation_checkpoint_interval=int(
                                              hp.get("activation_checkpoint_interval", 0)))
        else:
            model = gpt2.GPT(cfg)
        engine, _, _, _ = det_ds.initialize(model=model, config=ds_config, mpu=grid)
        self.engine = context.wrap_model_engine(engine)
        if grid is not None:
            # every TP rank of a data-parallel group reads the same shard of the data
            context.set_mpu(det_ds.ModelParallelUnit(
                data_parallel_rank=grid.get_data_parallel_rank(),
                data_parallel_world_size=grid.get_data_parallel_world_size(),
                should_report_metrics=True, should_build_data_loader=True))
        self.vocab = cfg.vocab_size

    def train_batch(self, it, epoch_idx, batch_idx):
        if self.context.use_pipeline_parallel:
            return {"loss": self.engine.train_batch(it)}
        x, y = self.context.to_device(next(it))
        _, loss = self.engine(x, y)
        self.engine.backward(loss)
        self.engine.step()
        return {"loss": loss}

    def evaluate_batch(self, it, batch_idx):
        if self.context.use_pipeline_parallel:
            return {"lm_loss": self.engine.eval_batch(it)}
        x, y = self.context.to_device(next(it))
        with torch.no_grad():
            _, loss = self.engine(x, y)
        return {"lm_loss": loss}

    def build_training_data_loader(self):
        return pytorch.DataLoader(TokenData(1 << 20, self.seq, self.vocab, 0),
                                  batch_size=self.context.train_micro_batch_size_per_gpu)

    def build_validation_data_loader(self):
        return pytorch.DataLoader(TokenData(64, self.seq, self.vocab, 1),
                                  batch_size=self.context.train_micro_batch_size_per_gpu)
