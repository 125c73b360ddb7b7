"""Textual inversion on the latent-diffusion model family, driven by the Core API.

Reference: `examples/diffusion/textual_inversion_stable_diffusion/detsd/trainer.py` and
`pipeline.py` (``DetSDTextualInversionTrainer.train_on_cluster`` / ``DetSDTextualInversionPipeline
.generate_on_cluster``). Behaviour kept: each concept string becomes ``len(initializer tokens)``
new placeholder tokens whose embeddings start as copies of the initializer tokens' rows and are the
ONLY trainable parameters (``ExtendedEmbedding``); a step = VAE-encode images to latents, add DDPM
noise at random timesteps, predict the noise with the UNet conditioned on the placeholder prompt,
MSE loss (+ optional embedding-norm and hidden-state regularisers), gradient accumulation;
metrics every ``metric_report_freq`` steps, checkpoints every ``checkpoint_freq`` (learned
embeddings dict + optimizer state + metadata), preemption, resume; generation loads learned
embeddings from checkpoints (by storage id) or local files and writes images to TensorBoard and
checkpoints.

MI355X-specific: the frozen UNet / VAE / text encoder run in bf16 NHWC on the GPU with the MFMA
flash-attention kernels (``models/diffusion.py``); the tiny trainable table is fp32 and optimised
with the fused HIP Adam (``ops/optim.py``); data-parallel slots all-reduce just that table.

Base weights: no pretrained checkpoint is available offline, so the frozen networks are
random-initialised from ``model_seed`` -- the same seed in the fine-tuning and the generation
experiments gives the same "pretrained" model, so learned embeddings transfer between them.
"""
import json
import logging
import math
import os
import pathlib
import random
from typing import Any, Dict, List, Optional, Sequence

import torch
import torch.nn.functional as F

from determined_clone_amd.models import diffusion as ldm

logger = logging.getLogger("determined_clone_amd.model_hub.diffusion")

TEMPLATES = {
    "object": ["a photo of a {}", "a rendering of a {}", "a cropped photo of the {}",
               "the photo of a {}", "a close-up photo of a {}", "a bright photo of the {}",
               "a good photo of a {}", "a photo of one {}", "a rendition of the {}"],
    "style": ["a painting in the style of {}", "a rendering in the style of {}",
              "a cropped painting in the style of {}", "the painting in the style of {}",
              "a clean painting in the style of {}", "a picture in the style of {}",
              "a cool painting in the style of {}", "a small painting in the style of {}"],
}


class TextualInversionDataset(torch.utils.data.Dataset):
    """(prompt, image in [-1, 1]) pairs for each concept. Images come from the concept's
    directory (any PIL-readable file, resized to ``img_size``); a missing or empty directory
    yields deterministic synthetic images (smooth random fields) so the pipeline runs without
    data."""

    def __init__(self, img_dirs: Sequence[str], concept_strs: Sequence[str],
                 learnable_properties: Sequence[str], img_size: int = 512, flip_p: float = 0.0,
                 repeats: int = 100, seed: int = 0) -> None:
        if not (len(img_dirs) == len(concept_strs) == len(learnable_properties)):
            raise ValueError("img_dirs, concept_strs and learnable_properties must have equal lengths")
        for p in learnable_properties:
            if p not in TEMPLATES:
                raise ValueError(f"learnable_properties must be one of {list(TEMPLATES)}, not {p}")
        self.items: List[Any] = []
        g = torch.Generator().manual_seed(seed)
        for d, concept, prop in zip(img_dirs, concept_strs, learnable_properties):
            imgs = self._load_dir(d, img_size) or [self._synthetic(img_size, g) for _ in range(4)]
            for img in imgs:
                self.items.append((concept, prop, img))
        self.repeats = repeats
        self.flip_p = flip_p

    @staticmethod
    def _load_dir(d: str, size: int) -> List[torch.Tensor]:
        if not d or not os.path.isdir(d):
            return []
        from PIL import Image

        out = []
        for name in sorted(os.listdir(d)):
            try:
                im = Image.open(os.path.join(d, name)).convert("RGB").resize((size, size), Image.BICUBIC)
            except Exception:
                continue
            t = torch.frombuffer(bytearray(im.tobytes()), dtype=torch.uint8).view(size, size, 3)
            out.append(t.permute(2, 0, 1).float() / 127.5 - 1.0)
        return out

    @staticmethod
    def _synthetic(size: int, g: torch.Generator) -> torch.Tensor:
        low = torch.rand(1, 3, 8, 8, generator=g) * 2 - 1
        return F.interpolate(low, size=(size, size), mode="bicubic", align_corners=False)[0].clamp(-1, 1)

    def __len__(self) -> int:
        return len(self.items) * self.repeats

    def __getitem__(self, i: int):
        concept, prop, img = self.items[i % len(self.items)]
        rng = random.Random(i)
        prompt = rng.choice(TEMPLATES[prop]).format(concept)
        if self.flip_p and rng.random() < self.flip_p:
            img = img.flip(-1)
        return prompt, img


class TextualInversionTrainer:
    def __init__(self, concept_strs: Sequence[str], initializer_strs: Sequence[str],
                 learnable_properties: Sequence[str], img_dirs: Sequence[str],
                 model_preset: str = "tiny", model_seed: int = 0, img_size: int = 64,
                 train_batch_size: int = 1, gradient_accumulation_steps: int = 1,
                 optimizer_name: str = "adam", learning_rate: float = 5e-4,
                 checkpoint_freq: int = 50, metric_report_freq: int = 50,
                 norm_reg_weight: float = 0.0, hidden_reg_weight: float = 0.0,
                 num_train_timesteps: int = 1000, beta_start: float = 0.00085,
                 beta_end: float = 0.012, beta_schedule: str = "scaled_linear",
                 generate_training_images: bool = False, inference_prompts: Sequence[str] = (),
                 num_pipeline_calls: int = 1, inference_steps: int = 25, guidance_scale: float = 7.5,
                 inference_scheduler_name: str = "pndm", seed: int = 2147483647,
                 device: Optional[torch.device] = None, rank: int = 0, world: int = 1) -> None:
        self.concept_strs = list(concept_strs)
        self.initializer_strs = list(initializer_strs)
        self.learnable_properties = list(learnable_properties)
        self.img_dirs = list(img_dirs)
        self.img_size = img_size
        self.train_batch_size = train_batch_size
        self.grad_accum = gradient_accumulation_steps
        self.checkpoint_freq = checkpoint_freq
        self.metric_report_freq = metric_report_freq
        self.norm_reg_weight = norm_reg_weight
        self.hidden_reg_weight = hidden_reg_weight
        self.generate_training_images = generate_training_images
        self.inference_prompts = list(inference_prompts)
        self.num_pipeline_calls = num_pipeline_calls
        self.inference_steps = inference_steps
        self.guidance_scale = guidance_scale
        self.inference_scheduler_name = inference_scheduler_name
        self.beta = (beta_start, beta_end, beta_schedule)
        self.rank, self.world = rank, world
        self.device = device or (torch.device("cuda", torch.cuda.current_device())
                                 if torch.cuda.is_available() else torch.device("cpu"))
        self.steps_completed = 0
        self.metrics_history: Dict[str, List[float]] = {"loss": [], "noise_pred_loss": []}
        self.last_mean_loss: Optional[float] = None

        torch.manual_seed(model_seed)
        self.model = ldm.LatentDiffusion(ldm.LDMConfig.preset(model_preset))
        self.concept_to_dummy_strs: Dict[str, str] = {}
        self.concept_to_dummy_ids: Dict[str, List[int]] = {}
        self._add_new_tokens()
        self._freeze_layers()
        dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.model.to_mi355x_layout(self.device, dtype)
        emb = self.model.text_encoder.token_embedding.new_embedding
        emb.float()  # the trainable rows stay fp32
        self.init_embedding_norm_mean = float(emb.weight.detach().norm(dim=1).mean())
        self.optimizer = self._build_optimizer(optimizer_name, learning_rate)
        self.scheduler = ldm.DDPMScheduler(num_train_timesteps, beta_start, beta_end, beta_schedule)
        self.num_train_timesteps = num_train_timesteps
        self.gen = torch.Generator(device="cpu").manual_seed(seed + rank)
        ds = TextualInversionDataset(self.img_dirs, self.concept_strs, self.learnable_properties,
                                     img_size, seed=model_seed)
        sampler = torch.utils.data.DistributedSampler(ds, world, rank, shuffle=True, seed=seed) \
            if world > 1 else torch.utils.data.RandomSampler(ds, generator=torch.Generator().manual_seed(seed))
        self.loader = torch.utils.data.DataLoader(ds, batch_size=train_batch_size, sampler=sampler,
                                                  drop_last=True)

    # ------------------------------------------------------------------ setup
    def _add_new_tokens(self) -> None:
        tok = self.model.tokenizer
        enc = self.model.text_encoder
        rows = []
        for concept, init in zip(self.concept_strs, self.initializer_strs):
            init_ids = tok.word_ids(init)
            if not init_ids:
                raise ValueError(f"initializer string for {concept!r} has no tokens")
            dummies = [f"<{concept}_{i}>" for i in range(len(init_ids))]
            ids = tok.add_tokens(dummies)
            self.concept_to_dummy_strs[concept] = " ".join(dummies)
            self.concept_to_dummy_ids[concept] = ids
            rows.append(enc.token_embedding.weight.detach()[torch.tensor(init_ids)].clone())
            logger.info(f"added {len(ids)} tokens for {concept!r}")
        enc.add_concept_rows(torch.cat(rows, 0))

    def _freeze_layers(self) -> None:
        for p in self.model.parameters():
            p.requires_grad_(False)
        for p in self.model.text_encoder.token_embedding.new_embedding.parameters():
            p.requires_grad_(True)

    def _build_optimizer(self, name: str, lr: float) -> torch.optim.Optimizer:
        params = list(self.model.text_encoder.token_embedding.new_embedding.parameters())
        if self.device.type == "cuda":
            from determined_clone_amd.ops import optim as fopt

            if name == "adam":
                return fopt.FusedAdam(params, lr=lr)
            if name == "sgd":
                return fopt.FusedSGD(params, lr=lr)
        if name == "adam":
            return torch.optim.Adam(params, lr=lr)
        if name == "sgd":
            return torch.optim.SGD(params, lr=lr)
        raise ValueError(f"optimizer_name must be adam or sgd, not {name!r}")

    def replace_concepts_with_dummies(self, text: str) -> str:
        for concept, dummies in self.concept_to_dummy_strs.items():
            text = text.replace(concept, dummies)
        return text

    def replace_concepts_with_initializers(self, text: str) -> str:
        for concept, init in zip(self.concept_strs, self.initializer_strs):
            text = text.replace(concept, init)
        return text

    @property
    def new_embedding(self) -> torch.nn.Embedding:
        return self.model.text_encoder.token_embedding.new_embedding

    # ------------------------------------------------------------------ training
    def train_one_batch(self, prompts: Sequence[str], imgs: torch.Tensor) -> float:
        m = self.model
        dtype = m.unet.conv_in.weight.dtype
        imgs = imgs.to(self.device, dtype)
        if self.device.type == "cuda":
            imgs = imgs.contiguous(memory_format=torch.channels_last)
        with torch.no_grad():
            latents = m.vae.sample_latents(imgs).float()
            noise = torch.randn(latents.shape, generator=self.gen).to(self.device)
            t = torch.randint(0, self.num_train_timesteps, (latents.shape[0],), generator=self.gen).to(self.device)
            noisy = self.scheduler.add_noise(latents, noise, t).to(dtype)
        dummy = [self.replace_concepts_with_dummies(p) for p in prompts]
        ctx = m.encode_text(dummy)
        pred = m.unet(noisy, t, ctx).float()
        loss = F.mse_loss(pred, noise)
        total = loss
        self.metrics_history["noise_pred_loss"].append(float(loss.detach()))
        if self.norm_reg_weight:
            norms = self.new_embedding.weight.norm(dim=1)
            reg = self.norm_reg_weight * (self.init_embedding_norm_mean - norms).pow(2).sum()
            self.metrics_history.setdefault("norm_reg_loss", []).append(float(reg.detach()))
            total = total + reg
        if self.hidden_reg_weight:
            with torch.no_grad():
                init_ctx = m.encode_text([self.replace_concepts_with_initializers(p) for p in prompts])
            reg = self.hidden_reg_weight * F.mse_loss(ctx.float(), init_ctx.float())
            self.metrics_history.setdefault("hidden_reg_loss", []).append(float(reg.detach()))
            total = total + reg
        (total / self.grad_accum).backward()
        self.metrics_history["loss"].append(float(total.detach()))
        return float(total.detach())

    def optimizer_step(self) -> None:
        w = self.new_embedding.weight
        if self.world > 1 and w.grad is not None:
            import torch.distributed as dist

            dist.all_reduce(w.grad)
            w.grad.div_(self.world)
        self.optimizer.step()
        self.optimizer.zero_grad()

    def train_steps(self, target_steps: int, on_step=None) -> None:
        """Run optimizer steps until ``steps_completed == target_steps`` (``on_step()`` after each;
        returning True stops early)."""
        while self.steps_completed < target_steps:
            micro = 0
            for prompts, imgs in self.loader:
                self.train_one_batch(prompts, imgs)
                micro += 1
                if micro % self.grad_accum:
                    continue
                self.optimizer_step()
                self.steps_completed += 1
                if on_step is not None and on_step():
                    return
                if self.steps_completed >= target_steps:
                    return

    def pop_metrics(self) -> Dict[str, float]:
        out = {k: sum(v) / len(v) for k, v in self.metrics_history.items() if v}
        for v in self.metrics_history.values():
            v.clear()
        if "loss" in out:
            self.last_mean_loss = out["loss"]
        return out

    # ------------------------------------------------------------------ checkpoints
    def learned_embeddings_dict(self) -> Dict[str, Any]:
        w = self.new_embedding.weight.detach().float().cpu()
        out, off = {}, 0
        for concept, init in zip(self.concept_strs, self.initializer_strs):
            n = len(self.concept_to_dummy_ids[concept])
            out[concept] = {"initializer_strs": init, "learned_embeddings": w[off:off + n].clone()}
            off += n
        return out

    def save(self, path: pathlib.Path, trial_id: Optional[int] = None) -> None:
        torch.save(self.learned_embeddings_dict(), path / "learned_embeddings_dict.pt")
        torch.save(self.optimizer.state_dict(), path / "optimizer_state_dict.pt")
        with open(path / "metadata.json", "w") as f:
            json.dump({"steps_completed": self.steps_completed, "trial_id": trial_id}, f)

    def restore(self, path: pathlib.Path, trial_id: Optional[int] = None) -> None:
        d = torch.load(path / "learned_embeddings_dict.pt", weights_only=True)
        with torch.no_grad():
            rows = torch.cat([d[c]["learned_embeddings"] for c in self.concept_strs], 0)
            self.new_embedding.weight.copy_(rows.to(self.new_embedding.weight))
        with open(path / "metadata.json") as f:
            md = json.load(f)
        if trial_id is None or md.get("trial_id") == trial_id:
            # same trial: continue where it stopped (a fork starts its step count over)
            self.steps_completed = int(md["steps_completed"])
            self.optimizer.load_state_dict(torch.load(path / "optimizer_state_dict.pt", weights_only=True))

    # ------------------------------------------------------------------ images
    def generate(self, prompts: Sequence[str], seed: int = 0) -> torch.Tensor:
        pipe = ldm.LatentDiffusionPipeline(self.model, self.inference_scheduler_name, *self.beta)
        g = torch.Generator(device="cpu").manual_seed(seed)
        return pipe([self.replace_concepts_with_dummies(p) for p in prompts],
                    self.inference_steps, self.guidance_scale, self.img_size, self.img_size, g)

    # ------------------------------------------------------------------ on-cluster entry point
    @classmethod
    def train_on_cluster(cls) -> None:
        from determined_clone_amd import core, get_cluster_info
        from determined_clone_amd.tensorboard import EventFileWriter

        info = get_cluster_info()
        assert info is not None, "train_on_cluster() must run on a cluster (use the trainer directly)"
        hp = info.trial.hparams
        distributed = None
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            distributed = core.DistributedContext.from_torch_distributed()
        with core.init(distributed=distributed, tensorboard_mode=core.TensorboardMode.MANUAL) as ctx:
            rank, world = ctx.distributed.rank, ctx.distributed.size
            if torch.cuda.is_available():
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
            trainer = cls(**hp.get("concepts", {}), **hp.get("model", {}), **hp.get("training", {}),
                          **hp.get("inference", {}), rank=rank, world=world)
            trial_id = info.trial.trial_id
            if info.latest_checkpoint is not None:
                with ctx.checkpoint.restore_path(info.latest_checkpoint) as path:
                    trainer.restore(pathlib.Path(path), trial_id)
            tb = EventFileWriter(str(ctx.train.get_tensorboard_path())) if rank == 0 else None

            def checkpoint() -> None:
                if rank == 0:  # the learned table is identical on every rank (all-reduced grads)
                    with ctx.checkpoint.store_path({"steps_completed": trainer.steps_completed}) as (path, _):
                        trainer.save(pathlib.Path(path), trial_id)

            for op in ctx.searcher.operations():
                state = {"stop": False}

                def on_step() -> bool:
                    end = trainer.steps_completed >= op.length
                    if end or trainer.steps_completed % trainer.metric_report_freq == 0:
                        metrics = trainer.pop_metrics()
                        if rank == 0:
                            ctx.train.report_training_metrics(trainer.steps_completed, metrics)
                            op.report_progress(trainer.steps_completed)
                    if end or trainer.steps_completed % trainer.checkpoint_freq == 0:
                        checkpoint()
                        if trainer.generate_training_images and tb is not None and trainer.inference_prompts:
                            for call in range(trainer.num_pipeline_calls):
                                imgs = trainer.generate(trainer.inference_prompts, seed=call)
                                for i, im in enumerate(imgs):
                                    tb.add_image(f"prompt_{i}/call_{call}", im.numpy(), trainer.steps_completed)
                            tb.flush()
                            ctx.train.upload_tensorboard_files()
                        if ctx.preempt.should_preempt():
                            state["stop"] = True
                            return True
                    return False

                trainer.train_steps(op.length, on_step)
                if state["stop"]:
                    return
                if rank == 0:
                    op.report_completed(trainer.last_mean_loss if trainer.last_mean_loss is not None else math.nan)


def load_learned_embeddings(paths: Sequence[str], filename: str = "learned_embeddings_dict.pt") -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for p in paths:
        f = os.path.join(p, filename) if os.path.isdir(p) else p
        out.update(torch.load(f, weights_only=True))
    return out


class TextualInversionPipeline:
    """Generation with learned concept embeddings (reference: ``detsd/pipeline.py``)."""

    def __init__(self, learned: Dict[str, Any], model_preset: str = "tiny", model_seed: int = 0,
                 scheduler_name: str = "pndm", beta_start: float = 0.00085, beta_end: float = 0.012,
                 beta_schedule: str = "scaled_linear", use_bf16: bool = True,
                 device: Optional[torch.device] = None) -> None:
        self.device = device or (torch.device("cuda", torch.cuda.current_device())
                                 if torch.cuda.is_available() else torch.device("cpu"))
        torch.manual_seed(model_seed)
        self.model = ldm.LatentDiffusion(ldm.LDMConfig.preset(model_preset))
        self.concept_to_dummy: Dict[str, str] = {}
        rows = []
        for concept, d in learned.items():
            emb = d["learned_embeddings"]
            dummies = [f"<{concept}_{i}>" for i in range(emb.shape[0])]
            self.model.tokenizer.add_tokens(dummies)
            self.concept_to_dummy[concept] = " ".join(dummies)
            rows.append(emb)
        if rows:
            self.model.text_encoder.add_concept_rows(torch.cat(rows, 0).float())
        dtype = torch.bfloat16 if (self.device.type == "cuda" and use_bf16) else torch.float32
        self.model.to_mi355x_layout(self.device, dtype)
        self.pipe = ldm.LatentDiffusionPipeline(self.model, scheduler_name, beta_start, beta_end, beta_schedule)

    def __call__(self, prompt: Sequence[str], num_inference_steps: int = 50, guidance_scale: float = 7.5,
                 height: int = 64, width: int = 64, seed: int = 0) -> torch.Tensor:
        texts = []
        for p in prompt:
            for concept, dummy in self.concept_to_dummy.items():
                p = p.replace(concept, dummy)
            texts.append(p)
        g = torch.Generator(device="cpu").manual_seed(seed)
        return self.pipe(texts, num_inference_steps, guidance_scale, height, width, g)

    @classmethod
    def generate_on_cluster(cls) -> None:
        from determined_clone_amd import core, get_cluster_info
        from determined_clone_amd.tensorboard import EventFileWriter

        info = get_cluster_info()
        assert info is not None, "generate_on_cluster() must run on a cluster"
        hp = info.trial.hparams
        distributed = None
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            distributed = core.DistributedContext.from_torch_distributed()
        with core.init(distributed=distributed, tensorboard_mode=core.TensorboardMode.MANUAL) as ctx:
            rank = ctx.distributed.rank
            pcfg = dict(hp.get("pipeline", {}))
            fname = pcfg.pop("learned_embeddings_filename", "learned_embeddings_dict.pt")
            paths = list(hp.get("local_checkpoint_paths") or [])
            learned: Dict[str, Any] = {}
            for uuid in hp.get("uuids") or []:
                with ctx.checkpoint.restore_path(uuid) as p:
                    learned.update(load_learned_embeddings([str(p)], fname))
            learned.update(load_learned_embeddings(paths, fname))
            pipe = cls(learned, **pcfg)
            call = dict(hp.get("call_kwargs", {}))
            bs = int(hp.get("batch_size", 1))
            seed = int(hp.get("main_process_generator_seed", 0)) + rank
            save_freq = int(hp.get("save_freq", 0))
            tb = EventFileWriter(str(ctx.train.get_tensorboard_path()))
            steps, pending = 0, []
            for op in ctx.searcher.operations():
                while steps < op.length:
                    imgs = pipe([call.get("prompt", "")] * bs, int(call.get("num_inference_steps", 50)),
                                float(call.get("guidance_scale", 7.5)), int(call.get("height", 64)),
                                int(call.get("width", 64)), seed + 1000 * steps)
                    for i, im in enumerate(imgs):
                        tb.add_image(f"rank_{rank}/img_{i}", im.numpy(), steps)
                        pending.append(im)
                    steps += 1
                    tb.flush()
                    ctx.train.upload_tensorboard_files()
                    if save_freq and (steps % save_freq == 0 or steps == op.length):
                        from PIL import Image

                        with ctx.checkpoint.store_path({"steps_completed": steps}, shard=True) as (path, _):
                            for j, im in enumerate(pending):
                                Image.fromarray(im.numpy()).save(os.path.join(path, f"rank{rank}_{steps}_{j}.png"))
                        pending = []
                    if rank == 0:
                        op.report_progress(steps)
                    if ctx.preempt.should_preempt():
                        return
                if rank == 0:
                    op.report_completed(0.0)
