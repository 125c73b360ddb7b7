"""Latent-diffusion model family + textual inversion (reference:
`examples/diffusion/textual_inversion_stable_diffusion`): shapes, schedulers (exact x0 recovery
under a perfect noise predictor), tokenizer, only-concept-rows training, checkpoint round trip,
and the fine-tune -> generate experiments on an in-process cluster."""
import base64
import glob
import os
import shutil
import tempfile
import time

import pytest
import torch
import yaml

from determined_clone_amd.models import diffusion as ldm
from determined_clone_amd.model_hub.diffusion import (TextualInversionPipeline,
                                                       TextualInversionTrainer, load_learned_embeddings)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples", "diffusion", "textual_inversion")


def test_shapes_and_param_counts():
    torch.manual_seed(0)
    m = ldm.LatentDiffusion(ldm.LDMConfig.preset("tiny"))
    x = torch.randn(2, 3, 64, 64)
    z = m.vae.sample_latents(x)
    assert z.shape == (2, 4, 8, 8)
    ctx = m.encode_text(["a photo of a cat", ""])
    assert ctx.shape == (2, 16, 64)
    assert m.unet(z, torch.tensor([1, 999]), ctx).shape == z.shape
    assert m.vae.decode(z).shape == x.shape
    sd = ldm.LDMConfig.preset("sd2-base")
    n = sum(p.numel() for p in ldm.UNet2DCondition(sd.unet).parameters())
    assert 860e6 < n < 870e6  # the SD-2 UNet shape (865.9M)


def test_tokenizer_added_tokens_and_padding():
    tok = ldm.HashTokenizer(1000, 8)
    ids = tok.add_tokens(["<cat_0>", "<cat_1>"])
    assert ids == [1000, 1001] and len(tok) == 1002
    row = tok(["a photo of <cat_0> <cat_1>"])[0].tolist()
    assert row[0] == tok.bos and row[4:6] == [1000, 1001] and row[6] == tok.eos
    assert row[7] == tok.pad and len(row) == 8
    assert tok(["x " * 20])[0].tolist()[-1] == tok.eos  # truncation keeps EOS


@pytest.mark.parametrize("name", ["ddim", "pndm"])
def test_samplers_recover_x0_with_perfect_noise_prediction(name):
    """With eps_theta(x_t, t) = the true eps of x_t = sqrt(a_t) x0 + sqrt(1 - a_t) eps, every
    DDIM / PLMS step stays on that trajectory and lands on x0."""
    sch = ldm.SCHEDULERS[name]()
    torch.manual_seed(0)
    x0 = torch.randn(2, 4, 8, 8, dtype=torch.float64)
    eps = torch.randn_like(x0)
    ts = sch.set_timesteps(20)
    a = float(sch.alphas_cumprod[ts[0]])
    x = a ** 0.5 * x0 + (1 - a) ** 0.5 * eps
    for t in ts:
        x = sch.step(eps, t, x)
    a0 = float(sch.alphas_cumprod[0])
    torch.testing.assert_close(x, a0 ** 0.5 * x0 + (1 - a0) ** 0.5 * eps, rtol=1e-6, atol=1e-6)


def test_ddpm_add_noise():
    sch = ldm.DDPMScheduler()
    x0, n = torch.ones(3, 2), torch.zeros(3, 2)
    out = sch.add_noise(x0, n, torch.tensor([0, 500, 999]))
    assert torch.allclose(out[:, 0], sch.alphas_cumprod[[0, 500, 999]].sqrt().float())
    assert sch.betas[0] == pytest.approx(0.00085) and sch.betas[-1] == pytest.approx(0.012)


def _trainer(**kw):
    args = dict(concept_strs=["det-logo"], initializer_strs=["brain logo"],
                learnable_properties=["object"], img_dirs=["/nonexistent"], model_preset="tiny",
                img_size=64, train_batch_size=2, learning_rate=1e-2, device=torch.device("cpu"))
    args.update(kw)
    return TextualInversionTrainer(**args)


def test_textual_inversion_trains_only_concept_rows(tmp_path):
    tr = _trainer(gradient_accumulation_steps=2, norm_reg_weight=0.1, hidden_reg_weight=0.1)
    assert tr.concept_to_dummy_strs["det-logo"] == "<det-logo_0> <det-logo_1>"
    enc = tr.model.text_encoder
    base = enc.token_embedding.original.weight.detach().clone()
    new0 = tr.new_embedding.weight.detach().clone()
    init_ids = tr.model.tokenizer.word_ids("brain logo")
    torch.testing.assert_close(new0, base[torch.tensor(init_ids)])  # initialised from initializers
    unet0 = [p.detach().clone() for p in tr.model.unet.parameters()]
    tr.train_steps(3)
    assert tr.steps_completed == 3
    m = tr.pop_metrics()
    assert {"loss", "noise_pred_loss", "norm_reg_loss", "hidden_reg_loss"} <= set(m)
    assert torch.isfinite(torch.tensor(m["loss"]))
    assert torch.equal(enc.token_embedding.original.weight, base)
    assert all(torch.equal(a, b) for a, b in zip(unet0, tr.model.unet.parameters()))
    assert not torch.equal(tr.new_embedding.weight, new0)
    # checkpoint round trip (weights_only loads)
    tr.save(tmp_path, trial_id=7)
    tr2 = _trainer()
    tr2.restore(tmp_path, trial_id=7)
    assert tr2.steps_completed == 3
    torch.testing.assert_close(tr2.new_embedding.weight, tr.new_embedding.weight)
    learned = load_learned_embeddings([str(tmp_path)])
    assert learned["det-logo"]["learned_embeddings"].shape == (2, 64)
    # generation with the learned concept
    pipe = TextualInversionPipeline(learned, model_preset="tiny", device=torch.device("cpu"))
    imgs = pipe(["a photo of a det-logo"], num_inference_steps=3, height=64, width=64)
    assert imgs.shape == (1, 64, 64, 3) and imgs.dtype == torch.uint8
    # the same model_seed rebuilds the same frozen base model
    assert torch.equal(pipe.model.unet.conv_in.weight, tr.model.unet.conv_in.weight)


@pytest.fixture(scope="module")
def cluster():
    from determined_clone_amd.agent import Agent
    from determined_clone_amd.common.api import Session
    from determined_clone_amd.master import Master, MasterServer

    tmp = tempfile.mkdtemp(prefix="det-sd-")
    m = Master(os.path.join(tmp, "m.db"), checkpoint_storage={"type": "shared_fs", "host_path": os.path.join(tmp, "ckpt")})
    srv = MasterServer(m, "127.0.0.1", 0).start()
    agent = Agent(m.master_url, "agent-0", artificial_slots=2).start_background()
    s = Session(m.master_url)
    s.token = s.post("/api/v1/auth/login", {"username": "admin", "password": ""})["token"]
    yield s, tmp
    agent.stop()
    srv.stop()
    shutil.rmtree(tmp, ignore_errors=True)


def _run(s, cfg, timeout=400):
    from determined_clone_amd.util import tar_directory

    body = {"config": cfg, "model_definition": base64.b64encode(tar_directory(EX)).decode()}
    eid = s.post("/api/v1/experiments", body)["experiment"]["id"]
    t0 = time.time()
    while time.time() - t0 < timeout:
        st = s.get(f"/api/v1/experiments/{eid}")["experiment"]["state"]
        if st in ("COMPLETED", "CANCELED", "ERROR"):
            return eid, st
        time.sleep(0.5)
    raise TimeoutError(st)


def test_finetune_then_generate_on_cluster(cluster):
    s, tmp = cluster
    cfg = yaml.safe_load(open(os.path.join(EX, "finetune_const.yaml")))
    cfg["entrypoint"] = "python3 finetune.py"
    cfg["resources"]["slots_per_trial"] = 1
    cfg["searcher"]["max_length"] = 4
    hp = cfg["hyperparameters"]
    hp["model"].update(model_preset="tiny", img_size=64)
    hp["training"].update(checkpoint_freq=2, metric_report_freq=2, gradient_accumulation_steps=1)
    hp["inference"].update(inference_steps=2, num_pipeline_calls=1, inference_prompts=["a det-logo"])
    eid, st = _run(s, cfg)
    assert st == "COMPLETED"
    t = s.get(f"/api/v1/experiments/{eid}/trials")["trials"][0]
    ms = s.get(f"/api/v1/trials/{t['id']}/metrics", params={"group": "training"})["metrics"]
    assert [m["steps_completed"] for m in ms] == [2, 4]
    ckpts = s.get(f"/api/v1/trials/{t['id']}/checkpoints")["checkpoints"]
    assert len(ckpts) == 2
    uuid = ckpts[-1]["uuid"]
    tb = glob.glob(os.path.join(tmp, "ckpt", "**", "events.out.tfevents.*"), recursive=True)
    assert tb  # training images written to tensorboard storage

    g = yaml.safe_load(open(os.path.join(EX, "generate_grid.yaml")))
    g["entrypoint"] = "python3 generate.py"
    g["resources"] = {"slots_per_trial": 1}
    g["searcher"] = {"name": "single", "metric": "none", "max_length": 2}
    hp = g["hyperparameters"]
    hp.update(main_process_generator_seed=3, save_freq=2, uuids=[uuid])
    hp["pipeline"].update(model_preset="tiny")
    hp["call_kwargs"] = {"prompt": "a painting of a det-logo", "num_inference_steps": 2,
                         "guidance_scale": 3.0, "height": 64, "width": 64}
    eid2, st2 = _run(s, g)
    assert st2 == "COMPLETED"
    t2 = s.get(f"/api/v1/experiments/{eid2}/trials")["trials"][0]
    c2 = s.get(f"/api/v1/trials/{t2['id']}/checkpoints")["checkpoints"]
    pngs = glob.glob(os.path.join(tmp, "ckpt", c2[-1]["uuid"], "*.png"))
    assert len(pngs) == 2 * 2  # batch_size x calls
