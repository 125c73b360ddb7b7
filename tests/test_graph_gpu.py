"""HIP-graph captured training step (optimizations.hip_graph) vs the eager step, through the real
PyTorchTrial controller: fused BN / MIOpen convolutions / fused SGD with a per-batch LR schedule,
and a transformer with fused AdamW + gradient clipping."""
import pytest
import torch
import torch.nn.functional as F

from determined_clone_amd import pytorch

pytestmark = pytest.mark.gpu

STEPS = 10


class _ResNetTrial(pytorch.PyTorchTrial):
    def __init__(self, context):
        from determined_clone_amd.models import resnet

        self.context = context
        torch.manual_seed(0)
        self.model = context.wrap_model(resnet.to_mi355x_layout(resnet.resnet18_bottleneck_tiny(10)))
        self.opt = context.wrap_optimizer(torch.optim.SGD(self.model.parameters(), lr=0.05, momentum=0.9,
                                                          weight_decay=1e-4))
        sched = torch.optim.lr_scheduler.LambdaLR(self.opt, lambda s: 1.0 / (1 + s))
        self.sched = context.wrap_lr_scheduler(sched, pytorch.LRScheduler.StepMode.STEP_EVERY_BATCH)

    def train_batch(self, batch, epoch_idx, batch_idx):
        x, y = batch
        loss = F.cross_entropy(self.model(x).float(), y)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss}

    def evaluate_batch(self, batch, batch_idx):
        x, y = batch
        return {"val_loss": F.cross_entropy(self.model(x).float(), y)}

    def _data(self):
        g = torch.Generator().manual_seed(1)
        dev = self.context.device
        batches = [(torch.randn(8, 3, 32, 32, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last),
                    torch.randint(0, 10, (8,), generator=g).to(dev)) for _ in range(4)]
        return pytorch.DataLoader(pytorch.DeviceBatchDataset(batches, 64), batch_size=None)

    def build_training_data_loader(self):
        return self._data()

    def build_validation_data_loader(self):
        return self._data()


class _GPTTrial(_ResNetTrial):
    def __init__(self, context):
        from determined_clone_amd.models import gpt2

        self.context = context
        torch.manual_seed(0)
        self.model = context.wrap_model(gpt2.cast_for_mi355x(gpt2.gpt2("tiny", max_seq_len=64)))
        self.opt = context.wrap_optimizer(torch.optim.AdamW(self.model.parameters(), lr=1e-3, weight_decay=0.01))
        sched = torch.optim.lr_scheduler.LambdaLR(self.opt, lambda s: min(1.0, (s + 1) / 4))
        self.sched = context.wrap_lr_scheduler(sched, pytorch.LRScheduler.StepMode.STEP_EVERY_BATCH)

    def train_batch(self, batch, epoch_idx, batch_idx):
        _, loss = self.model(batch, batch)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt, pytorch.clip_grad_norm(1.0))
        return {"loss": loss}

    def evaluate_batch(self, batch, batch_idx):
        _, loss = self.model(batch, batch)
        return {"val_loss": loss}

    def _data(self):
        g = torch.Generator().manual_seed(2)
        batches = [torch.randint(0, 512, (2, 64), generator=g).to(self.context.device) for _ in range(4)]
        return pytorch.DataLoader(pytorch.DeviceBatchDataset(batches, 64), batch_size=None)


def _run(trial_cls, graph, tmp_path, det_convs=False):
    opts = {"hip_graph": graph, "hip_graph_warmup_steps": 3, "hip_graph_deterministic_convs": det_convs}
    with pytorch.init(hparams={"global_batch_size": 8}, exp_conf={"optimizations": opts}) as ctx:
        ctx._core.checkpoint._storage_manager = __import__(
            "determined_clone_amd.common.storage", fromlist=["x"]).SharedFSStorageManager(str(tmp_path / f"ck{graph}"))
        trial = trial_cls(ctx)
        ctrl = pytorch.Trainer(trial, ctx).fit(max_length=pytorch.Batch(STEPS), reporting_period=pytorch.Batch(STEPS),
                                              checkpoint_policy="none")
        torch.cuda.synchronize()
        graphed = getattr(ctrl, "_graphed", None) if ctrl is not None else None
        params = {n: p.detach().float().cpu().clone() for n, p in trial.model.named_parameters()}
        lr = trial.opt.param_groups[0]["lr"]
        return params, graphed, lr, trial.opt._step


@pytest.mark.parametrize("trial_cls", [_ResNetTrial, _GPTTrial])
def test_graph_step_matches_eager(trial_cls, tmp_path, monkeypatch):
    """Replays are bit-exact with the eager step. The ResNet's MIOpen convolutions run their
    deterministic solvers in both runs (the graph runner switches them on; the eager reference
    needs the same solvers to be comparable bit for bit)."""
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    eager, _, lr_e, step_e = _run(trial_cls, False, tmp_path)
    graph, runner, lr_g, step_g = _run(trial_cls, True, tmp_path)
    assert runner is not None and runner.replays == STEPS - 3  # warm-up 3, capture+replay at 4
    assert step_g == step_e == STEPS and lr_g == lr_e
    for n, e in eager.items():
        torch.testing.assert_close(graph[n], e, atol=0, rtol=0, msg=lambda m: f"{n}: {m}")


def test_graph_with_miopen_convolutions_switches_to_deterministic_solvers(tmp_path, monkeypatch):
    """With hip_graph_deterministic_convs the runner's own step calls use the deterministic solvers;
    the process-wide flag is back to its previous value afterwards (evaluation and other models keep
    the default solvers). Without it (the default) the runner leaves the solvers alone."""
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", False)
    _, runner0, _, _ = _run(_ResNetTrial, True, tmp_path / "default")
    assert runner0 is not None and not runner0._deterministic
    _, runner, _, step = _run(_ResNetTrial, True, tmp_path, det_convs=True)
    assert runner is not None and runner.replays == STEPS - 3 and step == STEPS
    assert runner._deterministic
    assert not torch.backends.cudnn.deterministic
    seen = []
    runner.fn = lambda **kw: seen.append(torch.backends.cudnn.deterministic)
    runner._eager(None, 0, 0)
    assert seen == [True] and not torch.backends.cudnn.deterministic
