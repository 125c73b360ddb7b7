"""One-weight linear model trial: data = label = 1, MSE loss, plain SGD, so every step's weight is
known in closed form: w' = w + 2*lr*(1 - w). Used to check the controller end to end."""
from typing import Any, Dict, List

import torch

from determined_clone_amd import pytorch


class Ones(torch.utils.data.Dataset):
    def __init__(self, n: int = 64) -> None:
        self.n = n

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i: int):
        return torch.tensor([1.0]), torch.tensor([1.0])


class LabelSum(pytorch.MetricReducer):
    def __init__(self) -> None:
        self.reset()

    def reset(self) -> None:
        self.total = 0.0

    def update(self, v: float) -> None:
        self.total += float(v)

    def per_slot_reduce(self) -> Any:
        return self.total

    def cross_slot_reduce(self, per_slot: List[Any]) -> Any:
        return sum(per_slot)


class Recorder(pytorch.PyTorchCallback):
    def __init__(self) -> None:
        self.val: List[Dict[str, Any]] = []
        self.train: List[Dict[str, Any]] = []
        self.uuids: List[str] = []
        self.epochs_ended: List[int] = []

    def on_validation_end(self, metrics: Dict[str, Any]) -> None:
        self.val.append(metrics)

    def on_training_workload_end(self, avg_metrics, batch_metrics) -> None:
        self.train.append(avg_metrics)

    def on_checkpoint_upload_end(self, uuid: str) -> None:
        self.uuids.append(uuid)

    def on_training_epoch_end(self, epoch_idx: int) -> None:
        self.epochs_ended.append(epoch_idx)

    def state_dict(self) -> Dict[str, Any]:
        return {"epochs_ended": list(self.epochs_ended)}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        self.epochs_ended = list(sd["epochs_ended"])


class OneVarTrial(pytorch.PyTorchTrial):
    LR = 0.001

    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        model = torch.nn.Linear(1, 1, bias=False)
        model.weight.data.fill_(0.0)
        self.model = context.wrap_model(model)
        fused = bool(context.get_hparams().get("fused", False))
        self.opt = context.wrap_optimizer(torch.optim.SGD(self.model.parameters(), lr=self.LR), fused=fused)
        self.reducer = context.wrap_reducer(LabelSum(), name="label_sum")
        self.recorder = Recorder()
        self.batch_size = int(context.get_hparams().get("batch_size", 4))

    def train_batch(self, batch, epoch_idx: int, batch_idx: int):
        data, label = batch
        self.reducer.update(label.sum())
        w_before = self.model.weight.detach().clone().reshape(())
        out = self.model(data)
        loss = torch.nn.functional.mse_loss(out, label)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        w_after = self.model.weight.detach().clone().reshape(())
        w_exp = w_before + 2 * self.LR * (1 - w_before)
        return {"loss": loss, "w_before": w_before, "w_after": w_after, "w_exp": w_exp}

    def evaluate_batch(self, batch, batch_idx: int) -> Dict[str, Any]:
        data, label = batch
        loss = torch.nn.functional.mse_loss(self.model(data), label)
        return {"val_loss": loss, "weight": self.model.weight.detach().reshape(())}

    def build_training_data_loader(self):
        return pytorch.DataLoader(Ones(), batch_size=self.batch_size)

    def build_validation_data_loader(self):
        return pytorch.DataLoader(Ones(16), batch_size=self.batch_size)

    def build_callbacks(self):
        return {"recorder": self.recorder}
