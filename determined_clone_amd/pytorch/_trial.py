"""PyTorchTrial interface and training-length units
(reference: `harness/determined/pytorch/_pytorch_trial.py:44-182, 1416-1663`)."""
import abc
import collections.abc
import sys
from typing import Any, Dict, Optional, Union

import torch

from determined_clone_amd import core
from determined_clone_amd.pytorch._callback import PyTorchCallback
from determined_clone_amd.pytorch._data import DataLoader, TorchData, data_length
from determined_clone_amd.pytorch._reducer import Reducer


class TrainUnit:
    """``Batch(n)`` / ``Epoch(n)``: an int is a period, a container is an explicit schedule."""

    def __init__(self, value: Union[int, collections.abc.Container]) -> None:
        self.value = value

    @staticmethod
    def _from_searcher_unit(length: int, unit: Optional[core.Unit],
                            global_batch_size: Optional[int] = None) -> "TrainUnit":
        if unit == core.Unit.EPOCHS:
            return Epoch(length)
        if unit == core.Unit.RECORDS:
            if global_batch_size is None:
                raise ValueError("global_batch_size required for searcher unit Records.")
            return Batch._from_records(length, global_batch_size)
        if unit == core.Unit.BATCHES:
            return Batch(length)
        raise ValueError(f"unrecognized searcher unit {unit}")

    def _to_searcher_unit(self) -> core.Unit:
        return core.Unit.BATCHES if isinstance(self, Batch) else core.Unit.EPOCHS

    @staticmethod
    def _from_values(batches: Optional[int] = None, records: Optional[int] = None,
                     epochs: Optional[int] = None,
                     global_batch_size: Optional[int] = None) -> "TrainUnit":
        if sum((batches is not None, records is not None, epochs is not None)) != 1:
            raise ValueError(f"invalid config: batches={batches} records={records} epochs={epochs}")
        if batches is not None:
            return Batch(batches if batches >= 1 else sys.maxsize)
        if records is not None:
            if not global_batch_size:
                raise ValueError("global_batch_size is required for RECORD units.")
            return Batch._from_records(records if records >= 1 else sys.maxsize, global_batch_size)
        return Epoch(epochs if epochs >= 1 else sys.maxsize)  # type: ignore[operator]

    def should_stop(self, step_num: int) -> bool:
        if isinstance(self.value, int):
            return self._divides(step_num)
        return step_num in self.value

    def _divides(self, steps: int) -> bool:
        assert isinstance(self.value, int)
        if self.value < 1:
            return True
        if steps == 0:
            return False
        return steps % self.value == 0

    def __repr__(self) -> str:
        return f"{type(self).__name__}({self.value})"


class Epoch(TrainUnit):
    pass


class Batch(TrainUnit):
    @staticmethod
    def _from_records(records: int, global_batch_size: int) -> "Batch":
        return Batch(max(records // global_batch_size, 1))


class PyTorchTrial(metaclass=abc.ABCMeta):
    """Subclass and implement ``__init__(context)``, ``train_batch``, data loaders and one of
    ``evaluate_batch`` / ``evaluate_full_dataset``."""

    trial_context_class: Any = None  # set in __init__.py to PyTorchTrialContext

    @abc.abstractmethod
    def __init__(self, context: Any) -> None:
        pass

    @abc.abstractmethod
    def train_batch(self, batch: TorchData, epoch_idx: int, batch_idx: int) -> Union[torch.Tensor, Dict[str, Any]]:
        pass

    @abc.abstractmethod
    def build_training_data_loader(self) -> DataLoader:
        pass

    @abc.abstractmethod
    def build_validation_data_loader(self) -> DataLoader:
        pass

    def build_callbacks(self) -> Dict[str, PyTorchCallback]:
        return {}

    def evaluate_batch(self, batch: TorchData, batch_idx: int) -> Dict[str, Any]:
        pass  # type: ignore[return-value]

    def evaluation_reducer(self) -> Union[Reducer, Dict[str, Reducer]]:
        return Reducer.AVG

    def evaluate_full_dataset(self, data_loader: torch.utils.data.DataLoader) -> Dict[str, Any]:
        pass  # type: ignore[return-value]

    def get_batch_length(self, batch: Any) -> int:
        return data_length(batch)
