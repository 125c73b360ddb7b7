"""Helpers shared by the model-hub trials (reference: ``model_hub/model_hub/utils.py``)."""
import logging
import os
import urllib.parse
from typing import Any, Dict, List, Union

import numpy as np
import torch


class AttrDict(dict):
    """A dict whose keys are also attributes (nested dicts are converted on access)."""

    def __init__(self, *args: Any, **kwargs: Any) -> None:
        super().__init__(*args, **kwargs)
        for k, v in list(self.items()):
            if isinstance(v, dict) and not isinstance(v, AttrDict):
                self[k] = AttrDict(v)

    def __getattr__(self, name: str) -> Any:
        try:
            return self[name]
        except KeyError as e:
            raise AttributeError(name) from e

    def __setattr__(self, name: str, value: Any) -> None:
        self[name] = value


def expand_like(arrays: List[np.ndarray], fill: float = -100) -> np.ndarray:
    """Concatenate arrays along dim 0 whose dim 1 may differ, padding dim 1 with ``fill``."""
    if arrays[0].ndim == 1:
        return np.concatenate(arrays)
    rows = sum(a.shape[0] for a in arrays)
    width = max(a.shape[1] for a in arrays)
    out = np.full((rows, width) + tuple(arrays[0].shape[2:]), fill, dtype=np.result_type(*arrays, fill))
    r = 0
    for a in arrays:
        out[r:r + a.shape[0], :a.shape[1]] = a
        r += a.shape[0]
    return out


def numpify(x: Union[List, np.ndarray, torch.Tensor]) -> np.ndarray:
    if isinstance(x, np.ndarray):
        return x
    if isinstance(x, list):
        return np.array(x)
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    raise TypeError("expected a list, numpy array or torch tensor")


def download_url(download_directory: str, url: str) -> str:
    """Fetch ``url`` once into ``download_directory`` (file-locked against concurrent ranks)."""
    import filelock
    import requests

    name = urllib.parse.urlparse(url).path.rsplit("/", 1)[-1]
    os.makedirs(download_directory, exist_ok=True)
    path = os.path.join(download_directory, name)
    with filelock.FileLock(path + ".lock"):
        if not os.path.exists(path):
            logging.info(f"downloading {url} to {path}")
            r = requests.get(url, stream=True)
            r.raise_for_status()
            with open(path, "wb") as f:
                for chunk in r.iter_content(chunk_size=1 << 16):
                    f.write(chunk)
    return path


def compute_num_training_steps(experiment_config: Dict[str, Any], global_batch_size: int) -> int:
    """Optimizer steps implied by ``searcher.max_length`` (batches, records or epochs)."""
    max_length = experiment_config["searcher"]["max_length"]
    if isinstance(max_length, int):
        return max_length
    unit, n = next(iter(max_length.items()))
    if unit == "batches":
        return int(n)
    if unit == "records":
        return int(n) // global_batch_size
    if unit == "epochs":
        rpe = experiment_config.get("records_per_epoch")
        if not rpe:
            raise ValueError("searcher.max_length in epochs needs records_per_epoch")
        return int(n) * int(rpe) // global_batch_size
    raise ValueError(f"unknown max_length unit {unit}")
