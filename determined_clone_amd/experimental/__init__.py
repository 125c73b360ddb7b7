"""Experimental APIs (reference: `harness/determined/experimental/__init__.py`): the Python client
SDK lives in :mod:`.client`."""
from determined_clone_amd.experimental import client
from determined_clone_amd.experimental.client import (Checkpoint, CheckpointState, Determined,
                                                      DownloadMode, Experiment, ExperimentState,
                                                      Model, ModelVersion, OrderBy, Project, Trial,
                                                      TrialMetrics, TrialState, User, Workspace)
