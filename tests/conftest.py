import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# parallel test workers (pytest -n) each run their own masters: give each a disjoint range of
# rendezvous ports so two workers' 2-rank tasks never share a c10d store port
_w = os.environ.get("PYTEST_XDIST_WORKER", "")
if _w.startswith("gw") and _w[2:].isdigit():
    os.environ.setdefault("DET_RENDEZVOUS_PORT_BASE", str(30000 + 700 * int(_w[2:])))
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
