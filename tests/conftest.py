import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    config.addinivalue_line("markers", "optin: tests an opt-in kernel / fusion not yet validated on "
                                       "hardware; runs only with SCFLOW_TEST_OPTIN=1")


def pytest_collection_modifyitems(config, items):
    import torch
    if os.environ.get("SCFLOW_TEST_OPTIN") != "1":
        optin = pytest.mark.skip(reason="opt-in path awaiting hardware validation "
                                        "(SCFLOW_TEST_OPTIN=1 runs it)")
        for item in items:
            if "optin" in item.keywords:
                item.add_marker(optin)
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
