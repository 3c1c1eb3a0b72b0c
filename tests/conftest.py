import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle  # oracle/oracle.py (test infrastructure)
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def p64():
    import p64_amd
    p64_amd.lib()
    return p64_amd


@pytest.fixture(scope="session")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test scheduled but no HIP device is visible")
    return torch
