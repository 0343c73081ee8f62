import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via `pytest -m gpu`)")
    config.addinivalue_line("markers", "slow: long CPU oracle run")


@pytest.fixture(scope="session")
def hecdna():
    # torch ships its own HIP runtime (torch/lib/libamdhip64.so, soname libamdhip64.so.7).  Initialising
    # torch first lets libhecdna bind to that same runtime; loading libhecdna first would pull in
    # /opt/rocm's copy and leave torch's second runtime without a device (tests that exchange device
    # tensors with torch need both on one runtime).
    import torch
    torch.cuda.is_available()
    from _helpers import load_hecdna
    return load_hecdna()


@pytest.fixture(scope="session")
def orc():
    from _helpers import load_oracle
    return load_oracle()
