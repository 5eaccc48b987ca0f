import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_built():
    so = os.path.join(REPO, "oracle", "_build", "liboracle.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
    return so


@pytest.fixture(scope="session")
def emu_built():
    so = os.path.join(REPO, "tests", "native", "_build", "libnfa_emu.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "tests", "native")])
    return so


def pytest_sessionstart(session):
    # torch ships its own HIP runtime (ROCm 7.0) beside the engine's /opt/rocm one: when a GPU session uses
    # both (device-resident inputs from torch tensors), torch's runtime must initialise first.
    if "gpu" in (session.config.getoption("markexpr") or "") and "not gpu" not in session.config.getoption("markexpr"):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass
