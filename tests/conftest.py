"""Shared test setup.

`gpu`-marked tests need an MI355X and call the product only through the C ABI
(libfaer_amg_amd.so via faer_amg_amd); everything else runs on CPU.  The oracle
(oracle/) is used only as the checker.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "faer-amg_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X) and the HIP library")


@pytest.fixture(scope="session")
def ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import faer_amg_amd as fa
    return fa.Context(0)


@pytest.fixture(scope="session")
def dev():
    import torch
    return torch.device("cuda:0")


@pytest.fixture
def no_tail():
    """The cycle without its dense tail (flag dense_tail = 0, ops.hip
    ensure_tail): for tests about the launches of the coarse levels it replaces."""
    import faer_amg_amd as fa
    fa.set_flag("dense_tail", 0)
    yield
    fa.set_flag("dense_tail", 4096)
