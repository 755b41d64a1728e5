import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "tests"), os.path.join(REPO, "oracle"), os.path.join(REPO, "rust-crdt_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def oracle():
    import oracle_ffi

    oracle_ffi.lib()
    return oracle_ffi


@pytest.fixture(scope="session")
def gpu():
    """The product library bound to cuda:0. Fails loudly when the HIP path is missing."""
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test run without a visible GPU")
    import crdts_hip

    return crdts_hip.Engine(device=0)
