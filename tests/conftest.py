import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "draid-spdk_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


@pytest.fixture(scope="session")
def golden():
    import json
    gdir = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(gdir, "manifest.json")) as f:
        man = json.load(f)
    man["_dir"] = gdir
    return man


@pytest.fixture(scope="session")
def ec():
    """The product library through its C ABI; fails loudly if it or the GPU is missing."""
    import torch
    import draid_ec
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    draid_ec.lib()
    torch.cuda.init()
    return draid_ec
