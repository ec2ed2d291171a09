import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: larger CPU-side cases")


@pytest.fixture(scope="session")
def kats():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gpu_lib():
    """The product library on a real device; fails loudly (no skip) when the
    HIP library is missing on a GPU run.  torch is initialised first: its
    wheel bundles its own libamdhip64, and whichever HIP runtime a process
    loads first is the one both then share (same soname) -- torch's must win
    for torch.cuda to see the GPU."""
    import torch

    torch.cuda.init()
    import ouroboros_network_amd as ona

    lib = ona._native.load()
    return lib
