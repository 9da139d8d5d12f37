"""pytest configuration: `gpu` marker, repo on sys.path, shared fixtures."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def load_npz(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden_fixed():
    return load_npz("fixed_k10_L1350.npz")


@pytest.fixture(scope="session")
def golden_shapes():
    return load_npz("shapes.npz")


@pytest.fixture(scope="session")
def golden_ragged():
    return load_npz("ragged.npz")


@pytest.fixture(scope="session")
def ctx():
    """One qfec context on cuda:0 for the whole GPU session (fails loudly)."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    from libquic_amd import qfec
    c = qfec.Context(0)
    c.set_stream(torch.cuda.current_stream())  # order with torch's copies/fills
    yield c
    c.close()
