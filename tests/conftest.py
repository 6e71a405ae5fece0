import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsparc_amp.so)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


@pytest.fixture(scope="session")
def lib_gpu():
    """The HIP library on a visible device; a GPU test fails (not skips) without it."""
    import sparc_ldpc_amd as s
    lib = s.load_library()
    assert lib.sa_device_count() > 0, "no HIP device visible: -m gpu tests need an MI355X"
    return lib
