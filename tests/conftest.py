import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle_c
    oracle_c.lib()
    return oracle_c


def variant_ctx(v: int):
    """Variant 0 runs on the product library; any other variant on the diagnostics
    build (libzs3gpu_diag.so), selected for this thread only."""
    import contextlib
    import zs3server_amd as z
    return contextlib.nullcontext() if v == 0 else z.diag(v)
