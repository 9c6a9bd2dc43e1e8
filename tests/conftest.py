import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def rcdc_lib():
    from rustic_core_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.lib()


@pytest.fixture(scope="session")
def gpu_ctx(rcdc_lib):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import oracle
    from rustic_core_amd.chunker import Context
    return Context.get(oracle.DEFAULT_POLY, oracle.DEFAULT_MIN, oracle.DEFAULT_AVG,
                       oracle.DEFAULT_MAX, device=0)
