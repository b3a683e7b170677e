import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: longer-running CPU test")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def brr():
    import bayesrrcpp_amd as B
    B.build_library()
    return B


def gpu_available() -> bool:
    try:
        import bayesrrcpp_amd as B
        return B.lib().brr_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def require_gpu(brr):
    # GPU tests must run the HIP path: no silent skip on a GPU box, loud failure instead.
    n = brr.lib().brr_device_count()
    assert n > 0, "no HIP device visible to libbrr.so"
    return n


CVA = np.array([1e-4, 1e-3, 1e-2])
HYP = dict(sigma0=0.01, v0E=1e-4, s02E=1e-3, v0G=1e-4, s02G=1e-3)  # vignettes/BayesRR.Rmd:93-98
