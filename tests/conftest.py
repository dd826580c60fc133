import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the native HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def dtc():
    import dtc_import
    return dtc_import.load()


@pytest.fixture(scope="session")
def cuda(dtc):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    # a native fault prints the faulting thread and its frames (then Python's faulthandler runs), also into
    # gpurun_out/dtc_crash.log: pytest's fd capture loses what a dying test wrote to fd 2
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    os.environ.setdefault("DTC_CRASH_LOG", os.path.join(ROOT, "gpurun_out", "dtc_crash.log"))
    dtc._native.lib.dtc_install_crash_handler()
    return torch.device("cuda:0")


def rel_err(a, b):
    import numpy as np
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = np.linalg.norm(b.ravel())
    return float(np.linalg.norm((a - b).ravel()) / (den if den > 0 else 1.0))
