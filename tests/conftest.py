import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def cuda_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gnnqc.utils.native import hip_ops
    hip_ops()
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def cml_windows():
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.synthetic import make_cml_raw
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=14, n_minutes=6 * 1440, seed=11))
    return pc, ws
