import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libcad_hip.so)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def cad():
    import cad_pkg
    return cad_pkg.load()


@pytest.fixture(scope="session")
def oracle():
    import torch
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    from oracle import cad_oracle
    return cad_oracle


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def max_rel_err(a, b):
    """max |a - b| / max |b| (normalised max error, the north-star's 'relative fp32' metric)."""
    import torch
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    den = b.abs().max().item()
    return (a - b).abs().max().item() / (den if den > 0 else 1.0)
