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


def grad_close(ours, g64, witnesses, k=3.0, bulk_floor=1e-3, max_floor=5e-2):
    """A gradient against fp64 next to fp32 witnesses (paths whose distance from fp64 shows the
    gradient's conditioning).  The bulk — the 99.9th percentile of |ours - fp64| / max|fp64| — must be
    within max(bulk_floor, k x the witnesses'), the max within max(max_floor, k x theirs): ReLU / max-pool
    decisions that sit within fp32 rounding of a tie move a handful of entries by O(1) on any fp32 path,
    so the max alone cannot be held tight.  Returns (ok, (max, bulk, witness bulk))."""
    import torch
    g64 = torch.as_tensor(g64).double().cpu()
    scale = g64.abs().max().item() or 1.0

    def err(a):
        return (torch.as_tensor(a).double().cpu() - g64).abs().flatten() / scale

    def bulk(e):
        return torch.quantile(e, 0.999).item() if e.numel() > 1 else e.max().item()
    e = err(ours)
    wb = max(bulk(err(w)) for w in witnesses)
    wm = max(err(w).max().item() for w in witnesses)
    ok = bulk(e) <= max(bulk_floor, k * wb) and e.max().item() <= max(max_floor, k * wm)
    return ok, (e.max().item(), bulk(e), wb)
