import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# every GPU test runs with the launch-level aliasing guard on (csrc/host/alias.cpp; include/cad/cad.h
# cad_set_alias_check): a launch whose output overlaps one of its inputs fails with CAD_ERR_INVALID
# instead of racing (an environment value set by the caller, e.g. log:<path>, wins)
os.environ.setdefault("CAD_ALIAS_CHECK", "1")
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libcad_hip.so)")
    config.addinivalue_line("markers", "slow: long-running")


# Order of the slow (full-size) tests at the end of the session: cheapest first, so a session that
# runs out of time loses the fewest checks.
_SLOW_ORDER = ("test_gpu_fullsize_bf16.py::test_bs32_480x640_resunet", "test_gpu_fullsize.py",
               "test_gpu_fullsize_bf16.py::test_bs32_480x640_bf16_step_vs_oracle[baseline]",
               "test_gpu_fullsize_bf16.py::test_bs32_480x640_bf16_step_vs_oracle[rayfilm]")


def pytest_collection_modifyitems(session, config, items):
    """Slow-marked items run after everything else (stable order otherwise): a full-size test that
    overruns the session's time budget can then never starve the operator, fixture and model tests."""
    def rank(it):
        if it.get_closest_marker("slow") is None:
            return 0
        for k, pat in enumerate(_SLOW_ORDER):
            if pat in it.nodeid:
                return 1 + k
        return 1 + len(_SLOW_ORDER)
    items[:] = [it for _, _, it in sorted((rank(it), i, it) for i, it in enumerate(items))]


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

    def bulk(e):   # torch.quantile(e, 0.999) (linear interpolation), without its 2^24-element limit
        n = e.numel()
        if n <= 1:
            return e.max().item()
        pos = 0.999 * (n - 1)
        lo = int(pos)
        vlo = torch.kthvalue(e, lo + 1).values.item()
        vhi = torch.kthvalue(e, min(lo + 2, n)).values.item()
        return vlo + (vhi - vlo) * (pos - lo)
    e = err(ours)
    wb = max(bulk(err(w)) for w in witnesses)
    wm = max(err(w).max().item() for w in witnesses)
    ok = bulk(e) <= max(bulk_floor, k * wb) and e.max().item() <= max(max_floor, k * wm)
    return ok, (e.max().item(), bulk(e), wb)


def unet_bn_blocks(model="baseline"):
    """(GPU debug-buffer tag, oracle DoubleConv prefix, level) of every DoubleConv of the U-Net family:
    enc0..enc4 = enc1, enc2.conv .. bottleneck.conv; dec0..dec3 = dec1.conv .. dec4.conv."""
    enc = [("enc0", "enc1.", 0)] + [(f"enc{l}", f"{n}.conv.", l)
                                     for l, n in zip(range(1, 5), ("enc2", "enc3", "enc4", "bottleneck"))]
    return enc + [(f"dec{l}", f"dec{l + 1}.conv.", l) for l in range(4)]


def geo_bn_blocks(model):
    """(geonet debug-buffer suffix, oracle DoubleConv prefix, level) of every FiLM DoubleConv of the
    geometry-aware family (cad_geonet_debug_buffer "y1<suffix>" / "y2<suffix>")."""
    from oracle import cad_oracle as O
    nl, enc = O._geo_names(model)
    return ([("e0", "enc1.", 0)] + [(f"e{l}", f"{enc[l]}.conv.", l) for l in range(1, nl)] +
            [(f"d{l}", f"dec{l + 1}.conv.", l) for l in range(nl - 1)])


def relu_decisions_from(y, gamma, beta, B, h, w, C, dev):
    """sign(bn(y)) exactly as the BN-apply kernel evaluates it (see gpu_relu_decisions): (B, C, h, w) bool."""
    import numpy as np
    import torch
    eps = float(np.float32(1e-5))
    y = y[: B * h * w * C].to(dev).double().reshape(B * h * w, C)
    mu32 = y.mean(0).float()
    inv = (1.0 / torch.sqrt(y.var(0, unbiased=False) + eps)).float()
    sc = gamma.float().to(dev) * inv
    sh = (beta.double().to(dev) - mu32.double() * sc.double()).float()   # fma(-mean, scale, beta)
    z = y * sc.double() + sh.double()
    return (z > 0).reshape(B, h, w, C).permute(0, 3, 1, 2).contiguous().cpu()


def geo_relu_decisions(net, params, f, B, H, W, model, dev=None):
    """The ReLU decisions of a geometry-aware net's last train-mode forward, for cad_oracle.RELU_FORCE,
    rebuilt from its stored pre-BN conv outputs like gpu_relu_decisions."""
    import torch
    dev = dev or torch.device("cpu")
    masks = {}
    for sfx, pre, l in geo_bn_blocks(model):
        C, h, w = f << l, H >> l, W >> l
        for k in ("1", "2"):
            masks[pre + "bn" + k] = relu_decisions_from(net.debug_buffer(f"y{k}{sfx}"), params[pre + "bn" + k + ".weight"],
                                                        params[pre + "bn" + k + ".bias"], B, h, w, C, dev)
    return masks


def gpu_relu_decisions(net, params, f, B, H, W, model="baseline", dev=None):
    """The ReLU decisions of `net`'s last train-mode forward, for cad_oracle.RELU_FORCE.

    Rebuilt from the stored pre-BN conv outputs (cad_unet_debug_buffer "<tag>_y1|_y2", the values the
    GPU normalised) exactly as the BN-apply kernel takes them: batch statistics in fp64, mean and
    1/sqrt(var + eps) rounded to fp32, scale = gamma * invstd and shift = beta - mean * scale in fp32,
    decision = sign(y * scale + shift) (the kernel's fused multiply-add keeps the exact sign, which the
    fp64 evaluation of the same product and sum reproduces).  `dev`: where this bookkeeping runs (the
    GPU at full size: it is test arithmetic on the stored values, not the oracle); masks come back on
    the host."""
    import numpy as np
    import torch
    masks = {}
    eps = float(np.float32(1e-5))
    dev = dev or torch.device("cpu")
    for tag, pre, l in unet_bn_blocks(model):
        C, h, w = f << l, H >> l, W >> l
        for k in ("1", "2"):
            y = net.debug_buffer(f"{tag}_y{k}")[: B * h * w * C].to(dev).double().reshape(B * h * w, C)
            mu = y.mean(0)
            var = y.var(0, unbiased=False)
            mu32 = mu.float()
            inv = (1.0 / torch.sqrt(var + eps)).float()
            g = params[pre + "bn" + k + ".weight"].float().to(dev)
            b = params[pre + "bn" + k + ".bias"].float().to(dev)
            sc = g * inv
            sh = (b.double() - mu32.double() * sc.double()).float()   # fma(-mean, scale, beta)
            z = y * sc.double() + sh.double()
            del y
            masks[pre + "bn" + k] = (z > 0).reshape(B, h, w, C).permute(0, 3, 1, 2).contiguous().cpu()
            del z
    return masks


def gpu_film_params(net, params, f, B, model="rayfilm"):
    """The FiLM (gamma, beta) of every FiLM DoubleConv of `net`'s last forward (cad_unet_debug_buffer
    "<tag>_gamma|_beta", (B, C) each), keyed like cad_oracle.FILM_FORCE ("enc1.film.", ...)."""
    out = {}
    for tag, pre, l in unet_bn_blocks(model):
        if pre + "film.fc1.weight" not in params:
            continue
        C = f << l
        out[pre + "film."] = tuple(net.debug_buffer(f"{tag}_{t}")[: B * C].reshape(B, C).clone()
                                   for t in ("gamma", "beta"))
    return out


def gpu_conv_outputs(net, f, B, H, W, model="baseline"):
    """The stored pre-BN outputs of every 3x3 convolution of `net`'s last forward (bf16 values on the
    bf16 engine), NCHW float, keyed like cad_oracle.Y_FORCE ("enc1.conv1", "dec2.conv.conv2", ...)."""
    out = {}
    for tag, pre, l in unet_bn_blocks(model):
        C, h, w = f << l, H >> l, W >> l
        for k in ("1", "2"):
            y = net.debug_buffer(f"{tag}_y{k}")[: B * h * w * C].reshape(B, h, w, C)
            out[pre + "conv" + k] = y.permute(0, 3, 1, 2).contiguous()
    return out
