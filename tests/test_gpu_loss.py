"""Fused loss kernels vs the REFERENCE's CombinedDepthLoss (golden fixtures written by the compiled
reference headers, tests/golden/loss_*) and vs the oracle restatement at the bench shape.
Tolerance: 1e-4 relative on the loss values, 1e-3 normalised max error on dL/dpred."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, max_rel_err

pytestmark = pytest.mark.gpu

LOSS_FIXTURES = ["loss_b2_120x160", "loss_b3_50x70", "loss_b2_32x48_allholes", "loss_b2_48x64_mask"]


def _pred(B, H, W):
    from oracle.cad_oracle import u01
    return (np.float32(0.05) + np.float32(9.9) * u01(0xBEEF, np.arange(B * H * W, dtype=np.uint64))).reshape(B, 1, H, W)


@pytest.mark.parametrize("name", LOSS_FIXTURES)
def test_loss_vs_reference_fixture(cad, dev, oracle, name):
    fx, meta = oracle.load_fixture(os.path.join(GOLDEN, name))
    B, H, W = meta["B"], meta["H"], meta["W"]
    rgb, gt, K = oracle.synth_batch(B, H, W)
    pred = _pred(B, H, W)
    assert np.array_equal(pred, fx["input.pred"].numpy())
    gt = fx["input.gt"].numpy()
    loss = cad.CombinedDepthLoss(*meta["weights"], batch=B, height=H, width=W)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    # forwardWithIntrinsics' optional valid_mask (depth_loss.h:416-433) when the fixture has one
    mask = t(fx["input.mask"].numpy() > 0.5) if "input.mask" in fx else None
    loss5, dpred = loss.forward_with_intrinsics(t(pred), t(gt), t(rgb), t(K), valid_mask=mask)
    v = loss5.cpu().numpy()
    comps = meta["components"]
    ref = [meta["total"], comps["si_loss"], comps["grad_loss"], comps["smooth_loss"], comps["reproj_loss"]]
    for got, want in zip(v, ref):
        assert abs(got - want) <= 1e-4 * max(abs(want), 1e-3), (v, ref)
    assert max_rel_err(dpred.cpu(), fx["dpred"]) < 1e-3


def test_loss_bench_shape_vs_oracle(cad, dev, oracle):
    """bs2 at the full 480x640 resolution, oracle on host cores."""
    B, H, W = 2, 480, 640
    rgb, gt, K = oracle.synth_batch(B, H, W)
    pred = _pred(B, H, W)
    w = (1.0, 0.1, 0.001, 0.01)
    total, comps, dref = oracle.loss_and_dpred(torch.from_numpy(pred), torch.from_numpy(gt), torch.from_numpy(rgb),
                                               torch.from_numpy(K), w)
    loss = cad.CombinedDepthLoss(*w, batch=B, height=H, width=W)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    loss5, dpred = loss.forward_with_intrinsics(t(pred), t(gt), t(rgb), t(K))
    v = loss5.cpu().numpy()
    ref = [total, comps["si_loss"], comps["grad_loss"], comps["smooth_loss"], comps["reproj_loss"]]
    for got, want in zip(v, ref):
        assert abs(got - want) <= 1e-4 * max(abs(want), 1e-3), (v, ref)
    assert max_rel_err(dpred.cpu(), dref) < 1e-3


def test_loss_deterministic(cad, dev, oracle):
    B, H, W = 2, 96, 128
    rgb, gt, K = oracle.synth_batch(B, H, W)
    pred = _pred(B, H, W)
    loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    a5, ad = loss.forward_with_intrinsics(t(pred), t(gt), t(rgb), t(K))
    a5, ad = a5.clone(), ad.clone()
    b5, bd = loss.forward_with_intrinsics(t(pred), t(gt), t(rgb), t(K))
    assert torch.equal(a5, b5) and torch.equal(ad, bd)


def test_depth_metrics(cad, dev, oracle):
    B, H, W = 3, 64, 80
    _, gt, _ = oracle.synth_batch(B, H, W)
    pred = _pred(B, H, W)
    m = cad.depth_metrics(torch.from_numpy(pred).to(dev), torch.from_numpy(gt).to(dev))
    ref = {k: 0.0 for k in m}
    for b in range(B):
        r = oracle.depth_metrics(torch.from_numpy(pred[b]), torch.from_numpy(gt[b]))
        for k in ref:
            ref[k] += r[k] / B
    for k in m:
        assert abs(m[k] - ref[k]) <= 1e-4 * max(1.0, abs(ref[k])), (k, m[k], ref[k])
