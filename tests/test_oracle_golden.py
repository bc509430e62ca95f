"""Pin the oracle restatement (oracle/cad_oracle.py) to the REFERENCE: golden fixtures in
tests/golden/ were produced by the reference's own headers (src/models/baseline_unet.h,
src/loss/depth_loss.h) compiled against LibTorch and driven exactly like
tensorboard_trainer_enhanced.h:287-304 (oracle/ref_harness.cpp, oracle/gen_golden.py).
CPU only; single-threaded like the fixture generation."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, max_rel_err

TRAIN = ["train_f4_b2_64x64", "train_f4_b3_96x128_si"]
LOSS = ["loss_b2_120x160", "loss_b3_50x70", "loss_b2_32x48_allholes"]


@pytest.fixture(autouse=True)
def _one_thread():
    n = torch.get_num_threads()
    torch.set_num_threads(1)
    yield
    torch.set_num_threads(n)


def test_param_count_known_answers(oracle):
    # BaselineUNet(3,64) prints "Total parameters: 31037633" (tfevents record; test_models.cpp)
    assert oracle.num_params(64) == 31037633
    assert oracle.num_params(96) == 69823777
    assert oracle.num_params(8) == 486553
    assert oracle.num_params(4) == 122093


@pytest.mark.parametrize("name", TRAIN)
def test_manifest_order_matches_param_spec(oracle, name):
    fx, meta = oracle.load_fixture(os.path.join(GOLDEN, name))
    names = [k[len("init."):] for k in fx if k.startswith("init.") and "running" not in k]
    assert names == [n for n, _ in oracle.param_spec(meta["f"])]
    for n, s in oracle.param_spec(meta["f"]):
        assert tuple(fx["init." + n].shape) == s
    bnames = [k[len("init."):] for k in fx if k.startswith("init.") and "running" in k]
    assert bnames == [n for n, _ in oracle.buffer_spec(meta["f"])]
    assert meta["num_params"] == oracle.num_params(meta["f"])


@pytest.mark.parametrize("name", TRAIN)
def test_synthetic_inputs_bitwise(oracle, name):
    fx, meta = oracle.load_fixture(os.path.join(GOLDEN, name))
    rgb, gt, K = oracle.synth_batch(meta["B"], meta["H"], meta["W"])
    assert np.array_equal(rgb, fx["input.rgb"].numpy())
    assert np.array_equal(K, fx["input.K"].numpy())
    # gt goes through sin(): allow 1-ulp libm differences, require >= 99.9% bitwise
    g = fx["input.gt"].numpy()
    assert np.mean(gt == g) > 0.999 and np.max(np.abs(gt - g)) < 1e-5


@pytest.mark.parametrize("name", TRAIN)
def test_oracle_train_steps_vs_reference(oracle, name):
    fx, meta = oracle.load_fixture(os.path.join(GOLDEN, name))
    f = meta["f"]
    params = {n: fx["init." + n] for n, _ in oracle.param_spec(f)}
    bufs = {n: fx["init." + n] for n, _ in oracle.buffer_spec(f)}
    tr = oracle.Trainer(params, bufs, weights=meta["weights"])
    rgb, gt, K = fx["input.rgb"], fx["input.gt"], fx["input.K"]
    r = tr.step(rgb, gt, K)
    assert max_rel_err(r["pred"], fx["step1.pred"]) < 1e-6
    assert max_rel_err(r["dpred"], fx["step1.dpred"]) < 1e-5
    assert abs(r["loss"] - meta["losses"][0]) <= 1e-6 * abs(meta["losses"][0])
    for k, v in meta["step1_components"].items():
        assert abs(r["comps"][k] - v) <= 1e-5 * max(abs(v), 1e-6), k
    assert abs(r["norm"] - meta["step1_total_norm"]) <= 1e-5 * meta["step1_total_norm"]
    for (n, _), g in zip(oracle.param_spec(f), r["grads"]):
        assert max_rel_err(g, fx["step1.grad." + n]) < 1e-4, n
    for n, _ in oracle.param_spec(f):
        assert (tr.p[n] - fx["step1.param." + n]).abs().max().item() < 1e-6, n
    for n, _ in oracle.buffer_spec(f):
        assert max_rel_err(tr.bufs[n], fx["step1." + n]) < 1e-5, n
    losses = [r["loss"]] + [tr.step(rgb, gt, K)["loss"] for _ in range(meta["steps"] - 1)]
    np.testing.assert_allclose(losses, meta["losses"], rtol=1e-5)
    for n, _ in oracle.param_spec(f):
        assert (tr.p[n] - fx["final.param." + n]).abs().max().item() < 1e-5, n
    pe = tr.predict_eval(rgb)
    assert max_rel_err(pe, fx["final.pred_eval"]) < 1e-5
    assert abs(oracle.abs_rel_per_sample(pe, gt) - meta["final_abs_rel_eval"]) < 1e-5


@pytest.mark.parametrize("name", LOSS)
def test_oracle_loss_vs_reference(oracle, name):
    fx, meta = oracle.load_fixture(os.path.join(GOLDEN, name))
    B, H, W = meta["B"], meta["H"], meta["W"]
    rgb, _, K = oracle.synth_batch(B, H, W)
    total, comps, dpred = oracle.loss_and_dpred(fx["input.pred"], fx["input.gt"], torch.from_numpy(rgb),
                                                torch.from_numpy(K), meta["weights"])
    assert abs(total - meta["total"]) <= 1e-6 * max(1.0, abs(meta["total"]))
    for k, v in meta["components"].items():
        assert abs(comps[k] - v) <= 1e-6 * max(1.0, abs(v)), k
    assert max_rel_err(dpred, fx["dpred"]) < 1e-6


def test_all_holes_fixture_semantics(oracle):
    """n == 0: SI and reprojection return zeros(1) (depth_loss.h:53-55, :325-327); grad-matching and
    smoothness still contribute (the gradient loss ignores the mask, :137)."""
    fx, meta = oracle.load_fixture(os.path.join(GOLDEN, "loss_b2_32x48_allholes"))
    assert meta["components"]["si_loss"] == 0.0 and meta["components"]["reproj_loss"] == 0.0
    assert meta["components"]["grad_loss"] > 0 and meta["components"]["smooth_loss"] > 0
    assert meta["total_dim"] == 1   # CombinedDepthLoss returns shape [1]
