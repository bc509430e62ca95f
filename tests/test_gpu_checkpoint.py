"""torch::save / torch::load checkpoints of a live model on the MI355X (cad_unet_save_torch /
cad_unet_load_torch; format and LibTorch byte-parity in test_checkpoint.py).

* round trip: a trained model saved and loaded into a fresh one gives bit-identical parameters,
  BatchNorm buffers and num_batches_tracked, and the same eval-mode output;
* a checkpoint the reference's torch::save wrote (tests/golden/ckpt_baseline_f4, reference code run
  in the build container) loads, and the model then predicts what the oracle predicts with the same
  weights;
* a checkpoint of another architecture is refused and leaves the model untouched.
"""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, max_rel_err
from test_checkpoint import _read_all

pytestmark = pytest.mark.gpu


def _trained(cad, oracle, model_cls, f, B, H, W, steps, seed=1):
    kind = {cad.BaselineUNet: "baseline", cad.RayConditionedUNet: "rayfilm"}[model_cls]
    m = model_cls(3, f, max_depth=10.0, batch=B, height=H, width=W)
    state = dict(oracle.synth_init(f, model=kind))
    state.update(oracle.init_buffers(f, model=kind))
    m.load_state_dict(state)
    loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
    tr = cad.Trainer(m, loss)
    rgb, gt, K = [torch.from_numpy(a).cuda() for a in oracle.synth_batch(B, H, W, rgb_seed=seed)]
    for _ in range(steps):
        tr.train_step(rgb, gt, K)
    torch.cuda.synchronize()
    return m, rgb, K


@pytest.mark.parametrize("kind", ["baseline", "rayfilm"])
def test_save_load_round_trip(cad, dev, oracle, tmp_path, kind):
    cls = cad.BaselineUNet if kind == "baseline" else cad.RayConditionedUNet
    f, B, H, W = 8, 2, 64, 64
    m, rgb, K = _trained(cad, oracle, cls, f, B, H, W, steps=3)
    assert m.num_batches_tracked() == 3
    path = tmp_path / "baseline_unet_epoch_3.pt"
    cad.save(m, path)
    m2 = cls(3, f, max_depth=10.0, batch=B, height=H, width=W)
    cad.load(m2, path)
    for (n, a), (n2, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert n == n2 and torch.equal(a, b), n
    assert m2.num_batches_tracked() == 3
    m.eval()
    m2.eval()
    cam = torch.stack([K[:, 0, 0], K[:, 1, 1], K[:, 0, 2], K[:, 1, 2]], 1).contiguous()
    args = (rgb,) if kind == "baseline" else (rgb, cam)
    assert torch.equal(m(*args), m2(*args))
    # the archive lists every module tensor with its num_batches_tracked counter
    arch = _read_all(cad, path)
    assert int(arch["dec1.conv.bn2.num_batches_tracked"]) == 3
    if kind == "rayfilm":   # FiLM's BatchNorm1d ran in every step (B = 2 > 1)
        assert int(arch["enc1.film.bn1.num_batches_tracked"]) == 3
    assert {n for n in arch if not n.endswith("num_batches_tracked")} == set(m.state_dict())


def test_load_reference_checkpoint(cad, dev, oracle):
    path = os.path.join(ROOT, "tests", "golden", "ckpt_baseline_f4", "baseline_unet_epoch_1.pt")
    arch = _read_all(cad, path)
    B, H, W = 2, 32, 32
    m = cad.BaselineUNet(3, 4, 10.0, batch=B, height=H, width=W)
    cad.load(m, path)
    sd = m.state_dict()
    for n, v in sd.items():
        assert np.array_equal(v.numpy(), arch[n]), n
    assert m.num_batches_tracked() == int(arch["enc1.bn1.num_batches_tracked"]) == 1
    params = {n: torch.from_numpy(arch[n]) for n, _ in oracle.param_spec(4)}
    bufs = {n: torch.from_numpy(arch[n]) for n in oracle.init_buffers(4)}
    ref = oracle.Trainer(params, bufs)
    rgb = torch.from_numpy(oracle.synth_batch(B, H, W, rgb_seed=5)[0])
    m.eval()
    ours = m.forward(rgb.to(dev)).cpu()
    assert max_rel_err(ours, ref.predict_eval(rgb)) < 1e-5


def test_load_refuses_other_architecture(cad, dev, oracle, tmp_path):
    m, _, _ = _trained(cad, oracle, cad.BaselineUNet, 8, 2, 32, 32, steps=1)
    path = tmp_path / "f8.pt"
    cad.save(m, path)
    other = cad.BaselineUNet(3, 4, 10.0, batch=2, height=32, width=32)
    before = other.state_dict()
    with pytest.raises(cad.CadError, match="shape mismatch"):
        cad.load(other, path)
    film = cad.IntrinsicsConditionedUNet(3, 8, 4, 10.0, batch=2, height=32, width=32)
    with pytest.raises(cad.CadError, match="has no"):
        cad.load(film, path)
    for (n, a), b in zip(before.items(), other.state_dict().values()):
        assert torch.equal(a, b), n
