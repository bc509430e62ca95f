"""Device batch assembly (cad_batcher_assemble) vs the oracle's restatement of
SunRGBDLoader::getSample (sunrgbd_loader.cpp:105-169: load, resize, augment, resize) on the same
decoded samples.  Down- and up-sampling, the identity size, BGR input, crops including the window
the reference clamps (crop_x = W - crop_w + 1 at scale 1), flips and colour jitter, mixed with
resize-only samples in one batch.  Tolerances: rgb within 2e-6 absolute (bilinear weights are the
ATen formula in fp32; the CPU kernels may fuse a multiply-add, 1 ulp), depth and K bit-exact
(nearest index and single-precision scale / K updates are the reference's own float operations)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

H, W = 48, 64


def _sample(rng, h0, w0, bgr=0, **aug):
    rgb = rng.integers(0, 256, size=(h0, w0, 3), dtype=np.uint8)
    depth = rng.integers(0, 12000, size=(h0, w0), dtype=np.uint16)
    depth[rng.random((h0, w0)) < 0.1] = 0
    K = np.array([[518.858 * w0 / 640, 0, 325.582 * w0 / 640], [0, 519.470 * h0 / 480, 253.736 * h0 / 480],
                  [0, 0, 1]], dtype=np.float32)
    return dict(rgb_np=rgb, depth_np=depth, K=K, bgr=bgr, **aug)


def _run(cad, oracle, dev, samples):
    asm = cad.BatchAssembler(len(samples), H, W)
    dsamples = []
    for s in samples:
        d = dict(s)
        d["rgb"] = torch.from_numpy(s["rgb_np"]).to(dev)
        d["depth"] = torch.from_numpy(s["depth_np"].view(np.int16)).to(dev)
        dsamples.append(d)
    rgb, depth, K = asm.assemble(dsamples)
    torch.cuda.synchronize()
    for i, s in enumerate(samples):
        r_rgb, r_depth, r_K = oracle.get_sample(s["rgb_np"], s["depth_np"], s["K"], H, W,
                                                aug=s if s.get("aug") else None, bgr=bool(s["bgr"]))
        assert (rgb[i].cpu() - r_rgb).abs().max().item() <= 2e-6, i
        assert torch.equal(depth[i].cpu(), r_depth), i
        assert torch.equal(K[i].cpu(), r_K), (i, K[i].cpu(), r_K)


def test_resize_only(cad, oracle, dev):
    rng = np.random.default_rng(0)
    _run(cad, oracle, dev, [_sample(rng, 53, 71), _sample(rng, H, W), _sample(rng, 24, 32, bgr=1),
                            _sample(rng, 100, 130), _sample(rng, 37, 200)])


def test_augmented(cad, oracle, dev):
    rng = np.random.default_rng(1)
    samples = [
        _sample(rng, 100, 130, bgr=1, aug=1, crop=1, crop_scale=0.8, crop_x=5, crop_y=3, flip=1, jitter=1,
                brightness=1.1, contrast=0.85),
        _sample(rng, 53, 71),   # resize only, mixed into the same batch
        _sample(rng, 60, 80, aug=1, crop=1, crop_scale=1.0, crop_x=1, crop_y=1),   # clamped window
        _sample(rng, H, W, aug=1, flip=1, jitter=1, brightness=0.8, contrast=1.2),  # no crop: no 2nd resize
        _sample(rng, 96, 128, aug=1, crop=1, crop_scale=0.7, crop_x=19, crop_y=14, jitter=1, brightness=1.2,
                contrast=1.2),
    ]
    _run(cad, oracle, dev, samples)


def test_sampler_driven_batch(cad, oracle, dev):
    """A training batch as the loader would build it: draws from AugSampler (seed 42, defaults)."""
    rng = np.random.default_rng(2)
    sampler = cad.AugSampler(42)
    samples = []
    for i in range(8):
        s = _sample(rng, 70 + 3 * i, 90 + 5 * i, bgr=i % 2)
        s.update(sampler.draw(H, W))
        samples.append(s)
    _run(cad, oracle, dev, samples)


def test_batch_feeds_the_step(cad, dev):
    """The assembled batch drives one training step (shapes and layouts are the step's)."""
    rng = np.random.default_rng(3)
    samples = [_sample(rng, 96, 128) for _ in range(2)]
    for s in samples:
        s["rgb"] = torch.from_numpy(s["rgb_np"]).to(dev)
        s["depth"] = torch.from_numpy(s["depth_np"].view(np.int16)).to(dev)
    rgb, depth, K = cad.BatchAssembler(2, H, W).assemble(samples)
    model = cad.BaselineUNet(3, 8, 10.0, batch=2, height=H, width=W)
    loss = cad.CombinedDepthLoss(batch=2, height=H, width=W)
    tr = cad.Trainer(model, loss, lr=1e-4, weight_decay=1e-5, grad_clip=1.0)
    l5 = tr.train_step(rgb, depth, K)
    torch.cuda.synchronize()
    assert torch.isfinite(l5).all()
