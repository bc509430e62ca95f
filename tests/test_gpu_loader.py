"""The prefetch ring on the MI355X (cad_loader_*: worker-thread decode into pinned buffers, upload on a
copy stream, device assembly by the batcher).  Its batches must equal, bit for bit, what the batcher
makes from the same decoded samples handed over directly (test_gpu_batch.py pins the batcher to the
restated reference resize/augmentation), with augmentSample's draws taken in sample order from one
mt19937 — the reference loader's single rng_ (sunrgbd_loader.cpp:185, 352-443)."""
import json

import numpy as np
import pytest
import torch

from test_dataset import MANIFEST, _tree

pytestmark = pytest.mark.gpu

AUG = dict(enable_random_crop=1, crop_scale_min=0.7, crop_scale_max=1.0, enable_horizontal_flip=1,
           horizontal_flip_prob=0.5, enable_color_jitter=1, brightness_delta=0.2, contrast_delta=0.2)


def _direct(cad, ds, idx, H, W, sampler=None):
    """The same batch through BatchAssembler from host-decoded samples."""
    smp = []
    for i in idx:
        s = ds.read(i)
        d = {"rgb": torch.from_numpy(s["rgb"]).cuda(), "depth": torch.from_numpy(s["depth"].view(np.int16)).cuda(),
             "depth_scale": s["depth_scale"], "K": torch.from_numpy(s["K"])}
        if sampler is not None:
            d.update(sampler.draw(H, W))
        smp.append(d)
    return cad.BatchAssembler(len(idx), H, W).assemble(smp)


@pytest.mark.parametrize("aug", [False, True])
def test_loader_matches_direct_assembly_synthetic(cad, dev, aug):
    n, B, H, W = 11, 4, 48, 64
    ds = cad.SunRGBDDataset.synthetic(n, 60, 80, seed=3)
    L = cad.PrefetchLoader(ds, B, H, W, aug=AUG if aug else None, seed=42, threads=3, slots=2)
    sampler = cad.AugSampler(42, **AUG) if aug else None
    order = list(range(n))
    for epoch in range(2):   # the ring restarts cleanly; the rng continues across epochs like rng_
        got = [tuple(t.clone() for t in b) for b in L.epoch(order)]
        assert [b[0].shape[0] for b in got] == [4, 4, 3]
        for k, b in enumerate(got):
            want = _direct(cad, ds, order[k * B:(k + 1) * B], H, W, sampler)
            for x, y in zip(b, want):
                assert torch.equal(x, y), (epoch, k)
        order = order[::-1]


def test_loader_png_tree_depth_of_own_size(cad, dev, tmp_path, monkeypatch):
    man = json.load(open(MANIFEST))
    monkeypatch.chdir(tmp_path)
    _tree(tmp_path, man, with_intrinsics=lambda k: True, size=(60, 80))   # depth maps (60+k, 80+2k)
    ds = cad.SunRGBDDataset(MANIFEST)
    L = cad.PrefetchLoader(ds, 3, 48, 64, threads=2, slots=3)
    got = [tuple(t.clone() for t in b) for b in L.epoch()]
    assert [b[0].shape[0] for b in got] == [3, 1]
    for k, b in enumerate(got):
        want = _direct(cad, ds, list(range(k * 3, min(4, k * 3 + 3))), 48, 64)
        for x, y in zip(b, want):
            assert torch.equal(x, y)


def test_loader_reports_decode_errors(cad, dev, tmp_path, monkeypatch):
    man = json.load(open(MANIFEST))
    monkeypatch.chdir(tmp_path)
    _tree(tmp_path, man, with_intrinsics=lambda k: True)
    for f in (tmp_path / man["images"][2]["path"] / "depth").iterdir():
        f.unlink()
    ds = cad.SunRGBDDataset(MANIFEST)
    L = cad.PrefetchLoader(ds, 2, 32, 32)
    it = L.epoch()
    next(it)   # samples 0, 1
    with pytest.raises(cad.CadError, match="sample 2: Depth image not found"):
        next(it)
    # the loader is reusable after an error
    assert sum(b[0].shape[0] for b in L.epoch([0, 1, 3])) == 3
