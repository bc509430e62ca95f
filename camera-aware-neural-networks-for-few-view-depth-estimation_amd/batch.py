"""Device-side batch assembly: SunRGBDLoader::getSample's resize + augmentation and the trainer's
batch stack (cad_batcher_* / cad_aug_sampler_* in include/cad/cad.h).

Reference: src/data/sunrgbd_loader.cpp getSample :105-169 (resizeSample, then augmentSample and
resizeSample again for training), resizeSample :445-489, augmentSample :352-443; the trainer stacks
samples and copies them to the device (tensorboard_trainer_enhanced.h:277-289).  Decoding (cv::imread)
stays with the caller: samples arrive as decoded u8 HWC images and u16 depth maps in device memory.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _abi
from ._abi import check


def _ptr(t: torch.Tensor):
    return C.c_void_p(t.data_ptr())


def _stream(device=None):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class AugSampler:
    """augmentSample's random draws (std::mt19937 seeded with config.random_seed, same distributions in
    the same order: crop scale, crop x, crop y, flip, brightness, contrast)."""

    def __init__(self, seed: int = 42, **config):
        self.lib = _abi.load()
        self.cfg = _abi.AugConfig(**config)
        h = C.c_void_p()
        check(self.lib.cad_aug_sampler_create(C.byref(self.cfg), seed, C.byref(h)), "cad_aug_sampler_create")
        self.h = h

    def draw(self, height: int, width: int) -> dict:
        s = _abi.Sample()
        check(self.lib.cad_aug_sampler_draw(self.h, height, width, C.byref(s)), "cad_aug_sampler_draw")
        return {k: getattr(s, k) for k in ("aug", "crop", "crop_scale", "crop_x", "crop_y", "flip", "jitter",
                                           "brightness", "contrast")}

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.cad_aug_sampler_destroy(self.h)
            self.h = None


class BatchAssembler:
    """Decoded samples -> (rgb (B,3,H,W), depth (B,1,H,W), K (B,3,3)) fp32 on the device.

    A sample is a dict: rgb (uint8 HWC device tensor), depth (16-bit HW device tensor), K (3x3),
    optional bgr (default 0), depth_scale (default 1/1000) and augmentation fields (AugSampler.draw,
    or aug=0 / absent for resize only)."""

    def __init__(self, max_batch: int, height: int, width: int, device: int = 0):
        self.lib = _abi.load()
        self.B, self.H, self.W, self.device = max_batch, height, width, device
        h = C.c_void_p()
        check(self.lib.cad_batcher_create(max_batch, height, width, device, C.byref(h)), "cad_batcher_create")
        self.h = h

    def assemble(self, samples, out=None):
        B = len(samples)
        arr = (_abi.Sample * B)()
        keep = []
        for i, s in enumerate(samples):
            rgb, dep = s["rgb"], s["depth"]
            assert rgb.dtype == torch.uint8 and rgb.dim() == 3 and rgb.shape[2] == 3 and rgb.is_contiguous()
            assert dep.element_size() == 2 and dep.dim() == 2 and dep.is_contiguous()
            keep += [rgb, dep]
            a = arr[i]
            a.rgb, a.depth = rgb.data_ptr(), dep.data_ptr()
            a.h0, a.w0 = rgb.shape[0], rgb.shape[1]
            if tuple(dep.shape) != tuple(rgb.shape[:2]):   # depth map of its own size (kv2)
                a.dh0, a.dw0 = dep.shape
            a.bgr = int(s.get("bgr", 0))
            a.depth_scale = float(s.get("depth_scale", 1.0 / 1000.0))
            K = torch.as_tensor(s["K"], dtype=torch.float32).reshape(9)
            for e in range(9):
                a.K[e] = float(K[e])
            for k in ("aug", "crop", "crop_x", "crop_y", "flip", "jitter"):
                setattr(a, k, int(s.get(k, 0)))
            for k in ("crop_scale", "brightness", "contrast"):
                setattr(a, k, float(s.get(k, 1.0)))
        dev = torch.device("cuda", self.device)
        if out is None:
            out = (torch.empty((B, 3, self.H, self.W), device=dev), torch.empty((B, 1, self.H, self.W), device=dev),
                   torch.empty((B, 3, 3), device=dev))
        rgb, depth, K = out
        check(self.lib.cad_batcher_assemble(self.h, C.cast(arr, C.c_void_p), B, _ptr(rgb), _ptr(depth), _ptr(K),
                                            _stream(dev)), "cad_batcher_assemble")
        return rgb, depth, K

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.cad_batcher_destroy(self.h)
            self.h = None


class SunRGBDDataset:
    """SunRGBDLoader's sample list and decoding (cad_dataset_*; sunrgbd_loader.cpp:39-102, 221-275):
    SunRGBDDataset(manifest_path, sensor_types=None) or SunRGBDDataset.synthetic(n, height, width).
    read(i) -> dict(rgb uint8 (h0,w0,3) RGB, depth uint16 (dh0,dw0), depth_scale, K (3,3)) on the host."""

    def __init__(self, manifest_path=None, sensor_types=None, _handle=None):
        self.lib = _abi.load()
        if _handle is not None:
            self.h = _handle
            return
        h = C.c_void_p()
        st = [s.encode() for s in (sensor_types or [])]
        arr = (C.c_char_p * max(1, len(st)))(*st)
        check(self.lib.cad_dataset_open(str(manifest_path).encode(), arr if st else None, len(st), C.byref(h)),
              "cad_dataset_open")
        self.h = h

    @classmethod
    def synthetic(cls, n, height, width, seed=42):
        lib = _abi.load()
        h = C.c_void_p()
        check(lib.cad_dataset_synthetic(n, height, width, seed, C.byref(h)), "cad_dataset_synthetic")
        return cls(_handle=h)

    def __len__(self):
        return int(self.lib.cad_dataset_size(self.h))

    def image_dir(self, i):
        d = self.lib.cad_dataset_image_dir(self.h, i)
        return d.decode() if d else None

    def read(self, i):
        import numpy as np
        info = _abi.DecodedInfo()
        check(self.lib.cad_dataset_read(self.h, i, None, 0, None, 0, C.byref(info)), "cad_dataset_read")
        rgb = np.empty((info.h0, info.w0, 3), np.uint8)
        dep = np.empty((info.dh0, info.dw0), np.uint16)
        check(self.lib.cad_dataset_read(self.h, i, rgb.ctypes.data, rgb.nbytes, dep.ctypes.data, dep.size,
                                        C.byref(info)), "cad_dataset_read")
        return {"rgb": rgb, "depth": dep, "depth_scale": info.depth_scale,
                "K": np.array(list(info.K), np.float32).reshape(3, 3)}

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.cad_dataset_destroy(self.h)
            self.h = None


class PrefetchLoader:
    """Prefetch ring (cad_loader_*): worker threads decode upcoming batches into pinned buffers, a copy
    stream uploads them, the batcher assembles them on the current stream.  Iterating an epoch yields
    (rgb (B,3,H,W), depth (B,1,H,W), K (B,3,3)) device tensors; aug = dict of AugSampler options (or
    None: resize only, the validation loader)."""

    def __init__(self, dataset: SunRGBDDataset, batch, height, width, aug=None, seed=42, threads=4, slots=2,
                 device=0):
        self.lib = _abi.load()
        self.ds, self.B, self.H, self.W, self.device = dataset, batch, height, width, device
        self._aug = _abi.AugConfig(**aug) if aug is not None else None
        h = C.c_void_p()
        check(self.lib.cad_loader_create(dataset.h, batch, height, width,
                                         C.byref(self._aug) if self._aug is not None else None, seed, threads, slots,
                                         device, C.byref(h)), "cad_loader_create")
        self.h = h

    def epoch(self, order=None):
        n = len(self.ds) if order is None else len(order)
        arr = (C.c_int64 * max(1, n))(*(order or []))
        check(self.lib.cad_loader_start_epoch(self.h, arr if order is not None else None, n), "cad_loader_start_epoch")
        dev = torch.device("cuda", self.device)
        while True:
            rgb = torch.empty((self.B, 3, self.H, self.W), device=dev)
            depth = torch.empty((self.B, 1, self.H, self.W), device=dev)
            K = torch.empty((self.B, 3, 3), device=dev)
            b = self.lib.cad_loader_next(self.h, _ptr(rgb), _ptr(depth), _ptr(K), _stream(dev))
            if b < 0:
                raise _abi.CadError("cad_loader_next failed: " + self.lib.cad_last_error().decode(errors="replace"))
            if b == 0:
                return
            yield rgb[:b], depth[:b], K[:b]

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.cad_loader_destroy(self.h)
            self.h = None
