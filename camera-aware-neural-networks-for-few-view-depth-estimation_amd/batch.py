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
            assert dep.element_size() == 2 and dep.shape == rgb.shape[:2] and dep.is_contiguous()
            keep += [rgb, dep]
            a = arr[i]
            a.rgb, a.depth = rgb.data_ptr(), dep.data_ptr()
            a.h0, a.w0 = rgb.shape[0], rgb.shape[1]
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
