"""Synthetic SUN-RGB-D-shaped batches — the bench / smoke input generator.

Real SUN RGB-D is absent here (data/sunrgbd is git-ignored upstream, .MISSING_LARGE_BLOBS), so the
path is exercised on counter-based synthetic batches: splitmix64(seed, index) -> u32 ->
(u >> 8) * 2^-24, so that every consumer regenerates identical bytes.
  rgb  (B,3,H,W) i.i.d. U[0,1)                                     seed 0xC0FFEE
  gt   (B,1,H,W) 0.5 + 9(0.5 + 0.5 sin(2pi(u/W 1.3 + v/H 0.7 + 0.1 b))) clamped [0.5, 9.5],
       0 where U < 0.15 (seed 0xD3E7) and over the top H/16 rows (Kinect-style holes)
  K    (B,3,3) NYU/kv1 (even b) and Xtion (odd b) calibrations scaled by (W/640, H/480) like
       sunrgbd_loader.cpp:480-488
"""
from __future__ import annotations

import math

import numpy as np


def _splitmix64(seed: int, idx: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform01(seed: int, n: int, start: int = 0) -> np.ndarray:
    out = np.empty(n, np.float32)
    chunk = 1 << 24
    for a in range(0, n, chunk):
        idx = np.arange(start + a, start + min(n, a + chunk), dtype=np.uint64)
        u = (_splitmix64(seed, idx) >> np.uint64(32)).astype(np.uint32)
        out[a:a + len(idx)] = (u >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return out


def intrinsics(B: int, H: int, W: int) -> np.ndarray:
    K = np.zeros((B, 3, 3), np.float32)
    sx, sy = np.float32(W / 640.0), np.float32(H / 480.0)
    for b in range(B):
        fx, fy, cx, cy = ((518.858, 519.470, 325.582, 253.736) if b % 2 == 0 else (570.342, 570.342, 320.0, 240.0))
        K[b, 0, 0] = np.float32(fx) * sx
        K[b, 0, 2] = np.float32(cx) * sx
        K[b, 1, 1] = np.float32(fy) * sy
        K[b, 1, 2] = np.float32(cy) * sy
        K[b, 2, 2] = 1.0
    return K


def batch(B: int, H: int, W: int, rgb_seed: int = 0xC0FFEE, hole_seed: int = 0xD3E7):
    """Returns numpy (rgb, gt, K)."""
    rgb = uniform01(rgb_seed, B * 3 * H * W).reshape(B, 3, H, W)
    b = np.arange(B, dtype=np.float64)[:, None, None]
    v = np.arange(H, dtype=np.float64)[None, :, None]
    u = np.arange(W, dtype=np.float64)[None, None, :]
    d = np.clip(0.5 + 9.0 * (0.5 + 0.5 * np.sin(2.0 * math.pi * (u / W * 1.3 + v / H * 0.7 + 0.1 * b))), 0.5, 9.5)
    holes = uniform01(hole_seed, B * H * W).reshape(B, H, W) < np.float32(0.15)
    holes |= np.arange(H)[None, :, None] < H // 16
    gt = np.where(holes, 0.0, d).astype(np.float32).reshape(B, 1, H, W)
    return rgb, gt, intrinsics(B, H, W)


def device_batch(B: int, H: int, W: int, device):
    import torch
    rgb, gt, K = batch(B, H, W)
    return (torch.from_numpy(rgb).to(device), torch.from_numpy(gt).to(device), torch.from_numpy(K).to(device))
