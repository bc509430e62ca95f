"""configs[4]'s per-GPU step (ResNet-50 encoder + U-Net decoder, bs32 480x640, full loss, bf16 GEMM
operands; --fp8: forward conv-GEMMs on MXFP8 E4M3) for rocprofv3 runs: profiles/collect.sh <tag> 5|5x8.
  python3 profiles/c5_step.py [--fp8] [--steps K] [--warmup W]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import cad_pkg

ap = argparse.ArgumentParser()
ap.add_argument("--fp8", action="store_true")
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--warmup", type=int, default=1)
args = ap.parse_args()
cad = cad_pkg.load()
from cad_amd import synthetic
B, H, W = 32, 480, 640
dev = torch.device('cuda', 0)
m = cad.ResNetUNet(batch=B, height=H, width=W, fp8=args.fp8)
loss = cad.CombinedDepthLoss(1.0, 0.1, 0.001, 0.01, batch=B, height=H, width=W)
rgb, gt, K = (t.to(dev) for t in synthetic.device_batch(B, H, W, "cpu"))
pred = torch.empty((B, 1, H, W), device=dev); dpred = torch.empty_like(pred); l5 = torch.zeros(5, device=dev)
for _ in range(args.warmup):
    m.train_step(loss, rgb, gt, K, pred=pred, dpred=dpred, loss5=l5)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(args.steps):
    m.train_step(loss, rgb, gt, K, pred=pred, dpred=dpred, loss5=l5)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / max(1, args.steps)
print(f'{{"ms_per_step": {dt * 1e3:.3f}, "images_per_s": {B / dt:.3f}, "fp8": {str(args.fp8).lower()}, '
      f'"last_loss": {l5[0].item()!r}}}')
