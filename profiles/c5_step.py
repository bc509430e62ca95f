import sys, time
sys.path.insert(0, '.')
import torch
import cad_pkg
cad = cad_pkg.load()
from cad_amd import synthetic
B, H, W = 32, 480, 640
dev = torch.device('cuda', 0)
m = cad.ResNetUNet(batch=B, height=H, width=W)
loss = cad.CombinedDepthLoss(1.0, 0.1, 0.001, 0.01, batch=B, height=H, width=W)
rgb, gt, K = (t.to(dev) for t in synthetic.device_batch(B, H, W, "cpu"))
pred = torch.empty((B, 1, H, W), device=dev); dpred = torch.empty_like(pred); l5 = torch.zeros(5, device=dev)
for _ in range(4):
    m.train_step(loss, rgb, gt, K, pred=pred, dpred=dpred, loss5=l5)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    m.train_step(loss, rgb, gt, K, pred=pred, dpred=dpred, loss5=l5)
torch.cuda.synchronize()
print("ms/step", (time.perf_counter() - t0) / 3 * 1e3)
