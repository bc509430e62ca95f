"""Two training steps of the config-5 network (ResNet-50 encoder + U-Net decoder, resunet.cpp) on
cuda:0, saved for the A/B checks of its fused / alternative paths (tests/test_gpu_resunet_switches.py
runs it with one CAD_* switch at 0 and at its default and compares the files).
    python tools/resunet_ab.py <fp8 0|1> B H W out.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    fp8, B, H, W, out = int(sys.argv[1]), *map(int, sys.argv[2:5]), sys.argv[5]
    import cad_pkg
    cad = cad_pkg.load()
    from cad_amd import synthetic
    dev = torch.device("cuda:0")
    model = cad.ResNetUNet(batch=B, height=H, width=W, fp8=bool(fp8))
    loss = cad.CombinedDepthLoss(1.0, 0.1, 0.001, 0.01, batch=B, height=H, width=W)
    rgb, gt, K = synthetic.device_batch(B, H, W, dev)
    res = {}
    for s in range(2):
        pred = model.forward(rgb)
        loss5, dpred = loss.forward_with_intrinsics(pred, gt, rgb, K)
        model.backward(dpred)
        torch.cuda.synchronize()
        res[f"loss{s}"] = loss5.detach().cpu().clone()
        res[f"pred{s}"] = pred.detach().cpu().clone()
        if s == 0:
            for n, g in model.grads().items():
                res["grad." + n] = g.clone()
        model.clip_grad_norm_(1.0)
        model.adam_step(lr=1e-4, weight_decay=1e-5)
    for n, p in model.named_parameters().items():
        res["param." + n] = p.clone()
    torch.cuda.synchronize()
    torch.save(res, out)


if __name__ == "__main__":
    main()
