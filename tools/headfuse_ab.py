"""One training step of a U-Net on cuda:0, saved for the level-0 head-fusion A/B
(tests/test_gpu_headfuse.py runs it with CAD_HEADFUSE=0 and =1 and compares the files bitwise).
    python tools/headfuse_ab.py <model baseline|film|rayfilm> <engine 1|2> f B H W out.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    kind, eng, f, B, H, W, out = sys.argv[1], int(sys.argv[2]), *map(int, sys.argv[3:7]), sys.argv[7]
    import cad_pkg
    cad = cad_pkg.load()
    from cad_amd import synthetic
    dev = torch.device("cuda:0")
    cad.load_library().cad_set_gemm_engine(eng)
    cls = {"baseline": cad.BaselineUNet, "film": cad.IntrinsicsConditionedUNet, "rayfilm": cad.RayConditionedUNet}[kind]
    torch.manual_seed(f * 7 + B)
    args = (3, f, 10.0) if kind == "baseline" else (3, f, 4, 10.0)   # FiLM models take camera_dim
    model = cls(*args, batch=B, height=H, width=W)
    loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
    tr = cad.Trainer(model, loss)
    rgb, gt, K = synthetic.device_batch(B, H, W, dev)
    res = {}
    for s in range(2):
        res[f"loss{s}"] = tr.train_step(rgb, gt, K)[0].detach().cpu().clone()
        res[f"pred{s}"] = tr.pred.detach().cpu().clone()
    for n, g in model.grads().items():
        res["grad." + n] = g.detach().cpu().clone()
    for n, p in model.named_parameters().items():
        res["param." + n] = p.detach().cpu().clone()
    torch.cuda.synchronize()
    torch.save(res, out)


if __name__ == "__main__":
    main()
