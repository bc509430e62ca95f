"""GPU parity evidence for the bench line's "abs_rel vs CPU ref" (run on a GPU box):
    python tests/parity_report.py gpurun_out/parity.json   -> copy to profiles/parity_<round>.json

1. vs the REFERENCE itself (golden fixture from the compiled reference headers, f=4 64x64 bs2,
   3 steps): step-1 prediction / dL/dpred / gradients, losses, eval-mode prediction and abs_rel.
2. vs the oracle restatement at BASELINE configs[0]'s shape (baseline_unet f=64, bs2, 128x128,
   10 synthetic SUN-RGB-D samples = 5 steps = 1 epoch, default 4-term loss), then an eval-mode pass
   over the 10 samples: abs_rel (computeDepthMetrics, per-sample mean) GPU vs CPU, and the fp64
   oracle as the exact-arithmetic yardstick.
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import cad_pkg  # noqa: E402
from conftest import GOLDEN, max_rel_err  # noqa: E402
from oracle import cad_oracle as O  # noqa: E402


def fixture_parity(cad, dev):
    fx, meta = O.load_fixture(os.path.join(GOLDEN, "train_f4_b2_64x64"))
    f, B, H, W = meta["f"], meta["B"], meta["H"], meta["W"]
    model = cad.BaselineUNet(3, f, 10.0, batch=B, height=H, width=W)
    model.load_state_dict({k[5:]: v for k, v in fx.items() if k.startswith("init.")})
    loss = cad.CombinedDepthLoss(*meta["weights"], batch=B, height=H, width=W)
    tr = cad.Trainer(model, loss)
    rgb, gt, K = fx["input.rgb"].to(dev), fx["input.gt"].to(dev), fx["input.K"].to(dev)
    pred = model.forward(rgb)
    l5, dp = loss.forward_with_intrinsics(pred, gt, rgb, K)
    model.backward(dp)
    g = model.grads()
    out = {"pred_max_rel_err": max_rel_err(pred.cpu(), fx["step1.pred"]),
           "dpred_max_rel_err": max_rel_err(dp.cpu(), fx["step1.dpred"]),
           "worst_grad_max_rel_err": max(max_rel_err(g[n], fx["step1.grad." + n]) for n in g),
           "loss_step1": [l5[0].item(), meta["losses"][0]]}
    cad.clip_grad_norm_(model, 1.0)
    tr.optimizer.step()
    losses = [out["loss_step1"][0]] + [tr.train_step(rgb, gt, K)[0].item() for _ in range(meta["steps"] - 1)]
    model.eval()
    pe = model.forward(rgb)
    out.update(losses_gpu=losses, losses_ref=meta["losses"],
               eval_pred_max_rel_err=max_rel_err(pe.cpu(), fx["final.pred_eval"]),
               abs_rel_gpu=cad.depth_metrics(pe, gt)["abs_rel"], abs_rel_ref=meta["final_abs_rel_eval"])
    return out


def config0_parity(cad, dev):
    f, B, H, W, N = 64, 2, 128, 128, 10
    params, bufs = O.init_params(f, seed=2024), O.init_buffers(f)
    rgb, gt, K = [torch.from_numpy(a) for a in O.synth_batch(N, H, W)]
    ref, ref64 = O.Trainer(params, bufs), O.Trainer(params, bufs, dtype=torch.float64)
    model = cad.BaselineUNet(3, f, 10.0, batch=B, height=H, width=W)
    st = dict(params)
    st.update(bufs)
    model.load_state_dict(st)
    loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
    tr = cad.Trainer(model, loss)
    lg, lr_ = [], []
    for s in range(0, N, B):
        sl = slice(s, s + B)
        lr_.append(ref.step(rgb[sl], gt[sl], K[sl])["loss"])
        ref64.step(rgb[sl], gt[sl], K[sl])
        lg.append(tr.train_step(rgb[sl].to(dev), gt[sl].to(dev), K[sl].to(dev))[0].item())
    model.eval()
    pe, pr, p64 = [], [], []
    for s in range(0, N, B):
        sl = slice(s, s + B)
        pe.append(model.forward(rgb[sl].to(dev)).cpu())
        pr.append(ref.predict_eval(rgb[sl]))
        p64.append(ref64.predict_eval(rgb[sl]).float())
    pe, pr, p64 = torch.cat(pe), torch.cat(pr), torch.cat(p64)
    a_gpu = sum(cad.depth_metrics(pe[i:i + 1].contiguous().to(dev), gt[i:i + 1].to(dev))["abs_rel"] for i in range(N)) / N
    a_ref = O.abs_rel_per_sample(pr, gt)
    a_64 = O.abs_rel_per_sample(p64, gt)
    return {"shape": "baseline_unet f=64 bs2 128x128, 10 samples, 1 epoch (5 steps), 4-term loss",
            "losses_gpu": lg, "losses_cpu_ref": lr_,
            "eval_pred_max_rel_err_vs_cpu": max_rel_err(pe, pr), "eval_pred_max_rel_err_vs_fp64": max_rel_err(pe, p64),
            "cpu_fp32_eval_pred_max_rel_err_vs_fp64": max_rel_err(pr, p64),
            "abs_rel_gpu": a_gpu, "abs_rel_cpu_ref": a_ref, "abs_rel_fp64": a_64,
            "abs_rel_delta": abs(a_gpu - a_ref)}


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/parity.json"
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cad = cad_pkg.load()
    dev = torch.device("cuda", 0)
    rep = {"reference_fixture": fixture_parity(cad, dev), "config0_vs_cpu_ref": config0_parity(cad, dev)}
    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    with open(out_path, "w") as fh:
        json.dump(rep, fh, indent=1)
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
