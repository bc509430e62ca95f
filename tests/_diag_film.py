"""Diagnostic (GPU): per-parameter gradient error of the FiLM models, ours vs the fp64 oracle next to
the fp32 oracle's own distance from fp64 — separates kernel bugs from fp32 ill-conditioning.
    python tests/_diag_film.py [model f B H W]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import cad_pkg  # noqa: E402
from conftest import max_rel_err  # noqa: E402
from oracle import cad_oracle as O  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "rayfilm"
f, B, H, W = (int(x) for x in sys.argv[2:6]) if len(sys.argv) > 5 else (4, 3, 64, 96)
torch.set_num_threads(16)
cad = cad_pkg.load()
dev = torch.device("cuda", 0)
params, bufs = O.synth_init(f, model=model), O.init_buffers(f, model=model)
rgb, gt, K = [torch.from_numpy(a) for a in O.synth_batch(B, H, W)]
r32 = O.Trainer(params, bufs, model=model).forward_backward(rgb, gt, K)
r64 = O.Trainer(params, bufs, model=model, dtype=torch.float64).forward_backward(rgb, gt, K)
cls = {"film": cad.IntrinsicsConditionedUNet, "rayfilm": cad.RayConditionedUNet}[model]
net = cls(3, f, 4, 10.0, batch=B, height=H, width=W)
st = dict(params)
st.update(bufs)
net.load_state_dict(st)
loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
rg, gg, kg = rgb.to(dev), gt.to(dev), K.to(dev)
pred = net.forward_cam(rg, cad.camera_from_K(kg))
_, dp = loss.forward_with_intrinsics(pred, gg, rg, kg)
net.backward(dp)
g = net.grads()
print("pred  ours-64 %.2e  r32-64 %.2e" % (max_rel_err(pred.cpu(), r64[0]), max_rel_err(r32[0], r64[0])))
print("dpred ours-64 %.2e  r32-64 %.2e" % (max_rel_err(dp.cpu(), r64[1]), max_rel_err(r32[1], r64[1])))
for (n, _), a32, a64 in zip(O.param_spec(f, model=model), r32[4], r64[4]):
    if a64 is None:
        continue
    e_o, e_r = max_rel_err(g[n], a64), max_rel_err(a32, a64)
    cos = torch.nn.functional.cosine_similarity(g[n].double().reshape(1, -1), a64.reshape(1, -1)).item()
    flag = "  <<<" if e_o > max(1e-3, 5 * e_r) else ""
    print("%-40s ours %.2e  r32 %.2e  cos %.6f%s" % (n, e_o, e_r, cos, flag))

# per-term dL/dpred precision at this shape (pred from the forward above)
p = pred.detach().cpu()
for w in [(1, 0, 0, 0), (0, 1, 0, 0), (0, 0, 1, 0), (0, 0, 0, 1)]:
    lw = cad.CombinedDepthLoss(*w, batch=B, height=H, width=W)
    _, d_ours = lw.forward_with_intrinsics(pred, gg, rg, kg)
    _, _, d32 = O.loss_and_dpred(p, gt, rgb, K, w)
    _, _, d64 = O.loss_and_dpred(p.double(), gt.double(), rgb.double(), K.double(), w)
    e_o, e_r = max_rel_err(d_ours.cpu(), d64), max_rel_err(d32, d64)
    idx = (d_ours.cpu().double() - d64).abs().argmax().item()
    print("loss term %s: dpred ours %.2e  r32 %.2e  worst flat idx %d ours %.4e ref64 %.4e max|d64| %.3e"
          % (w, e_o, e_r, idx, d_ours.cpu().reshape(-1)[idx].item(), d64.reshape(-1)[idx].item(), d64.abs().max().item()))
