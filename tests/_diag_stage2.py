"""Debug tool: recompute decoder-level-1 (dec2) backward in fp64 from OUR forward buffers and our
stage-1 output gradient, and compare each intermediate with what the HIP kernels produced."""
import ctypes as C
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import cad_pkg  # noqa: E402

cad = cad_pkg.load()
from oracle import cad_oracle as O  # noqa: E402
from conftest import max_rel_err  # noqa: E402

dev = torch.device("cuda", 0)
f, B, H, W = 64, 1, 64, 64
l = 1
params = O.init_params(f, seed=f)
bufs = O.init_buffers(f)
rgb, gt, K = [torch.from_numpy(a) for a in O.synth_batch(B, H, W)]
st = dict(params)
st.update(bufs)
m = cad.BaselineUNet(3, f, 10.0, batch=B, height=H, width=W)
m.load_state_dict(st)
L = cad.CombinedDepthLoss(batch=B, height=H, width=W)
rg, gg, kg = rgb.to(dev), gt.to(dev), K.to(dev)
pr = m.forward(rg)
_, dp = L.forward_with_intrinsics(pr, gg, rg, kg)
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
assert m.lib.cad_unet_backward_stage(m.h, 0, C.c_void_p(dp.data_ptr()), s) == 0
assert m.lib.cad_unet_backward_stage(m.h, 1, C.c_void_p(dp.data_ptr()), s) == 0
Cl, Hl, Wl = f << l, H >> l, W >> l
M = B * Hl * Wl
g_in = m.debug_buffer("Sa")[: M * Cl].view(B, Hl, Wl, Cl).permute(0, 3, 1, 2).double()
y1 = m.debug_buffer(f"dec{l}.y1").view(B, Hl, Wl, Cl).permute(0, 3, 1, 2).double()
# a1 = relu(bn1(y1)) is never materialised: conv2's loaders apply it on the fly
a1 = F.relu(F.batch_norm(y1, None, None, None, None, True, 0.1, 1e-5))
y2 = m.debug_buffer(f"dec{l}.y2").view(B, Hl, Wl, Cl).permute(0, 3, 1, 2).double()
cat = m.debug_buffer(f"cat{l}").view(B, Hl, Wl, 2 * Cl).permute(0, 3, 1, 2).double()
w1 = params[f"dec{l + 1}.conv.conv1.weight"].double()
w2 = params[f"dec{l + 1}.conv.conv2.weight"].double()
assert m.lib.cad_unet_backward_stage(m.h, 2, C.c_void_p(dp.data_ptr()), s) == 0
torch.cuda.synchronize()
dY1_ours = m.debug_buffer("Sb")[: M * Cl].view(B, Hl, Wl, Cl).permute(0, 3, 1, 2).double()
dcat_ours = m.debug_buffer(f"dcat{l}").view(B, Hl, Wl, 2 * Cl).permute(0, 3, 1, 2).double()

# fp64 recomputation from our inputs
print("fwd check y2 == conv(a1):", max_rel_err(y2, F.conv2d(a1, w2, None, 1, 1)))
print("fwd check y1 == conv(cat):", max_rel_err(y1, F.conv2d(cat, w1, None, 1, 1)))
y2r = y2.clone().requires_grad_()
out2 = F.relu(F.batch_norm(y2r, None, None, None, None, True, 0.1, 1e-5))
out2.backward(g_in)
dY2 = y2r.grad
a1r = a1.clone().requires_grad_()
F.conv2d(a1r, w2, None, 1, 1).backward(dY2)
dA1 = a1r.grad
y1r = y1.clone().requires_grad_()
F.relu(F.batch_norm(y1r, None, None, None, None, True, 0.1, 1e-5)).backward(dA1)
dY1 = y1r.grad
catr = cat.clone().requires_grad_()
F.conv2d(catr, w1, None, 1, 1).backward(dY1)
print("dY1 ours vs fp64-from-our-inputs:", max_rel_err(dY1_ours, dY1))
print("dcat ours vs fp64:", max_rel_err(dcat_ours, catr.grad))
print("sum dz check: ", (dY1_ours - dY1).abs().sum((0, 2, 3))[:8])
# mean/var conditioning of y1 / y2 channels
for nm, t in [("y1", y1), ("y2", y2)]:
    mu = t.mean((0, 2, 3))
    sd = t.std((0, 2, 3))
    print(nm, "max |mean|/std", (mu.abs() / sd).max().item())
