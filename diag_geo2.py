import sys, os; R = os.path.dirname(os.path.abspath(__file__)); sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import torch
import cad_pkg
from oracle import cad_oracle as O
from conftest import max_rel_err
cad = cad_pkg.load()
dev = torch.device("cuda", 0)
torch.set_num_threads(16)
f, B, H, W = 16, 3, 64, 96
WT = (1.0, 0.0, 0.0, 0.0)
pcl, att = False, False
spec0 = O._geo_spec(f, 3, "geo", pcl, att)
O._cbam = lambda x, p, pre: x
O._pcl = lambda x, cam, p, pre: x
base_spec = O.param_spec
O.param_spec = lambda f_=64, in_ch=3, model="baseline": spec0 if model == "geo" else base_spec(f_, in_ch, model)
params, bufs = O.synth_init(f, model="geo"), O.init_buffers(f, model="geo")
rgb, gt, K = [torch.from_numpy(a) for a in O.synth_batch(B, H, W)]
net = cad.GeometryAwareNetwork(3, f, 4, 10.0, pcl, att, batch=B, height=H, width=W)
st = dict(params); st.update(bufs); net.load_state_dict(st)
loss = cad.CombinedDepthLoss(*WT, batch=B, height=H, width=W)
rg, gg, kg = rgb.to(dev), gt.to(dev), K.to(dev)
pred = net.forward(rg, cad.ray_directions(kg, H, W), cad.camera_from_K(kg))
_, dpred = loss.forward_with_intrinsics(pred, gg, rg, kg)
net.backward(dpred); torch.cuda.synchronize()
keep32 = {}
O.GEO_DEBUG["keep"] = keep32
r32 = O.Trainer(params, bufs, weights=WT, model="geo").forward_backward(rgb, gt, K)
keep = {}
O.GEO_DEBUG["keep"] = keep
r64 = O.Trainer(params, bufs, weights=WT, model="geo", dtype=torch.float64).forward_backward(rgb, gt, K)
print("dpred ours", max_rel_err(dpred.cpu(), r64[1]), "oracle32", max_rel_err(r32[1], r64[1]))
def nhwc(t):
    return t.detach().permute(0, 2, 3, 1).reshape(-1)
for l in range(4, -1, -1):
    for k in ("u", "cat", "x"):
        ours = net.debug_buffer(f"{k}{l}")
        ref = keep[f"{k}{l}"]
        print(k, l, "fwd", max_rel_err(ours, nhwc(ref)))
    g = keep[f"cat{l}"].grad
    ours = net.debug_buffer(f"dcat{l}").view(B, H >> l, W >> l, -1)
    C = ours.shape[-1] // 2
    gr = g.permute(0, 2, 3, 1)
    g32 = keep32[f"cat{l}"].grad.permute(0, 2, 3, 1)
    print("dcat", l, "up ours", max_rel_err(ours[..., C:], gr[..., C:]), "oracle32", max_rel_err(g32[..., C:], gr[..., C:]), flush=True)
    if l == 0:
        gx = keep[f"x{l}"].grad
        print("  x0 grad exists", gx is not None)
    if keep[f"x{l}"].grad is not None:
        pass
