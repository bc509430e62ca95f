"""Debug tool (not collected by pytest): stage-by-stage backward parity vs the fp64 oracle."""
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

torch.set_num_threads(16)
dev = torch.device("cuda", 0)


def run(f, B, H, W):
    params = O.init_params(f, seed=f)
    bufs = O.init_buffers(f)
    rgb, gt, K = [torch.from_numpy(a) for a in O.synth_batch(B, H, W)]
    # fp64 oracle with captured intermediates
    p = {k: v.double().requires_grad_() for k, v in params.items()}
    bb = {k: v.double().clone() for k, v in bufs.items()}
    acts = {}

    def keep(name, t):
        t.retain_grad()
        acts[name] = t
        return t

    x = rgb.double()
    s1 = keep("s1", O._double_conv(x, p, bb, "enc1.", True))
    s2 = keep("s2", O._double_conv(F.max_pool2d(s1, 2), p, bb, "enc2.conv.", True))
    s3 = keep("s3", O._double_conv(F.max_pool2d(s2, 2), p, bb, "enc3.conv.", True))
    s4 = keep("s4", O._double_conv(F.max_pool2d(s3, 2), p, bb, "enc4.conv.", True))
    xb = keep("bott", O._double_conv(F.max_pool2d(s4, 2), p, bb, "bottleneck.conv.", True))
    d3 = keep("dout3", O._decoder(xb, s4, p, bb, "dec4.", True))
    d2 = keep("dout2", O._decoder(d3, s3, p, bb, "dec3.", True))
    d1 = keep("dout1", O._decoder(d2, s2, p, bb, "dec2.", True))
    d0 = keep("dout0", O._decoder(d1, s1, p, bb, "dec1.", True))
    pred = torch.sigmoid(F.conv2d(d0, p["out_conv.weight"], p["out_conv.bias"])) * 10.0
    loss, _ = O.combined_loss(pred, gt.double(), x, K.double())
    loss.sum().backward()

    st = dict(params)
    st.update(bufs)
    m = cad.BaselineUNet(3, f, 10.0, batch=B, height=H, width=W)
    m.load_state_dict(st)
    L = cad.CombinedDepthLoss(batch=B, height=H, width=W)
    rg, gg, kg = rgb.to(dev), gt.to(dev), K.to(dev)
    pr = m.forward(rg)
    _, dp = L.forward_with_intrinsics(pr, gg, rg, kg)
    torch.cuda.synchronize()

    def nhwc(t):
        return t.detach().permute(0, 2, 3, 1).reshape(-1)

    for nm, buf in [("s1", None), ("dout0", "dout0"), ("dout1", "dout1"), ("bott", "bott")]:
        if buf:
            print("  fwd", nm, max_rel_err(m.debug_buffer(buf), nhwc(acts[nm])))
    lib = m.lib
    import ctypes as C
    names = [n for n, _ in O.param_spec(f)]
    after = {1: "dout1", 2: "dout2", 3: "dout3", 4: "bott"}
    for s in range(m.num_stages):
        assert lib.cad_unet_backward_stage(m.h, s, C.c_void_p(dp.data_ptr()),
                                           C.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
        torch.cuda.synchronize()
        off, cnt = m.stage_ranges[s]
        gr = m.grads()
        errs = []
        for n in names:
            pi = [i for i, (nn, _) in enumerate(m._param_info) if nn == n][0]
            # params belonging to this stage
            from cad_amd import _abi  # noqa
        stage_params = {0: ["out_conv."], 1: ["dec1."], 2: ["dec2."], 3: ["dec3."], 4: ["dec4."], 5: ["bottleneck."],
                        6: ["enc4."], 7: ["enc3."], 8: ["enc2."], 9: ["enc1."]}[s]
        for n in names:
            if any(n.startswith(q) for q in stage_params):
                errs.append((n, round(max_rel_err(gr[n], p[n].grad), 6)))
        line = f"stage {s}: " + ", ".join(f"{a}={b}" for a, b in errs)
        if s in after:
            g = acts[after[s]].grad
            sa = m.debug_buffer("Sa")[: g.numel()]
            line += f" | d{after[s]}={max_rel_err(sa, nhwc(g)):.3e}"
        print(line)


if __name__ == "__main__":
    for cfg in [(64, 1, 64, 64), (32, 1, 64, 64)]:
        print("config", cfg)
        run(*cfg)
