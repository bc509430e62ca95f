"""Diagnostic (GPU box): the dec2.conv.bn1.bias gradient (sum over pixels of g1 * relu mask) on the
GPU vs the fp64 / fp32 oracle, with the block's intermediates captured on the oracle side.

  python profiles/diag_bn1.py [f B H W seed]"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cad_pkg  # noqa: E402
from oracle import cad_oracle as O  # noqa: E402

torch.set_num_threads(16)
CAP = {}
_orig = O._double_conv


def _dc(x, p, bufs, pre, train, cam=None):
    if pre != "dec2.conv.":
        return _orig(x, p, bufs, pre, train, cam)
    y1 = O._conv3x3(x, p[pre + "conv1.weight"])
    y1.retain_grad()
    z1 = O._bn(y1, p, bufs, pre + "bn1", train)
    z1.retain_grad()
    a1 = F.relu(z1)
    a1.retain_grad()
    y2 = O._conv3x3(a1, p[pre + "conv2.weight"])
    z2 = O._bn(y2, p, bufs, pre + "bn2", train)
    CAP[x.dtype] = dict(x=x, y1=y1, z1=z1, a1=a1)
    return F.relu(z2)


O._double_conv = _dc


def main():
    f, B, H, W, seed = (int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (16, 2, 64, 96, 16)))
    cad = cad_pkg.load()
    lib = cad.load_library()
    dev = torch.device("cuda", 0)
    params, bufs = O.init_params(f, seed=seed), O.init_buffers(f)
    rgb, gt, K = [torch.from_numpy(a) for a in O.synth_batch(B, H, W)]
    r32 = O.Trainer(params, bufs).forward_backward(rgb, gt, K)
    r64 = O.Trainer(params, bufs, dtype=torch.float64).forward_backward(rgb, gt, K)
    names = [n for n, _ in O.param_spec(f)]
    ib = names.index("dec2.conv.bn1.bias")
    c64, c32 = CAP[torch.float64], CAP[torch.float32]
    g64 = c64["a1"].grad
    dz64 = c64["z1"].grad
    print("fp64 dbeta", r64[4][ib][:8].tolist())
    print("fp32 dbeta", r32[4][ib][:8].tolist())
    print("sum(dz64)", dz64.sum((0, 2, 3))[:8].tolist())
    print("cond: sum|dz| / |sum dz|", (dz64.abs().sum((0, 2, 3)) / dz64.sum((0, 2, 3)).abs())[:8].tolist())
    print("sum(g1 64) per channel (structural ~0)", g64.sum((0, 2, 3))[:8].tolist(), "vs sum|g1|",
          g64.abs().sum((0, 2, 3))[:4].tolist())
    for eng, name in ((1, "s3"), (0, "f32")):
        lib.cad_set_gemm_engine(eng)
        m = cad.BaselineUNet(3, f, 10.0, batch=B, height=H, width=W)
        st = dict(params)
        st.update(bufs)
        m.load_state_dict(st)
        loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
        rg, gg, kg = rgb.to(dev), gt.to(dev), K.to(dev)
        pred = m(rg)
        _, dpred = loss.forward_with_intrinsics(pred, gg, rg, kg)
        torch.cuda.synchronize()
        C = c64["y1"].shape[1]
        hh, ww = c64["y1"].shape[2], c64["y1"].shape[3]
        y1g = m.debug_buffer("dec1_y1").reshape(B, hh, ww, C).permute(0, 3, 1, 2).double()
        m.backward(dpred)
        torch.cuda.synchronize()
        grads = m.grads()
        db = grads["dec2.conv.bn1.bias"].double()
        e = (db - r64[4][ib]).abs().max().item() / r64[4][ib].abs().max().item()
        ey = (y1g - c64["y1"]).abs().max().item() / c64["y1"].abs().max().item()
        # the GPU's relu decisions: BN of its own y1 with fp64 statistics of its y1
        mu = y1g.mean((0, 2, 3), keepdim=True)
        var = y1g.var((0, 2, 3), unbiased=False, keepdim=True)
        zg = (y1g - mu) / torch.sqrt(var + 1e-5) * params["dec2.conv.bn1.weight"].double().view(1, -1, 1, 1) + \
            params["dec2.conv.bn1.bias"].double().view(1, -1, 1, 1)
        flips = ((zg > 0) != (c64["z1"] > 0)).sum().item()
        alt = (g64 * (zg > 0)).sum((0, 2, 3))
        ealt = (alt - r64[4][ib]).abs().max().item() / r64[4][ib].abs().max().item()
        near = (c64["z1"].abs() < 1e-4).sum().item()
        print(f"== {name}: dbeta err {e:.3e}; y1 err {ey:.3e}; relu flips {flips} of {zg.numel()} (|z|<1e-4: {near}); "
              f"fp64 g1 with GPU mask -> dbeta err {ealt:.3e}")
        print("   ours dbeta", db[:8].tolist())


if __name__ == "__main__":
    main()
