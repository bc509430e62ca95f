"""Diagnostic (GPU box): every parameter gradient of one small U-Net step on each fp32 GEMM engine
against the fp64 oracle, next to the LibTorch-fp32 oracle's own distance (the witness).  Prints one
line per parameter: bulk / max normalised error of ours and of the witness, cosine.

  python profiles/diag_grads.py [f B H W seed]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import cad_pkg  # noqa: E402
from oracle import cad_oracle as O  # noqa: E402

torch.set_num_threads(16)


def q(e):
    return torch.quantile(e, 0.999).item() if e.numel() > 1 else e.max().item()


def main():
    f, B, H, W, seed = (int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (16, 2, 64, 96, 16)))
    model = sys.argv[6] if len(sys.argv) > 6 else "baseline"
    cad = cad_pkg.load()
    lib = cad.load_library()
    dev = torch.device("cuda", 0)
    params, bufs = O.init_params(f, seed=seed, model=model), O.init_buffers(f, model=model)
    rgb, gt, K = [torch.from_numpy(a) for a in O.synth_batch(B, H, W)]
    r32 = O.Trainer(params, bufs, model=model).step(rgb, gt, K)
    r64 = O.Trainer(params, bufs, model=model, dtype=torch.float64).step(rgb, gt, K)
    out = {}
    for eng, name in ((1, "s3"), (0, "f32")):
        lib.cad_set_gemm_engine(eng)
        cls = {"baseline": cad.BaselineUNet, "film": cad.IntrinsicsConditionedUNet, "rayfilm": cad.RayConditionedUNet}[model]
        m = cls(3, f, 10.0, batch=B, height=H, width=W)
        st = dict(params)
        st.update(bufs)
        m.load_state_dict(st)
        loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
        rg, gg, kg = rgb.to(dev), gt.to(dev), K.to(dev)
        pred = m(rg, cad.camera_from_K(kg)) if m.conditioned else m(rg)
        _, dpred = loss.forward_with_intrinsics(pred, gg, rg, kg)
        m.backward(dpred)
        torch.cuda.synchronize()
        out[name] = (pred.cpu(), dpred.cpu(), m.grads())
    for name, (pred, dpred, grads) in out.items():
        pe = (pred.double() - r64["pred"]).abs().max().item() / r64["pred"].abs().max().item()
        de = (dpred.double() - r64["dpred"]).abs().max().item() / r64["dpred"].abs().max().item()
        pw = (r32["pred"].double() - r64["pred"]).abs().max().item() / r64["pred"].abs().max().item()
        dw = (r32["dpred"].double() - r64["dpred"]).abs().max().item() / r64["dpred"].abs().max().item()
        print(f"== engine {name}: pred {pe:.2e} (witness {pw:.2e}) dpred {de:.2e} (witness {dw:.2e})")
        for (n, _), g32, g64 in zip(O.param_spec(f, model=model), r32["grads"], r64["grads"]):
            if g64 is None:
                continue
            s = g64.abs().max().item() or 1.0
            e = (grads[n].double() - g64).abs().flatten() / s
            ew = (g32.double() - g64).abs().flatten() / s
            cos = torch.nn.functional.cosine_similarity(grads[n].double().reshape(1, -1), g64.reshape(1, -1)).item()
            flag = " <<<" if q(e) > max(5e-3, 3 * q(ew)) else ""
            print(f"  {n:40s} bulk {q(e):.2e} (w {q(ew):.2e})  max {e.max().item():.2e} (w {ew.max().item():.2e})  "
                  f"cos {cos:.7f}{flag}")


if __name__ == "__main__":
    main()
