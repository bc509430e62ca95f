"""Geometry-aware family on MI355X: GeometryAwareNetwork and
LightweightGeometryNetwork (src/models/geometry_aware_network.h) — RayEnhancedConv + FiLM blocks,
CBAM attention (src/layers/spatial_attention.h) and the Perspective Correction Layer's affine
grid_sample warp (src/layers/pcl_layer.h) — trained through libcad_hip.so (cad_geonet_*).

Pinned to the REFERENCE by tests/golden/train_geo{,lite}_* (the reference headers compiled against
LibTorch by oracle/ref_harness.cpp --model geo|geolite, one host thread) and to the oracle
restatement in fp64 (the exact-arithmetic yardstick).  The reference's single-threaded LibTorch
fp32 step sits up to 1e-2 (normalised max error) from fp64 on the level-0 gradients of the 5-level
net (the oracle run multi-threaded: 4e-6), so gradients are judged against fp64 next to the
reference's own distance from it (ours within max(1e-3, 3x the reference's)), as in
tests/test_gpu_film.py."""
import os

import pytest
import torch

from conftest import GOLDEN, geo_relu_decisions, max_rel_err

pytestmark = pytest.mark.gpu

GEO = ["train_geo_f4_b2_64x64", "train_geolite_f4_b3_48x64"]


def _net(cad, model, f, B, H, W, **kw):
    if model == "geo":
        return cad.GeometryAwareNetwork(3, f, 4, 10.0, batch=B, height=H, width=W, **kw)
    return cad.LightweightGeometryNetwork(3, f, 4, 10.0, batch=B, height=H, width=W, **kw)


def _zero_grad_bias(name, B):
    # Linear bias feeding a train-mode BatchNorm1d: exactly-zero true gradient (rounding noise only)
    return B > 1 and (name.endswith("film.fc1.bias") or name.endswith("film.fc2.bias"))


def _noise_grad_param(name, B):
    """Parameters whose gradient on a B-sample shard is rounding noise: the zero-gradient biases, and at
    B == 2 also FiLM's fc1 weight -- BatchNorm1d over two samples maps (x1, x2) to +-d / sqrt(d^2 + 4 eps)
    ~ +-1, so the gradient reaching fc1 is eps-scale and its sign is set by atomic-order rounding."""
    return _zero_grad_bias(name, B) or (B == 2 and name.endswith("film.fc1.weight"))


def cbam_decisions(net, model, oracle):
    """{CBAM prefix: (argmax pixel [B][C], argmax channel [B][H][W])} of the net's last forward
    (cad_geonet_debug_buffer "amax*/sidx*"), keyed like cad_oracle.GEO_DEBUG["force"] so the
    restatement routes its max-pool gradients exactly as the GPU run did."""
    nl, enc = oracle._geo_names(model)
    out = {}
    for l in range(1, nl):
        try:
            a = net.debug_buffer(f"amaxe{l}").long()
        except KeyError:
            return {}
        out[f"{enc[l]}.attention."] = (a, net.debug_buffer(f"sidxe{l}").long())
    for l in range(nl - 1):
        out[f"dec{l + 1}.attention."] = (net.debug_buffer(f"amaxd{l}").long(), net.debug_buffer(f"sidxd{l}").long())
    return out


def _q(err, q=0.999):
    return torch.quantile(err.flatten().double(), q).item() if err.numel() > 1 else err.max().item()


def _grad_ok(ours, g64, witnesses, k=3.0, bulk_floor=1e-4, cos_floor=0.9999):
    """One parameter gradient against fp64, next to fp32 witnesses (the reference's and/or the oracle's
    distance from fp64).  These nets carry ReLU / max-pool / argmax decisions on values that sit within
    fp32 rounding of a tie at a few elements per step: any two fp32 paths may take a different branch
    there, which moves a handful of gradient entries by O(1) (measured: the fp32 oracle alone, run on 8
    vs 16 host threads, moves one decoder gradient between 7e-6 and 5e-3).  So the bulk is held tight
    (99.9th percentile of |ours - fp64| / max|fp64| within max(1e-4, 3x the witnesses')), the direction
    too (cosine >= 0.9999), and the max only coarsely (<= max(5e-2, 3x the witnesses'))."""
    scale = g64.abs().max().item() or 1.0
    e = (ours.double() - g64).abs() / scale
    wq = max(_q((w.double() - g64).abs() / scale) for w in witnesses)
    wm = max(((w.double() - g64).abs() / scale).max().item() for w in witnesses)

    def cosine(a):
        return torch.nn.functional.cosine_similarity(a.double().reshape(1, -1), g64.reshape(1, -1)).item()
    cos = cosine(ours)
    wcos = min(cosine(w) for w in witnesses)
    ok = (_q(e) <= max(bulk_floor, k * wq) and e.max().item() <= max(5e-2, k * wm)
          and (cos >= cos_floor or 1 - cos <= k * (1 - wcos) or e.max().item() < 1e-3))
    return ok, (e.max().item(), _q(e), wq, cos)


def _state(oracle, f, model):
    s = dict(oracle.synth_init(f, model=model))
    s.update(oracle.init_buffers(f, model=model))
    return s


@pytest.mark.parametrize("name", GEO)
def test_geonet_train_steps_vs_reference_fixture(cad, dev, oracle, name):
    fx, meta = oracle.load_fixture(os.path.join(GOLDEN, name))
    model, f, B, H, W = meta["model"], meta["f"], meta["B"], meta["H"], meta["W"]
    net = _net(cad, model, f, B, H, W)
    assert net.count_parameters() == meta["num_params"]
    assert [n for n, _ in net._param_info] == [n for n, _ in oracle.param_spec(f, model=model)]
    assert [n for n, _ in net._buffer_info] == [n for n, _ in oracle.buffer_spec(f, model=model)]
    net.load_state_dict(_state(oracle, f, model))
    loss = cad.CombinedDepthLoss(*meta["weights"], batch=B, height=H, width=W)
    rgb, gt, K = fx["input.rgb"].to(dev), fx["input.gt"].to(dev), fx["input.K"].to(dev)
    rays = fx["input.rays"].to(dev)
    cam = cad.camera_from_K(K)
    assert torch.equal(cam.cpu(), fx["input.cam4"])
    # the device rays (RayDirectionComputer closed form) agree with the fixture's to rounding
    assert (cad.ray_directions(K, H, W).cpu() - fx["input.rays"]).abs().max().item() < 2e-7

    net.train()
    pred = net.forward(rgb, rays, cam)
    loss5, dpred = loss.forward_with_intrinsics(pred, gt, rgb, K)
    net.backward(dpred)
    torch.cuda.synchronize()
    assert max_rel_err(pred.cpu(), fx["step1.pred"]) < 1e-4
    assert abs(loss5[0].item() - meta["losses"][0]) <= 1e-4 * abs(meta["losses"][0])
    assert max_rel_err(dpred.cpu(), fx["step1.dpred"]) < 1e-3
    grads = net.grads()
    r64 = oracle.Trainer(oracle.synth_init(f, model=model), oracle.init_buffers(f, model=model),
                         weights=meta["weights"], dtype=torch.float64, model=model).forward_backward(
        fx["input.rgb"], fx["input.gt"], fx["input.K"])
    # a second fp32 witness of each gradient's conditioning: the oracle run multi-threaded (another
    # summation order than the single-threaded reference; e.g. an up.bias summing du over a PCL warp
    # that folds many pixels onto few is 1e-4 from fp64 in one order and 2e-3 in the other)
    r32 = oracle.Trainer(oracle.synth_init(f, model=model), oracle.init_buffers(f, model=model),
                         weights=meta["weights"], model=model).forward_backward(
        fx["input.rgb"], fx["input.gt"], fx["input.K"])
    worst, bad = [], []
    for (n, _), g32, g64 in zip(oracle.param_spec(f, model=model), r32[4], r64[4]):
        ref = fx["step1.grad." + n]
        if _zero_grad_bias(n, B):
            scale = fx["step1.grad." + n[: -len("bias")] + "weight"].abs().max().item()
            assert (grads[n] - ref).abs().max().item() / scale < 1e-2, n
            continue
        if g64.abs().max().item() == 0.0:   # e.g. a CBAM fc1 whose hidden units are all dead: exactly 0
            assert grads[n].abs().max().item() == 0.0 and ref.abs().max().item() == 0.0, n
            continue
        ok, st = _grad_ok(grads[n], g64, [ref, g32])
        worst.append((st, n))
        if not ok:
            bad.append((n, st))
    worst.sort(reverse=True)
    print("worst gradients vs fp64 ((max, p99.9, witness p99.9, cosine), name):", worst[:4])
    assert not bad, bad
    net.clip_grad_norm_(1.0)
    n64 = float(torch.sqrt(sum((g.double() ** 2).sum() for g in r64[4] if g is not None)))
    assert abs(net.last_grad_norm() - n64) <= max(1e-4 * n64, 3 * abs(meta["step1_total_norm"] - n64))
    net.adam_step(lr=meta["lr"], weight_decay=meta["wd"])

    losses = [loss5[0].item()]
    for _ in range(1, meta["steps"]):
        losses.append(net.train_step(loss, rgb, gt, K, lr=meta["lr"], weight_decay=meta["wd"], rays=rays)[0][0].item())
    t64 = oracle.Trainer(oracle.synth_init(f, model=model), oracle.init_buffers(f, model=model),
                         weights=meta["weights"], dtype=torch.float64, model=model)
    l64 = [t64.step(fx["input.rgb"], fx["input.gt"], fx["input.K"])["loss"] for _ in range(meta["steps"])]
    for ours, theirs, exact in zip(losses, meta["losses"], l64):
        assert abs(ours - exact) <= max(2e-4 * abs(exact), 3 * abs(theirs - exact)), (ours, theirs, exact)
    for n, b in net.named_buffers().items():
        ref = fx["final." + n]
        # running_mean of a FiLM BatchNorm1d follows the noise-gradient fc biases (momentum 0.1)
        tol = 0.1 * 2 * meta["lr"] * meta["steps"] if ".film.bn" in n and n.endswith("mean") else 0.0
        e64 = (t64.bufs[n] - ref.double()).abs().max().item()
        assert (b - ref).abs().max().item() <= 1e-4 * ref.abs().max().item() + 3 * e64 + tol, n
    net.eval()
    pe = net.forward(rgb, rays, cam).cpu()
    pe64 = t64.predict_eval(fx["input.rgb"], fx["input.K"])
    e_ref = max_rel_err(fx["final.pred_eval"], pe64)
    assert max_rel_err(pe, pe64) < max(1e-4, 3 * e_ref), (max_rel_err(pe, pe64), e_ref)


@pytest.mark.parametrize("engine", ["s3", "f32"])
@pytest.mark.parametrize("model,f,B,H,W", [("geo", 16, 3, 128, 192), ("geolite", 32, 3, 96, 128)])
def test_geonet_wider_step_vs_oracle(cad, dev, oracle, model, f, B, H, W, engine):
    """Wider nets (real channel counts: CBAM hidden widths > 1, PCL on 16-512 channels) vs the fp64
    oracle, next to the fp32 oracle's own distance from it, on the default S3 contraction engine and
    on the exact-fp32 one (F32: v_mfma_f32_32x32x2_f32, fmaf-chain results).  With the CBAM decisions
    pinned, these synth-init FiLM nets are still fp32-chaotic in their backward (max-pool and ReLU
    decisions within rounding of a tie; near-constant outputs): measured on MI355X, the rayfilm U-Net
    at f=16 bs3 128x192 has its decoder-input gradients 4e-2..1e-1 from fp64 in the LibTorch-fp32
    oracle (ours 8e-3..7e-2), and in this six-level net the fp32 paths land anywhere from 1e-4 to 1e-2
    of fp64 depending on the summation order (both GPU engines agree with each other to 3%).  The
    kernels themselves are pinned on well-conditioned inputs by test_op_cbam_vs_autograd /
    test_op_pcl_vs_autograd (1e-5); here the five-level net is held to 3x the two fp32 oracle runs'
    own deviation (bulk p99.9, max and 1 - cosine), the six-level net to the U-Net's floors: bulk within
    5e-3 of fp64 (or 3x the fp32 runs'), cosine >= 0.9999.  Both run with the GPU's ReLU decisions
    imposed on the oracle (round 5; cad_geonet_debug_buffer "y1/y2<e|d><l>" -> RELU_FORCE): before,
    a few pre-activations within rounding of zero flipped between the GPU and fp64 and moved whole BN
    gradients (dec2.conv.bn1.bias 2.4e-2 from fp64, floor 5e-2); with the decisions pinned the worst
    six-level tensor is 1.3e-3 (dec1.pcl.fc_transform.bias, fp32 witnesses 4.9e-3), cosine
    >= 0.999999 — a wiring error (a wrong buffer, level or channel offset) moves gradients by O(1)."""
    lib = cad.load_library()
    prev = lib.cad_get_gemm_engine()
    lib.cad_set_gemm_engine({"s3": 1, "f32": 0}[engine])
    try:
        _wider(cad, dev, oracle, model, f, B, H, W)
    finally:
        lib.cad_set_gemm_engine(prev)


def _wider(cad, dev, oracle, model, f, B, H, W):
    params, bufs = oracle.synth_init(f, model=model), oracle.init_buffers(f, model=model)
    rgb, gt, K = [torch.from_numpy(a) for a in oracle.synth_batch(B, H, W)]
    net = _net(cad, model, f, B, H, W)
    st = dict(params)
    st.update(bufs)
    net.load_state_dict(st)
    loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
    net.train()
    rg, gg, kg = rgb.to(dev), gt.to(dev), K.to(dev)
    pred = net.forward(rg, cad.ray_directions(kg, H, W), cad.camera_from_K(kg))
    _, dpred = loss.forward_with_intrinsics(pred, gg, rg, kg)
    net.backward(dpred)
    torch.cuda.synchronize()
    grads = net.grads()
    # CBAM's two max reductions route their gradient to one argmax; across ~2000 channels some top-2
    # gaps sit within fp32 rounding, so any two fp32 paths (the oracle on 8 vs 16 threads included)
    # pick different pixels for a few channels and their gradients differ by O(1) there.  The oracle
    # is therefore run with the GPU's own decisions (cad_geonet_debug_buffer "amax*/sidx*") — each
    # checked to be a true argmax of the fp64 run within 1e-4 relative, the fp32 forward's own drift
    # from fp64 at the deepest levels (4e-5 measured) — and the gradients compared tightly.
    oracle.GEO_DEBUG["force"] = cbam_decisions(net, model, oracle)
    oracle.GEO_DEBUG["gap"] = []
    # ... and with the GPU run's ReLU decisions (cad_oracle.RELU_FORCE, rebuilt from its stored pre-BN
    # conv outputs as in tests/test_gpu_model.py): a pre-activation within rounding of 0 is a tie
    # either fp32 path may break either way, and one such element moves a BN bias gradient whose
    # per-pixel terms cancel by a percent of its scale
    oracle.RELU_FORCE.update(geo_relu_decisions(net, params, f, B, H, W, model))
    try:
        r32 = oracle.Trainer(params, bufs, model=model).forward_backward(rgb, gt, K)
        nt = torch.get_num_threads()
        torch.set_num_threads(1)   # a second fp32 witness: another summation order
        try:
            r32b = oracle.Trainer(params, bufs, model=model).forward_backward(rgb, gt, K)
        finally:
            torch.set_num_threads(nt)
        r64 = oracle.Trainer(params, bufs, model=model, dtype=torch.float64).forward_backward(rgb, gt, K)
    finally:
        gaps = oracle.GEO_DEBUG.pop("gap", [])
        oracle.GEO_DEBUG.pop("force", None)
        oracle.RELU_FORCE.clear()
    assert gaps and max(gaps) < 1e-4, max(gaps)
    assert max_rel_err(pred.cpu(), r64[0]) < max(1e-4, 3 * max_rel_err(r32[0], r64[0]))
    worst, bad = [], []
    for (n, _), g32, g32b, g64 in zip(oracle.param_spec(f, model=model), r32[4], r32b[4], r64[4]):
        if _zero_grad_bias(n, B) or g64.abs().max().item() == 0.0:
            continue
        if model == "geo" and any(t in n for t in (".film.fc1.", ".film.fc2.", ".film.bn1.", ".film.bn2.")):
            # FiLM's camera MLP behind a BatchNorm1d over 3 samples: eps-dominated gradients (see
            # tests/test_gpu_film.py::_ill_conditioned); pinned by the reference fixtures above
            continue
        if model == "geo":
            ok, st = _grad_ok(grads[n], g64, [g32, g32b], bulk_floor=5e-3)
        else:
            ok, st = _grad_ok(grads[n], g64, [g32, g32b])
        worst.append((st, n))
        if not ok:
            bad.append((n, st))
    worst.sort(reverse=True)
    print("worst gradients vs fp64 ((max, p99.9, fp32-oracles p99.9, cosine), name):", worst[:4])
    if os.environ.get("CAD_GEO_ALLGRADS"):
        for st_, n_ in worst:
            print("  %-40s max %.2e p99.9 %.2e witness %.2e cos %.7f" % (n_, *st_))
    assert not bad, bad


def test_geonet_default_init_identity_pcl(cad, dev, oracle):
    """Default init (reference module defaults): fc_transform weight 0 / bias [1,1,0,0,0,0] make PCL an
    identity warp, so the network's prediction equals the oracle's with the same weights; flags
    use_pcl / use_attention off build the reduced parameter tables."""
    B, H, W, f = 2, 64, 64, 8
    net = _net(cad, "geo", f, B, H, W)
    st = net.state_dict()
    for n, v in st.items():
        if n.endswith("fc_transform.weight"):
            assert v.abs().max().item() == 0.0
        if n.endswith("fc_transform.bias"):
            assert v.tolist() == [1.0, 1.0, 0.0, 0.0, 0.0, 0.0]
    rgb, gt, K = [torch.from_numpy(a) for a in oracle.synth_batch(B, H, W)]
    net.train()
    pred = net.forward(rgb.to(dev), cad.ray_directions(K.to(dev), H, W), cad.camera_from_K(K.to(dev))).cpu()
    params = {n: v for n, v in st.items() if "running" not in n}
    bufs = {n: v for n, v in st.items() if "running" in n}
    ref = oracle.Trainer(params, bufs, model="geo", dtype=torch.float64).forward_backward(rgb, gt, K)[0]
    assert max_rel_err(pred, ref) < 1e-4
    for pcl, att in [(False, True), (True, False), (False, False)]:
        n2 = _net(cad, "geo", f, B, H, W, use_pcl=pcl, use_attention=att)
        names = [n for n, _ in n2._param_info]
        assert any(".pcl." in n for n in names) == pcl and any(".attention." in n for n in names) == att
        p2 = n2.forward(rgb.to(dev), cad.ray_directions(K.to(dev), H, W), cad.camera_from_K(K.to(dev)))
        _, d2 = cad.CombinedDepthLoss(batch=B, height=H, width=W).forward_with_intrinsics(
            p2, gt.to(dev), rgb.to(dev), K.to(dev))
        n2.backward(d2)
        torch.cuda.synchronize()
        assert torch.isfinite(p2).all() and all(torch.isfinite(g).all() for g in n2.grads().values())


def test_geonet_bench_shape_step(cad, dev):
    """GeometryAwareNetwork(f=64) train steps at 480x640 (bs 4): finite loss, prediction in (0, 10)."""
    B, H, W = 4, 480, 640
    net = cad.GeometryAwareNetwork(3, 64, 4, 10.0, batch=B, height=H, width=W)
    assert net.count_parameters() > 100_000_000
    loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
    from oracle import cad_oracle as O
    rgb, gt, K = [torch.from_numpy(a).to(dev) for a in O.synth_batch(B, H, W)]
    for _ in range(2):
        l5, pred = net.train_step(loss, rgb, gt, K)
    torch.cuda.synchronize()
    assert torch.isfinite(l5).all() and 0 < pred.min().item() and pred.max().item() < 10.0


# ---------------- operator level: CBAM and PCL against fp64 autograd ----------------
def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("B,H,W,C", [(2, 12, 20, 8), (3, 32, 48, 64), (2, 15, 20, 512)])
def test_op_cbam_vs_autograd(cad, dev, oracle, B, H, W, C):
    """cad_op_cbam (one CBAMImpl forward + backward: attn_kernels.hip) on continuous random inputs
    (no argmax near-ties) against the oracle's CBAM restatement under fp64 autograd."""
    g_ = torch.Generator().manual_seed(B * 1000 + C)
    cr = max(1, C // 16)
    x = torch.rand(B, C, H, W, generator=g_, dtype=torch.float64) * 2 - 0.5
    g = torch.randn(B, C, H, W, generator=g_, dtype=torch.float64)
    shapes = [("fc1.w", (cr, C)), ("fc1.b", (cr,)), ("fc2.w", (C, cr)), ("fc2.b", (C,)), ("sconv.w", (1, 2, 7, 7))]
    prm = {n: (torch.rand(s, generator=g_, dtype=torch.float64) * 2 - 1) * (0.5 if n != "sconv.w" else 0.2)
           for n, s in shapes}
    packed = torch.cat([prm[n].reshape(-1) for n, _ in shapes]).float()
    p = {"a.channel_attention.fc1.weight": prm["fc1.w"], "a.channel_attention.fc1.bias": prm["fc1.b"],
         "a.channel_attention.fc2.weight": prm["fc2.w"], "a.channel_attention.fc2.bias": prm["fc2.b"],
         "a.spatial_attention.conv.weight": prm["sconv.w"]}
    xr = x.clone().requires_grad_(True)
    for v in p.values():
        v.requires_grad_(True)
    out = oracle._cbam(xr, p, "a.")
    out.backward(g)
    lib = cad.load_library()
    xd, gd = _nhwc(x).float().to(dev), _nhwc(g).float().to(dev)
    pd = packed.to(dev)
    od, dxd, grd = torch.empty_like(xd), torch.empty_like(xd), torch.zeros_like(pd)
    from cad_amd.model import _ptr, _stream
    assert lib.cad_op_cbam(_ptr(xd), _ptr(gd), _ptr(pd), B, H, W, C, _ptr(od), _ptr(dxd), _ptr(grd),
                           _stream(dev)) == 0, lib.cad_last_error()
    assert max_rel_err(od.cpu(), _nhwc(out.detach())) < 1e-5
    assert max_rel_err(dxd.cpu(), _nhwc(xr.grad)) < 1e-5
    off = 0
    for (n, s), key in zip(shapes, p):
        k = int(torch.tensor(s).prod())
        assert max_rel_err(grd[off: off + k].cpu().view(s), p[key].grad) < 1e-5, n
        off += k


@pytest.mark.parametrize("B,H,W,C,scale", [(2, 16, 24, 8, 0.9), (3, 30, 40, 64, 0.6), (2, 8, 10, 256, 1.2)])
def test_op_pcl_vs_autograd(cad, dev, oracle, B, H, W, C, scale):
    """cad_op_pcl (localization MLP, affine matrix, grid_sample forward; input / grid / theta backward
    with the atomic scatter: attn_kernels.hip) against the oracle's PCL restatement (F.affine_grid +
    F.grid_sample) under fp64 autograd.  `scale` sets fc_transform's bias: < 1 folds several outputs
    onto one input pixel, > 1 samples past the border (zero padding)."""
    g_ = torch.Generator().manual_seed(B * 7 + C)
    hd = 128
    u = torch.randn(B, C, H, W, generator=g_, dtype=torch.float64)
    g = torch.randn(B, C, H, W, generator=g_, dtype=torch.float64)
    camn = torch.rand(B, 4, generator=g_, dtype=torch.float64) * 2 - 1
    shapes = [("loc_fc1.weight", (hd, C + 4)), ("loc_fc1.bias", (hd,)), ("loc_fc2.weight", (hd, hd)),
              ("loc_fc2.bias", (hd,)), ("fc_transform.weight", (6, hd)), ("fc_transform.bias", (6,))]
    p = {}
    for n, s in shapes:
        bound = 1.0 / (s[1] if len(s) > 1 else hd) ** 0.5
        p["q." + n] = (torch.rand(s, generator=g_, dtype=torch.float64) * 2 - 1) * bound
    p["q.fc_transform.weight"] *= 0.3
    p["q.fc_transform.bias"] = torch.tensor([scale, scale * 0.9, 0.1, -0.05, 0.2, 0.1], dtype=torch.float64)
    packed = torch.cat([p["q." + n].reshape(-1) for n, _ in shapes]).float()
    ur = u.clone().requires_grad_(True)
    for v in p.values():
        v.requires_grad_(True)
    out = oracle._pcl(ur, camn, p, "q.")
    out.backward(g)
    lib = cad.load_library()
    ud, gd = _nhwc(u).float().to(dev), _nhwc(g).float().to(dev)
    cd, pd = camn.float().to(dev), packed.to(dev)
    od, dud, grd = torch.empty_like(ud), torch.empty_like(ud), torch.zeros_like(pd)
    th = torch.empty(B, 6, device=dev)
    from cad_amd.model import _ptr, _stream
    assert lib.cad_op_pcl(_ptr(ud), _ptr(cd), _ptr(gd), _ptr(pd), B, H, W, C, _ptr(od), _ptr(dud), _ptr(grd),
                          _ptr(th), _stream(dev)) == 0, lib.cad_last_error()
    assert max_rel_err(od.cpu(), _nhwc(out.detach())) < 1e-5
    assert max_rel_err(dud.cpu(), _nhwc(ur.grad)) < 1e-5
    off = 0
    for n, s in shapes:
        k = int(torch.tensor(s).prod())
        assert max_rel_err(grd[off: off + k].cpu().view(s), p["q." + n].grad) < 1e-4, n
        off += k


def test_geonet_bf16_engine_step(cad, dev, oracle):
    """The geometry-aware net on the bf16 contraction engine (CAD_GEMM_BF16: bf16-rounded operands, fp32
    accumulation): a train step runs, and its prediction stays within bf16 operand rounding of the
    fp32 (S3) one."""
    B, H, W, f = 2, 64, 96, 16
    params, bufs = oracle.synth_init(f, model="geo"), oracle.init_buffers(f, model="geo")
    st = dict(params)
    st.update(bufs)
    rgb, gt, K = [torch.from_numpy(a).to(dev) for a in oracle.synth_batch(B, H, W)]
    lib = cad.load_library()
    prev = lib.cad_get_gemm_engine()
    preds = {}
    try:
        for eng in (1, 2):
            lib.cad_set_gemm_engine(eng)
            net = _net(cad, "geo", f, B, H, W)
            net.load_state_dict(st)
            loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
            l5, pred = net.train_step(loss, rgb, gt, K)
            torch.cuda.synchronize()
            assert torch.isfinite(l5).all() and all(torch.isfinite(g).all() for g in net.grads().values())
            preds[eng] = pred.cpu()
    finally:
        lib.cad_set_gemm_engine(prev)
    assert max_rel_err(preds[2], preds[1]) < 2e-2


# ---------------- data-parallel (two ranks sharing cuda:0 over gloo) ----------------
def _geo_dp_worker(rank, world, port, q):
    import os
    import sys
    import numpy as np
    import torch.distributed as dist
    from conftest import ROOT
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import cad_pkg
    cad = cad_pkg.load()
    from oracle import cad_oracle as O
    try:
        dev = torch.device("cuda", 0)
        B, H, W, f = 2, 64, 64, 8
        st = dict(O.synth_init(f, model="geolite"))
        st.update(O.init_buffers(f, model="geolite"))
        rgb, gt, K = [torch.from_numpy(a) for a in O.synth_batch(B * world, H, W)]
        sl = slice(rank * B, (rank + 1) * B)
        net = cad.LightweightGeometryNetwork(3, f, 4, 10.0, batch=B, height=H, width=W)
        net.load_state_dict(st)
        loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
        l5, _ = net.train_step(loss, rgb[sl].to(dev), gt[sl].to(dev), K[sl].to(dev), process_group=dist.group.WORLD)
        torch.cuda.synchronize()
        q.put((rank, l5[0].item(), {k: v.numpy() for k, v in net.named_parameters().items()}, net.last_grad_norm(),
               None))
    except Exception as e:   # report instead of hanging the parent on q.get
        q.put((rank, None, None, None, repr(e)))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_geonet_data_parallel_two_ranks(cad, dev, oracle):
    """GeometryAwareNetwork.train_step(process_group=...) (the flat gradient slab SUM-all-reduced, the
    1/world mean folded into the clip) on two ranks: replicas stay identical and equal a single-process
    emulation of the same two shards (per-shard forward / backward with each shard's own BatchNorm
    statistics, mean gradient, clip, Adam)."""
    import multiprocessing as mp
    import socket
    from cad_amd.model import _flat_view
    world = 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_geo_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r[0]: r[1:] for r in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
    assert all(r[-1] is None for r in res.values()), [r[-1] for r in res.values()]
    for n in res[0][1]:
        assert (res[0][1][n] == res[1][1][n]).all(), n
    assert res[0][2] == res[1][2]
    # emulation in this process: shard gradients, mean, clip + Adam on a third replica
    B, H, W, f = 2, 64, 64, 8
    st = dict(oracle.synth_init(f, model="geolite"))
    st.update(oracle.init_buffers(f, model="geolite"))
    rgb, gt, K = [torch.from_numpy(a).to(dev) for a in oracle.synth_batch(B * world, H, W)]
    gs, losses = [], []
    for r in range(world):
        net = cad.LightweightGeometryNetwork(3, f, 4, 10.0, batch=B, height=H, width=W)
        net.load_state_dict(st)
        loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
        sl = slice(r * B, (r + 1) * B)
        rays = cad.ray_directions(K[sl], H, W)
        pred = net.forward(rgb[sl], rays, cad.camera_from_K(K[sl]))
        l5, dpred = loss.forward_with_intrinsics(pred, gt[sl], rgb[sl], K[sl])
        net.backward(dpred)
        torch.cuda.synchronize()
        gs.append(_flat_view(net.flat_grads_ptr(), net.n_flat, dev).clone())
        losses.append(l5[0].item())
        assert abs(res[r][0] - losses[-1]) <= 1e-6 * abs(losses[-1]), (r, res[r][0], losses[-1])
    ref = cad.LightweightGeometryNetwork(3, f, 4, 10.0, batch=B, height=H, width=W)
    ref.load_state_dict(st)
    _flat_view(ref.flat_grads_ptr(), ref.n_flat, dev).copy_(gs[0] + gs[1])
    ref.clip_grad_norm_(1.0, 1.0 / world)
    ref.adam_step(lr=1e-4, weight_decay=1e-5)
    torch.cuda.synchronize()
    assert abs(ref.last_grad_norm() - res[0][2]) <= 1e-6 * res[0][2]
    # PCL's input gradient is an atomic scatter, so the two runs agree to rounding, not bit for bit:
    # Adam's first step (~lr * g / |g|) then differs by at most 2 lr where a gradient is rounding noise
    # — the Linear layers in front of FiLM's two-sample BatchNorm1d (_noise_grad_param) — and elsewhere
    # by lr times the relative rounding difference of the smallest gradients (measured up to 1.3e-6)
    for n, v in ref.named_parameters().items():
        d = (v - torch.from_numpy(res[0][1][n])).abs().max().item()
        assert d <= (2e-4 + 1e-7 if _noise_grad_param(n, B) else 1e-5), (n, d)
