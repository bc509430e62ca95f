"""Data-parallel training step on the MI355X.

* libcad's own RCCL exchange (Communicator / cad_unet_backward_allreduce, the path build/train
  runs) on a single-rank communicator: every collective is then the identity, so the trajectory
  must equal the plain single-process Trainer bit for bit — this pins the bucketing, the event
  hand-off between the compute and communication streams and the 1/world prescale.
* two ranks sharing cuda:0 over torch.distributed gloo (RCCL refuses two ranks on one device, and
  the 8-GPU runs are the driver's): each rank trains its shard through cad.Trainer's decoder-first
  bucketed all-reduce; the replicas must stay identical and equal the oracle's single-process
  emulation of DP (per-shard loss and BN statistics, mean gradient, global clip, Adam).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import grad_close, ROOT, max_rel_err

pytestmark = pytest.mark.gpu

F, B, H, W = 16, 2, 64, 96
WEIGHTS = (1.0, 0.1, 0.001, 0.01)


def _model(cad, state, batch=B):
    m = cad.BaselineUNet(3, F, 10.0, batch=batch, height=H, width=W)
    m.load_state_dict(state)
    return m, cad.CombinedDepthLoss(*WEIGHTS, batch=batch, height=H, width=W)


def test_single_rank_communicator_matches_plain(cad, dev, oracle):
    params, bufs = oracle.init_params(F, seed=5), oracle.init_buffers(F)
    state = dict(params)
    state.update(bufs)
    rgb, gt, K = [torch.from_numpy(a).to(dev) for a in oracle.synth_batch(B, H, W)]
    comm = cad.Communicator(cad.Communicator.unique_id(), 1, 0, 0)
    assert (comm.rank(), comm.size()) == (0, 1)
    # collectives on one rank: identity (sum and max), in place
    t = torch.randn(1000, device=dev)
    ref = t.clone()
    comm.allreduce(t)
    comm.allreduce(t, "max")
    torch.cuda.synchronize()
    assert torch.equal(t, ref)
    out = {}
    for use_comm in (False, True):
        m, loss = _model(cad, state)
        if use_comm:
            comm.broadcast_parameters(m)
        tr = cad.Trainer(m, loss, lr=1e-4, weight_decay=1e-5, grad_clip=1.0, communicator=comm if use_comm else None,
                         bucket_mb=0.5)   # 0.5 MB buckets: several buckets at f=16
        if use_comm:   # exchange accounting (bench.py's N > 1 "exchange" block) must not change the step
            tr.set_exchange_timing(True)
        losses = [tr.train_step(rgb, gt, K).clone() for _ in range(3)]
        torch.cuda.synchronize()
        out[use_comm] = (m.flat_params.clone(), torch.stack(losses), tr.pred.clone(), m.last_grad_norm())
        if use_comm:
            xs = tr.exchange_stats()
            assert xs["comm_size"] == 1 and xs["calls"] == 3 and xs["timed_calls"] == 3
            assert xs["bytes"] == 3 * 4 * m.n_flat or xs["bytes"] >= 3 * 4 * m.count_parameters()
            assert xs["buckets"] >= 3 * 2   # several buckets per step at 0.5 MB
            assert xs["exposed_ms"] >= 0 and xs["span_ms"] >= 0
            again = tr.exchange_stats()   # read resets
            assert again["calls"] == 0 and again["timed_calls"] == 0 and again["bytes"] == 0
        del tr, m, loss
    assert torch.equal(out[True][0], out[False][0])
    assert torch.equal(out[True][1], out[False][1])
    assert torch.equal(out[True][2], out[False][2])
    assert out[True][3] == out[False][3]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import cad_pkg
    cad = cad_pkg.load()
    from oracle import cad_oracle as O
    try:
        dev = torch.device("cuda", 0)
        params, bufs = O.init_params(F, seed=7), O.init_buffers(F)
        state = dict(params)
        state.update(bufs)
        rgb, gt, K = [torch.from_numpy(a) for a in O.synth_batch(B * world, H, W)]
        sl = slice(rank * B, (rank + 1) * B)
        m, loss = _model(cad, state)
        tr = cad.Trainer(m, loss, lr=1e-4, weight_decay=1e-5, grad_clip=1.0, process_group=dist.group.WORLD,
                         bucket_mb=0.5)
        l = tr.train_step(rgb[sl].to(dev), gt[sl].to(dev), K[sl].to(dev))[0].item()
        torch.cuda.synchronize()
        # numpy, not torch tensors: torch shares tensor storage through file descriptors that vanish
        # when this process exits
        np_ = lambda d: {k: v.numpy() for k, v in d.items()}
        # grads(): the exchanged mean gradient as the clip left it (clip scales in place)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from conftest import gpu_relu_decisions
        masks = np_(gpu_relu_decisions(m, params, F, B, H, W))   # this shard's ReLU decisions
        q.put((rank, l, m.flat_params.cpu().numpy(), np_(m.named_parameters()), np_(m.named_buffers()),
               m.last_grad_norm(), np_(m.grads()), masks, None))
    except Exception as e:   # report instead of hanging the parent on q.get
        q.put((rank, None, None, None, None, None, None, None, repr(e)))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_step_vs_oracle_dp(oracle):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r[0]: r[1:] for r in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
    assert all(r[-1] is None for r in res.values()), [r[-1] for r in res.values()]
    # replicas identical after the exchange
    assert (res[0][1] == res[1][1]).all()
    assert res[0][4] == res[1][4]
    # oracle emulation: per-shard forward/backward (own BN batch statistics), mean, clip, Adam
    params, bufs = oracle.init_params(F, seed=7), oracle.init_buffers(F)
    rgb, gt, K = [torch.from_numpy(a) for a in oracle.synth_batch(B * world, H, W)]
    shard, grads, grads64 = [], [], []
    for r in range(world):   # each shard with its replica's ReLU decisions (see test_gpu_model.py)
        oracle.RELU_FORCE.update({k: torch.from_numpy(v) for k, v in res[r][6].items()})
        try:
            t = oracle.Trainer(params, bufs, weights=WEIGHTS)
            sh = (rgb[r * B:(r + 1) * B], gt[r * B:(r + 1) * B], K[r * B:(r + 1) * B])
            _, _, lr_, _, g = t.forward_backward(*sh)
            # the exact-arithmetic yardstick: the same shard in fp64
            grads64.append(oracle.Trainer(params, bufs, weights=WEIGHTS, dtype=torch.float64).forward_backward(*sh)[4])
        finally:
            oracle.RELU_FORCE.clear()
        shard.append(t)
        grads.append(g)
        assert abs(res[r][0] - float(lr_)) <= 1e-4 * abs(float(lr_)), (r, res[r][0], float(lr_))
    mean = [sum(gs) / world for gs in zip(*grads)]
    mean64 = [sum(gs) / world for gs in zip(*grads64)]
    t = oracle.Trainer(params, bufs, weights=WEIGHTS)
    t.apply(mean)
    lr, wd, eps = 1e-4, 1e-5, 1e-8
    norm = float(torch.sqrt(sum((g.double() ** 2).sum() for g in mean)))
    assert abs(res[0][4] - norm) <= 1e-4 * norm, (res[0][4], norm)
    coef = min(1.0, 1.0 / (norm + 1e-6))   # clip_grad_norm_(1.0)
    bad = []
    for (n, _), g32, gd in zip(oracle.param_spec(F), mean, mean64):
        ours = torch.from_numpy(res[0][5][n]).double() / coef   # exchanged mean, before the clip scale
        assert torch.equal(torch.from_numpy(res[1][5][n]), torch.from_numpy(res[0][5][n])), n
        cos = torch.nn.functional.cosine_similarity(ours.reshape(1, -1), gd.reshape(1, -1)).item()
        e, e32 = max_rel_err(ours, gd), max_rel_err(g32, gd)
        ok, st = grad_close(ours, gd, [g32], bulk_floor=5e-3)   # criterion of test_gpu_model.py
        if not (cos >= 0.9999 and ok):
            bad.append(("grad", n, cos, e, e32, st))
        d = (torch.from_numpy(res[0][2][n]) - t.p[n]).abs()
        if d.max().item() > 2 * lr + 1e-6:
            bad.append(("step", n, d.max().item()))
        # Adam's first step is lr * g' / (|g'| + eps), g' = clipped g + wd * w: a weight moves by more
        # than rounding only where the two fp32 paths may disagree on g' (its sign, or its size where
        # |g'| is eps-sized), i.e. |g'| within 3x the larger path error against fp64
        err = max((ours - gd).abs().max().item(), (g32.double() - gd).abs().max().item())
        g_adam = (gd * coef + wd * params[n].double()).abs()
        flip = d > 1e-5
        if not (g_adam[flip] <= max(3 * err * coef, 100 * eps)).all():
            bad.append(("adam", n, int(flip.sum()), err, g_adam[flip].max().item()))
    assert not bad, bad
    # BN running statistics stay per replica: each rank's equal its own shard's
    for r in range(world):
        for n, b in res[r][3].items():
            assert max_rel_err(torch.from_numpy(b), shard[r].bufs[n]) < 1e-4, (r, n)


@pytest.mark.parametrize("model,engine", [("baseline", 1), ("baseline", 2), ("rayfilm", 2)])
def test_backward_stage_writes_stay_in_range(cad, dev, oracle, model, engine):
    """The overlapped exchange (cad_unet_backward_allreduce, dp.cpp) all-reduces a bucket in place on
    the communicator's stream while the compute stream runs the later backward stages; that is only
    correct if no stage writes a gradient outside its own slab range.  Fill the slab with
    a sentinel, run the backward stage by stage, and check after each stage that it changed nothing
    outside [offset, offset + count) — in particular nothing of the buckets already handed over."""
    lib = cad.load_library()
    prev = lib.cad_get_gemm_engine()
    lib.cad_set_gemm_engine(engine)
    try:
        f, B, H, W = 16, 2, 64, 64
        cls = {"baseline": cad.BaselineUNet, "rayfilm": cad.RayConditionedUNet}[model]
        m = cls(3, f, max_depth=10.0, batch=B, height=H, width=W)
        rgb, gt, K = [torch.from_numpy(a).to(dev) for a in oracle.synth_batch(B, H, W)]
        loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
        pred = m(rgb, cad.camera_from_K(K)) if m.conditioned else m(rgb)
        _, dpred = loss.forward_with_intrinsics(pred, gt, rgb, K)
        torch.cuda.synchronize()
        m.flat_grads.fill_(1234.5)
        snaps = [m.flat_grads.clone()]

        def on_stage(s, off, cnt):
            torch.cuda.synchronize()
            cur = m.flat_grads.clone()
            changed = (cur != snaps[-1]).nonzero().flatten()
            outside = changed[(changed < off) | (changed >= off + cnt)]
            assert outside.numel() == 0, (s, off, cnt, outside[:8].tolist())
            snaps.append(cur)
        m.backward(dpred, on_stage=on_stage)
        torch.cuda.synchronize()
        assert len(snaps) == m.num_stages + 1
        # every parameter gradient was written by some stage
        assert not (m.flat_grads == 1234.5).all()
    finally:
        lib.cad_set_gemm_engine(prev)


def _family(cad, oracle, family, B=2, H=64, W=64):
    if family == "resunet":
        from oracle import resunet_oracle as R
        p, b = R.init(seed=3)
        m = cad.ResNetUNet(batch=B, height=H, width=W)
        m.load_state_dict({**p, **b})
        step = lambda loss, rgb, gt, K, **kw: m.train_step(loss, rgb, gt, K, **kw)
    else:
        m = cad.GeometryAwareNetwork(3, 8, 4, 10.0, batch=B, height=H, width=W) if family == "geo" else \
            cad.LightweightGeometryNetwork(3, 8, 4, 10.0, batch=B, height=H, width=W)
        step = lambda loss, rgb, gt, K, **kw: m.train_step(loss, rgb, gt, K, **kw)
    return m, step


@pytest.mark.parametrize("family", ["resunet", "geo", "geolite"])
def test_other_families_staged_backward(cad, dev, oracle, family):
    """configs[4]'s network and the geometry-aware ones back-propagate in stages (cad_resunet_ /
    cad_geonet_backward_stage) that write only their own slab ranges (the overlapped exchange's
    invariant, as test_backward_stage_writes_stay_in_range) and together equal the one-call backward
    bit for bit."""
    B, H, W = 2, 64, 64
    m, _ = _family(cad, oracle, family, B, H, W)
    rgb, gt, K = [torch.from_numpy(a).to(dev) for a in oracle.synth_batch(B, H, W)]
    loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
    fwd = (lambda: m.forward(rgb)) if family == "resunet" else \
        (lambda: m.forward(rgb, cad.ray_directions(K, H, W), cad.camera_from_K(K)))
    pred = fwd()
    _, dpred = loss.forward_with_intrinsics(pred, gt, rgb, K)
    m.backward(dpred)
    torch.cuda.synchronize()
    plain = m.flat_grads.clone()
    pred = fwd()
    _, dpred = loss.forward_with_intrinsics(pred, gt, rgb, K)
    torch.cuda.synchronize()
    m.flat_grads.fill_(1234.5)
    snaps = [m.flat_grads.clone()]

    def on_stage(s, off, cnt):
        torch.cuda.synchronize()
        cur = m.flat_grads.clone()
        changed = (cur != snaps[-1]).nonzero().flatten()
        outside = changed[(changed < off) | (changed >= off + cnt)]
        assert outside.numel() == 0, (family, s, off, cnt, outside[:8].tolist())
        snaps.append(cur)
    m.backward(dpred, on_stage=on_stage)
    torch.cuda.synchronize()
    assert len(snaps) == m.num_stages + 1
    staged = m.flat_grads.clone()
    touched = staged != 1234.5
    assert torch.equal(staged[touched], plain[touched]), family
    assert (plain[~touched] == 0).all()   # untouched = alignment padding, zero in the plain run


@pytest.mark.parametrize("family", ["resunet", "geo"])
def test_other_families_single_rank_communicator_matches_plain(cad, dev, oracle, family):
    """train_step(communicator=...) — the staged backward with the RCCL bucket exchange on the
    communicator's stream (cad_resunet_ / cad_geonet_backward_allreduce) — on one rank equals the
    plain step bit for bit over three steps (identity all-reduce, stream hand-off, 1/world prescale)."""
    B, H, W = 2, 64, 64
    rgb, gt, K = [torch.from_numpy(a).to(dev) for a in oracle.synth_batch(B, H, W)]
    comm = cad.Communicator(cad.Communicator.unique_id(), 1, 0, 0)
    out = {}
    for use in (False, True):
        m, step = _family(cad, oracle, family, B, H, W)
        if use:
            comm.broadcast_parameters(m)
        loss = cad.CombinedDepthLoss(batch=B, height=H, width=W)
        losses = [step(loss, rgb, gt, K, communicator=comm if use else None, bucket_mb=0.25)[0].clone()
                  for _ in range(3)]
        torch.cuda.synchronize()
        out[use] = (m.flat_params.clone(), torch.stack(losses))
        del m, loss
    assert torch.equal(out[True][0], out[False][0]) and torch.equal(out[True][1], out[False][1])
