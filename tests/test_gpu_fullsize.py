"""Parity at the benchmarked size: one configs[1] training step (baseline_unet f=64, bs32, 480x640,
loss weights 1,0,0,0, fp32 = the S3 engine) on the MI355X against the oracle restatement run on the
box's host cores in fp32 (oracle/cad_oracle.py, ATen CPU — the same kernels the reference
dispatches; pinned to the reference's own fixtures by tests/test_oracle_golden.py).

This is the only parity check that exercises what the headline step alone exercises:
  * the ~680-slab two-level split-K reduction of the L0 weight gradients (conv_kernels.hip
    finish_slabs; the 64 x 576 GEMMs over 9.8 M pixels),
  * activation buffers past 4 GB (the dec1 concat buffer is 5 GB at bs32),
  * BatchNorm statistics over 9.8 M pixels per channel,
  * the global clip norm over all 31,037,633 gradients and the Adam step on them.

Step = TensorBoardTrainerEnhanced::trainEpoch body (tensorboard_trainer_enhanced.h:287-304).
Tolerances (fp32 vs fp32, different summation orders; the north-star's 1e-3 relative):
  prediction <= 1e-4 normalised max error (north-star bound 1e-3), loss <= 1e-5 relative (1e-4 bound),
  dL/dpred <= 1e-3, grad norm <= 1e-4 relative; parameter gradients are judged against the oracle
  in fp64 (the exact-arithmetic yardstick), like the small-size tests: cosine >= 0.9999 and normalised
  max error <= max(1e-2, 3x the fp32 oracle's own error).  A weight gradient in front of a train-mode
  BatchNorm sums millions of mean-free terms, so fp32 rounding on EITHER side is relatively large
  there (measured on MI355X: bottleneck.conv.conv2.weight is 3.7e-2 normalised max error from fp64,
  the LibTorch-fp32 oracle 2.9e-2, both at cosine 0.99998).  BN running stats <= 1e-4; parameters
  after Adam within 2 lr, moving by more than rounding only where the two fp32 gradients may disagree
  in sign (Adam's first step is lr * g / (|g| + eps): |g| within 3x their max error against fp64,
  checked element by element); the eval-mode prediction / abs_rel of the updated model <= 1e-4.
Host memory: the CPU autograd graph of the fp32 oracle step at bs32 480x640 is ~80 GB (the box allows
270 GB); the fp64 yardstick's (~160 GB) lives in the GPU's 288 GB HBM, after the product's buffers are
freed."""
import sys
import threading
import time

import pytest
import torch

from conftest import max_rel_err

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

B, H, W, F = 32, 480, 640, 64
WEIGHTS = (1.0, 0.0, 0.0, 0.0)


_CAPMAN = [None]


def _beat(msg, t0):
    # progress to the real terminal: pytest's fd-level capture swallows even sys.__stderr__, and a long
    # CPU oracle step must not look like a hung GPU job (a runner that sees no output for minutes
    # kills it), so global capture is suspended around the line
    line = f"[fullsize +{time.time() - t0:6.1f}s] {msg}"
    cm = _CAPMAN[0]
    if cm is None:
        print(line, file=sys.__stderr__, flush=True)
        return
    with cm.global_and_fixture_disabled():
        print(line, file=sys.stderr, flush=True)


def _heartbeat(t0, stop, period=30.0):
    while not stop.wait(period):
        _beat("... oracle still running", t0)


@pytest.mark.timeout(1500)
def test_bs32_480x640_train_step_vs_oracle(cad, dev, oracle, pytestconfig):
    _CAPMAN[0] = pytestconfig.pluginmanager.getplugin("capturemanager")
    t0 = time.time()
    stop = threading.Event()
    threading.Thread(target=_heartbeat, args=(t0, stop), daemon=True).start()
    try:
        _run(cad, dev, oracle, t0)
    finally:
        stop.set()


def _run(cad, dev, oracle, t0):
    params, bufs = oracle.init_params(F, seed=42), oracle.init_buffers(F)
    rgb, gt, K = [torch.from_numpy(a) for a in oracle.synth_batch(B, H, W)]

    # ---- MI355X: forward, loss + dL/dpred, backward, clip, Adam (one step) ----
    model = cad.BaselineUNet(3, F, 10.0, batch=B, height=H, width=W)
    assert model.count_parameters() == 31037633
    state = dict(params)
    state.update(bufs)
    model.load_state_dict(state)
    loss = cad.CombinedDepthLoss(*WEIGHTS, batch=B, height=H, width=W)
    tr = cad.Trainer(model, loss, lr=1e-4, weight_decay=1e-5, grad_clip=1.0)
    rg, gg, kg = rgb.to(dev), gt.to(dev), K.to(dev)
    model.train()
    _beat("model built; GPU forward", t0)
    pred = model.forward(rg)
    loss5, dpred = loss.forward_with_intrinsics(pred, gg, rg, kg)
    torch.cuda.synchronize()
    _beat("GPU forward + loss done; backward", t0)
    model.backward(dpred)
    torch.cuda.synchronize()
    g_pred, g_dpred, g_loss5 = pred.cpu(), dpred.cpu(), loss5.cpu()
    g_grads = model.grads()
    cad.clip_grad_norm_(model, 1.0)
    tr.optimizer.step()
    torch.cuda.synchronize()
    g_norm = model.last_grad_norm()
    g_params, g_bufs = model.named_parameters(), model.named_buffers()
    model.eval()
    g_eval = model.forward(rg[:4]).cpu()
    g_absrel = cad.depth_metrics(g_eval.to(dev), gg[:4])["abs_rel"]
    del model, loss, tr, pred, dpred
    torch.cuda.empty_cache()
    _beat("GPU step done; oracle step on the host cores", t0)

    # ---- oracle on the host: fp32 (the reference's arithmetic), then fp64 (the yardstick) ----
    ref = oracle.Trainer(params, bufs, weights=WEIGHTS)
    r = ref.step(rgb, gt, K)
    _beat(f"oracle fp32 step done (loss {r['loss']:.6f}, ours {g_loss5[0].item():.6f})", t0)
    # the fp64 yardstick is the same restatement evaluated by ATen's GPU kernels in fp64 (its host
    # evaluation took 220 s of the session's budget; any exact-enough arithmetic is a yardstick)
    g64 = [g.cpu() for g in oracle.Trainer(params, bufs, weights=WEIGHTS, dtype=torch.float64,
                                           device=dev).forward_backward(rgb, gt, K)[4]]
    torch.cuda.empty_cache()
    _beat("oracle fp64 forward/backward (ATen GPU kernels) done", t0)

    e_pred = max_rel_err(g_pred, r["pred"])
    assert e_pred < 1e-4, e_pred
    assert abs(g_loss5[0].item() - r["loss"]) <= 1e-5 * abs(r["loss"]), (g_loss5.tolist(), r["loss"])
    assert abs(g_loss5[1].item() - r["comps"]["si_loss"]) <= 1e-5 * abs(r["comps"]["si_loss"])
    assert max_rel_err(g_dpred, r["dpred"]) < 1e-3
    assert abs(g_norm - r["norm"]) <= 1e-4 * r["norm"], (g_norm, r["norm"])
    worst, flip_thr = [], {}
    for (n, _), g32, gd in zip(oracle.param_spec(F), r["grads"], g64):
        ours = g_grads[n]
        cos = torch.nn.functional.cosine_similarity(ours.double().reshape(1, -1), gd.reshape(1, -1)).item()
        worst.append((max_rel_err(ours, gd), max_rel_err(g32, gd), n, cos))
        # a gradient element whose sign the two fp32 paths may disagree on: |g| within 3x the larger
        # of the two paths' max error against fp64
        err = max((ours.double() - gd).abs().max().item(), (g32.double() - gd).abs().max().item())
        flip_thr[n] = (gd, 3 * err)
    del g64
    worst.sort(reverse=True)
    _beat(f"gradients vs fp64 (ours, fp32 oracle, name, cosine): {worst[:4]}; "
          f"lowest cosine {min(w[3] for w in worst):.7f}", t0)
    bad = [w for w in worst if not (w[3] >= 0.9999 and w[0] <= max(1e-2, 3 * w[1]))]
    assert not bad, bad
    lr, wd, eps = 1e-4, 1e-5, 1e-8
    coef = min(1.0, 1.0 / (r["norm"] + 1e-6))   # clip_grad_norm_(1.0) scale of the oracle step
    moved, diag = [], []
    ref_g32 = {n: g for (n, _), g in zip(oracle.param_spec(F), r["grads"])}
    for n, p in g_params.items():
        d = (p - ref.p[n]).abs()
        # Adam's first step is lr * g' / (|g'| + eps) with g' = clipped g + wd * w (coupled L2): a weight
        # moves by more than rounding only where the two fp32 paths may disagree on g' — its sign, or
        # its size where |g'| is comparable to eps
        g, thr = flip_thr[n]
        g_adam = (g * coef + wd * params[n].double()).abs()
        flip = d > 1e-5
        un = flip & (g_adam > max(thr * coef, 100 * eps))
        unexplained = int(un.sum())
        moved.append((unexplained, d.max().item(), int(flip.sum()), n))
        if unexplained:   # what each side saw for those weights
            w0 = params[n].double()
            idx = un.nonzero()[:4]
            diag.append((n, thr * coef, [(tuple(i.tolist()), (g * coef)[tuple(i)].item(), (g_grads[n].double() * coef)[tuple(i)].item(),
                                         (ref_g32[n].double() * coef)[tuple(i)].item(), (wd * w0)[tuple(i)].item(),
                                         (p.double() - w0)[tuple(i)].item(), (ref.p[n].double() - w0)[tuple(i)].item())
                                        for i in idx]))
    moved.sort(reverse=True)
    _beat(f"params after Adam (unexplained moves, max |diff|, moves > 1e-5, name): {moved[:3]}", t0)
    for dg in diag:
        _beat(f"unexplained {dg[0]} thr {dg[1]:.3e}: (index, fp64 g, ours, fp32 oracle, wd*w, our step, oracle step) {dg[2]}", t0)
    assert all(u == 0 and mx <= 2 * lr + 1e-6 for u, mx, _, _ in moved), moved[:3]
    for n, b in g_bufs.items():
        assert max_rel_err(b, ref.bufs[n]) < 1e-4, n
    # eval-mode forward of the updated model (BN running statistics) and the metric's abs_rel
    r_eval = ref.predict_eval(rgb[:4])
    assert max_rel_err(g_eval, r_eval) < 1e-4
    r_absrel = oracle.abs_rel_per_sample(r_eval, gt[:4])
    assert abs(g_absrel - r_absrel) <= 1e-4 * r_absrel, (g_absrel, r_absrel)
    _beat(f"pred {e_pred:.2e}; abs_rel gpu {g_absrel:.6f} cpu {r_absrel:.6f}", t0)
