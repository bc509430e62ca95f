"""The backward's second stream (csrc/host/cad_api.cpp wgrad_stream): on the S3 engine the
conv / ConvT weight gradients run beside the dgrad chain, reading bn2's / bn1's dL/dz from two buffer
pairs that the step's stream may only rewrite after the side's last reader (events evA / evB).  The
stream a kernel runs on changes no arithmetic, so three train steps with the overlap on
(CAD_SIDE_WGRAD=1), off (=0) and at the default must agree bit for bit, on both GEMM engines; a missing
wait (a pair rewritten while a weight gradient still reads it) shows up as a difference here.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

F, B, H, W = 32, 4, 96, 128


@pytest.fixture
def engine(cad, request):
    lib = cad.load_library()
    prev = lib.cad_get_gemm_engine()
    assert lib.cad_set_gemm_engine(request.param) == 0
    yield request.param
    lib.cad_set_gemm_engine(prev)


def _run(cad, state, batch, side):
    prev = os.environ.get("CAD_SIDE_WGRAD")
    if side is None:
        os.environ.pop("CAD_SIDE_WGRAD", None)
    else:
        os.environ["CAD_SIDE_WGRAD"] = side
    try:
        m = cad.BaselineUNet(3, F, 10.0, batch=B, height=H, width=W)
        m.load_state_dict(state)
        loss = cad.CombinedDepthLoss(1.0, 0.1, 0.001, 0.01, batch=B, height=H, width=W)
        tr = cad.Trainer(m, loss, lr=1e-4, weight_decay=1e-5, grad_clip=1.0)
        losses = [tr.train_step(*batch).clone() for _ in range(3)]
        torch.cuda.synchronize()
        return m.flat_params.clone(), torch.stack(losses), tr.pred.clone(), m.last_grad_norm()
    finally:
        if prev is None:
            os.environ.pop("CAD_SIDE_WGRAD", None)
        else:
            os.environ["CAD_SIDE_WGRAD"] = prev


@pytest.mark.parametrize("engine", [1, 2], ids=["s3", "bf16"], indirect=True)
def test_side_stream_weight_gradients_bit_identical(cad, dev, oracle, engine):
    params, bufs = oracle.init_params(F, seed=11), oracle.init_buffers(F)
    state = dict(params)
    state.update(bufs)
    batch = [torch.from_numpy(a).to(dev) for a in oracle.synth_batch(B, H, W)]
    ref = _run(cad, state, batch, "0")
    for side in ("1", None):
        got = _run(cad, state, batch, side)
        assert torch.equal(got[0], ref[0]), f"CAD_SIDE_WGRAD={side}: parameters differ"
        assert torch.equal(got[1], ref[1]), f"CAD_SIDE_WGRAD={side}: losses differ"
        assert torch.equal(got[2], ref[2]), f"CAD_SIDE_WGRAD={side}: predictions differ"
        assert got[3] == ref[3]
