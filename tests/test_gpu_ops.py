"""Operator-level parity of the HIP kernels (through the C ABI's cad_op_* entry points) against
the oracle's ATen CPU ops in fp64 — the contractions of SURVEY.md §8(a) a1-a5 at real channel
counts on small spatial sizes, including masked tails (M, N not multiples of the tile) and the
strided/offset views the U-Net uses for its concat buffer.  Tolerance: normalised max error
<= 1e-5 (fp32 MFMA accumulation vs fp64)."""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

from conftest import max_rel_err

pytestmark = pytest.mark.gpu

TOL = 2e-5


ENGINES = {"f32": 0, "s3": 1, "bf16": 2}


@pytest.fixture(params=list(ENGINES))
def engine(request, cad):
    """The contractions run on any GEMM engine (cad.h CAD_GEMM_*): exact fp32 MFMA, S3 (exact 3-way
    bf16 split on the bf16 matrix cores) or bf16 (operands rounded to bf16, fp32 accumulation).  All
    meet the same tolerance — for bf16 against the fp64 contraction of the bf16-ROUNDED operands
    (see q()), i.e. the only admitted error is fp32 accumulation."""
    lib = cad.load_library()
    prev = lib.cad_get_gemm_engine()
    assert lib.cad_set_gemm_engine(ENGINES[request.param]) == 0
    yield request.param
    lib.cad_set_gemm_engine(prev)


def q(t, engine):
    """The operand values the engine multiplies: bf16 round-to-nearest-even for the bf16 engine."""
    return t.bfloat16().float() if engine == "bf16" else t


def _p(t):
    return C.c_void_p(t.data_ptr())


def _s():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


CONV_SHAPES = [  # B, H, W, cin, cout
    (2, 16, 24, 4, 64), (2, 16, 16, 64, 64), (1, 8, 12, 128, 256), (2, 6, 8, 1024, 512), (3, 10, 14, 32, 16),
    (2, 4, 4, 8, 4), (1, 30, 40, 256, 128),
    # M <= 64 with N > 64: the 64x256 tile (bottleneck at small images)
    (1, 4, 4, 512, 1024), (1, 8, 8, 256, 512), (2, 3, 4, 64, 128),
    # few-channel input (enc1.conv1) at several split-K slices, two output-channel blocks
    (2, 40, 64, 4, 128), (1, 48, 96, 8, 64),
]


@pytest.mark.parametrize("B,H,W,cin,cout", CONV_SHAPES)
def test_conv3x3_fwd_dgrad_wgrad(cad, dev, engine, B, H, W, cin, cout):
    lib = cad.load_library()
    g = torch.Generator().manual_seed(B * 1000 + cin + cout)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    dy = torch.randn(B, cout, H, W, generator=g)
    xd, wd, dyd = q(x, engine).double().requires_grad_(), q(w, engine).double().requires_grad_(), q(dy, engine).double()
    y_ref = F.conv2d(xd, wd, None, 1, 1)
    y_ref.backward(dyd)
    # forward, written at channel offset 4 of a wider row (concat-buffer view)
    ld = cout + 8
    ybuf = torch.zeros(B, H, W, ld, device=dev)
    xg, wg = nhwc(x).to(dev), w.permute(0, 2, 3, 1).contiguous().to(dev)
    assert lib.cad_op_conv3x3_fwd(_p(xg), cin, 0, cin, _p(wg), cout, _p(ybuf), ld, 4, B, H, W, _s()) == 0
    torch.cuda.synchronize()
    assert max_rel_err(nchw(ybuf[..., 4:4 + cout].cpu()), y_ref.detach()) < TOL
    assert ybuf[..., :4].abs().max().item() == 0 and ybuf[..., 4 + cout:].abs().max().item() == 0
    # dgrad
    dx = torch.zeros(B, H, W, cin, device=dev)
    dyg = nhwc(dy).to(dev)
    assert lib.cad_op_conv3x3_dgrad(_p(dyg), cout, _p(wg), cin, _p(dx), cin, B, H, W, _s()) == 0
    torch.cuda.synchronize()
    assert max_rel_err(nchw(dx.cpu()), xd.grad) < TOL
    # wgrad
    dw = torch.zeros(cout, 3, 3, cin, device=dev)
    assert lib.cad_op_conv3x3_wgrad(_p(dyg), cout, _p(xg), cin, 0, cin, _p(dw), B, H, W, _s()) == 0
    torch.cuda.synchronize()
    assert max_rel_err(dw.cpu().permute(0, 3, 1, 2), wd.grad) < TOL


WIN_SHAPES = [  # B, H, W, cin, cout: the window-tiled S3 forward/dgrad (gemm_win.hpp) block shapes
    (2, 6, 64, 64, 128),    # R x CW = 2 x 64, three block rows
    (1, 9, 32, 32, 128),    # 4 x 32, last block row partial (rows past H)
    (2, 5, 48, 16, 128),    # 8 x 16 (48 = 3 x 16), 16 input channels (one channel block)
    (1, 4, 128, 64, 64),    # N <= 64: 256 x 64 tile, 2 x 128
    (2, 7, 64, 128, 64),    # N <= 64: 4 x 64, partial block row; dgrad N = 128: 2 x 64
    (1, 13, 40, 256, 256),  # 16 x 8, H = 13 < R
    (3, 5, 16, 64, 192),    # wgrad window: 16-pixel stages = whole rows, 3 images (halo rows at image edges)
]


@pytest.mark.parametrize("B,H,W,cin,cout", WIN_SHAPES)
def test_conv3x3_window_kernel(cad, dev, B, H, W, cin, cout):
    """S3 engine, window-tiled forward and dgrad (input read through a strided, channel-offset view as
    in the decoder concat buffer; output likewise) against fp64."""
    lib = cad.load_library()
    prev = lib.cad_get_gemm_engine()
    assert lib.cad_set_gemm_engine(1) == 0
    try:
        g = torch.Generator().manual_seed(H * W + cin + cout)
        x = torch.randn(B, cin, H, W, generator=g)
        w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
        dy = torch.randn(B, cout, H, W, generator=g)
        xd, wd = x.double().requires_grad_(), w.double()
        y_ref = F.conv2d(xd, wd, None, 1, 1)
        y_ref.backward(dy.double())
        ldx = cin + 12
        xbuf = torch.zeros(B, H, W, ldx)
        xbuf[..., 8:8 + cin] = nhwc(x)
        xg, wg = xbuf.to(dev), w.permute(0, 2, 3, 1).contiguous().to(dev)
        ld = cout + 8
        ybuf = torch.full((B, H, W, ld), 7.0, device=dev)
        assert lib.cad_op_conv3x3_fwd(_p(xg), ldx, 8, cin, _p(wg), cout, _p(ybuf), ld, 4, B, H, W, _s()) == 0
        torch.cuda.synchronize()
        assert max_rel_err(nchw(ybuf[..., 4:4 + cout].cpu()), y_ref.detach()) < TOL
        assert (ybuf[..., :4] == 7).all() and (ybuf[..., 4 + cout:] == 7).all()
        dx = torch.zeros(B, H, W, cin, device=dev)
        assert lib.cad_op_conv3x3_dgrad(_p(nhwc(dy).to(dev)), cout, _p(wg), cin, _p(dx), cin, B, H, W, _s()) == 0
        torch.cuda.synchronize()
        assert max_rel_err(nchw(dx.cpu()), xd.grad) < TOL
        # weight gradient: window-tiled when cout, cin % 64 == 0 and W % 16 == 0 (x read through the view)
        wdd = w.double().requires_grad_()
        F.conv2d(x.double(), wdd, None, 1, 1).backward(dy.double())
        dw = torch.zeros(cout, 3, 3, cin, device=dev)
        assert lib.cad_op_conv3x3_wgrad(_p(nhwc(dy).to(dev)), cout, _p(xg), ldx, 8, cin, _p(dw), B, H, W, _s()) == 0
        torch.cuda.synchronize()
        assert max_rel_err(dw.cpu().permute(0, 3, 1, 2), wdd.grad) < TOL
    finally:
        lib.cad_set_gemm_engine(prev)


def test_conv3x3_wgrad_strided_input(cad, dev):
    """wgrad reading its input from the skip half of a concat-style buffer (ld = 2C, coff = C)."""
    lib = cad.load_library()
    B, H, W, cin, cout = 2, 12, 20, 32, 64
    g = torch.Generator().manual_seed(7)
    big = torch.randn(B, H, W, 2 * cin, generator=g)
    x = nchw(big[..., cin:].contiguous())
    dy = torch.randn(B, cout, H, W, generator=g)
    xd = x.double().requires_grad_()
    wd = torch.zeros(cout, cin, 3, 3, dtype=torch.float64, requires_grad=True)
    F.conv2d(xd, wd, None, 1, 1).backward(dy.double())
    dw = torch.zeros(cout, 3, 3, cin, device=dev)
    bg = big.to(dev)
    assert lib.cad_op_conv3x3_wgrad(_p(nhwc(dy).to(dev)), cout, _p(bg), 2 * cin, cin, cin, _p(dw), B, H, W, _s()) == 0
    torch.cuda.synchronize()
    assert max_rel_err(dw.cpu().permute(0, 3, 1, 2), wd.grad) < TOL


WGRAD_BF16_SHAPES = [  # B, H, W, cin, cout, xcoff: the bf16 engine's weight gradient on bf16 twins
    (2, 6, 64, 64, 128, 0),     # window kernel, 32-pixel stages, two per row
    (3, 5, 16, 64, 192, 8),     # 16-pixel stages (W % 32 != 0), halo rows at image edges, channel offset
    (1, 40, 80, 64, 64, 0),     # 16-pixel strips two rows per step: 100 row pairs over several K-splits
    (2, 7, 48, 128, 64, 64),    # ... odd H (the last pair's second row past the image), channel offset
    (1, 40, 96, 128, 64, 0),    # 3 stages per row, many K-splits over 120 stages
    (2, 9, 32, 256, 128, 64),   # skip half of a concat-style twin
    (2, 6, 20, 64, 64, 0),      # W % 16 != 0: the im2col GEMM
    (2, 5, 16, 32, 64, 0),      # cin % 64 != 0: the im2col GEMM
    (2, 40, 64, 8, 64, 0),      # cin = 8 (the NHWC8 image twin): the im2col GEMM, several K-splits
    (1, 30, 80, 8, 128, 8),     # ... at a channel offset, two output-channel blocks
]


@pytest.mark.parametrize("B,H,W,cin,cout,xcoff", WGRAD_BF16_SHAPES)
def test_conv3x3_wgrad_bf16_twins(cad, dev, B, H, W, cin, cout, xcoff):
    """cad_op_conv3x3_wgrad_bf16 (B1 window weight gradient, conv3x3_wgrad_win_ps_body) against the
    fp64 contraction of the same bf16 operands: the only admitted error is fp32 accumulation."""
    lib = cad.load_library()
    prev = lib.cad_get_gemm_engine()
    assert lib.cad_set_gemm_engine(2) == 0
    try:
        g = torch.Generator().manual_seed(B * H * W + cin + cout + xcoff)
        x = torch.randn(B, cin, H, W, generator=g).bfloat16()
        dy = torch.randn(B, cout, H, W, generator=g).bfloat16()
        wd = torch.zeros(cout, cin, 3, 3, dtype=torch.float64, requires_grad=True)
        F.conv2d(x.double(), wd, None, 1, 1).backward(dy.double())
        ldx = xcoff + cin + 8
        xbuf = torch.zeros(B, H, W, ldx, dtype=torch.bfloat16)
        xbuf[..., xcoff:xcoff + cin] = nhwc(x)
        xg, dyg = xbuf.to(dev), nhwc(dy).to(dev)
        dw = torch.full((cout, 3, 3, cin), 7.0, device=dev)
        assert lib.cad_op_conv3x3_wgrad_bf16(_p(dyg), cout, cout, _p(xg), ldx, xcoff, cin, _p(dw), B, H, W,
                                             _s()) == 0, lib.cad_last_error()
        torch.cuda.synchronize()
        assert max_rel_err(dw.cpu().permute(0, 3, 1, 2), wd.grad) < TOL
    finally:
        lib.cad_set_gemm_engine(prev)


@pytest.mark.parametrize("B,H,W", [(2, 6, 64), (1, 9, 32), (3, 7, 128), (2, 5, 36)])
def test_conv3x3_wgrad_bf16_pair32(cad, dev, B, H, W):
    """cout = cin = 32 on dense twins: the 64-channel window weight gradient on pixel pairs folded back
    (k_wgrad_pair_fold; W / 2 = 32, 16 (odd H: the last row pair's second row past the image), 64-wide
    stages; W / 2 = 18 takes the im2col kernel) against the fp64 contraction of the same bf16 operands."""
    lib = cad.load_library()
    prev = lib.cad_get_gemm_engine()
    assert lib.cad_set_gemm_engine(2) == 0
    try:
        g = torch.Generator().manual_seed(B * H * W + 32)
        x = torch.randn(B, 32, H, W, generator=g).bfloat16()
        dy = torch.randn(B, 32, H, W, generator=g).bfloat16()
        wd = torch.zeros(32, 32, 3, 3, dtype=torch.float64, requires_grad=True)
        F.conv2d(x.double(), wd, None, 1, 1).backward(dy.double())
        xg, dyg = nhwc(x).to(dev), nhwc(dy).to(dev)
        dw = torch.full((32, 3, 3, 32), 7.0, device=dev)
        assert lib.cad_op_conv3x3_wgrad_bf16(_p(dyg), 32, 32, _p(xg), 32, 0, 32, _p(dw), B, H, W, _s()) == 0, \
            lib.cad_last_error()
        torch.cuda.synchronize()
        assert max_rel_err(dw.cpu().permute(0, 3, 1, 2), wd.grad) < TOL
    finally:
        lib.cad_set_gemm_engine(prev)


def test_conv3x3_wgrad_bf16_needs_bf16_engine(cad, dev):
    lib = cad.load_library()
    prev = lib.cad_get_gemm_engine()
    assert lib.cad_set_gemm_engine(1) == 0
    try:
        t = torch.zeros(64, dtype=torch.bfloat16, device=dev)
        dw = torch.zeros(64, device=dev)
        assert lib.cad_op_conv3x3_wgrad_bf16(_p(t), 64, 64, _p(t), 64, 0, 64, _p(dw), 1, 1, 1, _s()) != 0
        assert b"bf16 engine" in lib.cad_last_error()
    finally:
        lib.cad_set_gemm_engine(prev)


CONVT_SHAPES = [(2, 8, 12, 128, 64), (1, 4, 5, 1024, 512), (3, 6, 6, 32, 16), (2, 3, 4, 8, 4),
                # W % 32 == 0: the pixel-shuffle epilogue's one-run-per-block store; M = 96 leaves a
                # partial 128-row tile
                (2, 5, 32, 64, 32), (1, 3, 32, 128, 64), (1, 2, 64, 256, 128)]


@pytest.mark.parametrize("B,H,W,cin,cout", CONVT_SHAPES)
def test_convT(cad, dev, engine, B, H, W, cin, cout):
    lib = cad.load_library()
    g = torch.Generator().manual_seed(cin * 7 + cout)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cin, cout, 2, 2, generator=g) / cin ** 0.5
    b = torch.randn(cout, generator=g)
    dy = torch.randn(B, cout, 2 * H, 2 * W, generator=g)
    xd, wdd, bd = q(x, engine).double().requires_grad_(), q(w, engine).double().requires_grad_(), b.double().requires_grad_()
    y_ref = F.conv_transpose2d(xd, wdd, bd, stride=2)
    y_ref.backward(q(dy, engine).double())
    wg = w.permute(0, 2, 3, 1).contiguous().to(dev)   # [ci][dy][dx][co]
    # forward into the "up" half of a concat buffer
    ybuf = torch.zeros(B, 2 * H, 2 * W, 2 * cout, device=dev)
    xg = nhwc(x).to(dev)
    assert lib.cad_op_convT_fwd(_p(xg), cin, _p(wg), _p(b.to(dev)), cout, _p(ybuf), 2 * cout, cout, B, H, W, _s()) == 0
    torch.cuda.synchronize()
    assert max_rel_err(nchw(ybuf[..., cout:].cpu()), y_ref.detach()) < TOL
    # dgrad from the up half of a concat-gradient buffer
    gbuf = torch.zeros(B, 2 * H, 2 * W, 2 * cout)
    gbuf[..., cout:] = nhwc(dy)
    gg = gbuf.to(dev)
    dx = torch.zeros(B, H, W, cin, device=dev)
    assert lib.cad_op_convT_dgrad(_p(gg), 2 * cout, cout, cout, _p(wg), cin, _p(dx), B, H, W, _s()) == 0
    torch.cuda.synchronize()
    assert max_rel_err(nchw(dx.cpu()), xd.grad) < TOL
    dw = torch.zeros(cin, 2, 2, cout, device=dev)
    assert lib.cad_op_convT_wgrad(_p(xg), cin, _p(gg), 2 * cout, cout, cout, _p(dw), B, H, W, _s()) == 0
    torch.cuda.synchronize()
    assert max_rel_err(dw.cpu().permute(0, 3, 1, 2), wdd.grad) < TOL


CONVT_BF16_SHAPES = [(2, 8, 12, 128, 64), (1, 3, 32, 128, 64), (2, 5, 64, 64, 32), (1, 4, 40, 256, 128),
                     (1, 2, 160, 128, 64)]


@pytest.mark.parametrize("B,H,W,cin,cout", CONVT_BF16_SHAPES)
def test_convT_fwd_bf16(cad, dev, B, H, W, cin, cout):
    """bf16 engine ConvTranspose forward (cad_op_convT_fwd_bf16: bf16 twin in, bf16 up half of a concat
    twin out) against the fp64 contraction of the bf16-rounded operands plus bias, rounded to bf16: within
    one bf16 spacing (floored at that of 2^-10 of the largest output), under 1e-2 of the outputs differing;
    the other half of the concat rows untouched."""
    lib = cad.load_library()
    prev = lib.cad_get_gemm_engine()
    assert lib.cad_set_gemm_engine(2) == 0
    try:
        g = torch.Generator().manual_seed(5 * B + H + W + cin + cout)
        x = torch.randn(B, cin, H, W, generator=g).bfloat16()
        w = torch.randn(cin, cout, 2, 2, generator=g) / cin ** 0.5
        b = torch.randn(cout, generator=g)
        y_ref = F.conv_transpose2d(x.double(), w.bfloat16().double(), b.double(), stride=2)
        xg, wg = nhwc(x).to(dev), w.permute(0, 2, 3, 1).contiguous().to(dev)
        ybuf = torch.full((B, 2 * H, 2 * W, 2 * cout), 7.0, dtype=torch.bfloat16, device=dev)
        assert lib.cad_op_convT_fwd_bf16(_p(xg), cin, 0, cin, _p(wg), _p(b.to(dev)), cout, _p(ybuf), 2 * cout, cout,
                                         B, H, W, _s()) == 0, lib.cad_last_error()
        torch.cuda.synchronize()
        got = ybuf[..., cout:].cpu().float()
        assert (ybuf[..., :cout].cpu().float() == 7.0).all()
        want = nhwc(y_ref).bfloat16().float()
        diff = (got - want).abs()
        big = torch.maximum(got.abs(), want.abs()).clamp_min(2.0 ** -10 * want.abs().max().item())
        ulp = torch.exp2(torch.floor(torch.log2(big)) - 7)
        assert (diff <= ulp).all() and (diff > 0).float().mean().item() < 1e-2, (diff / ulp).max().item()
    finally:
        lib.cad_set_gemm_engine(prev)


def test_maxpool(cad, dev):
    lib = cad.load_library()
    B, H, W, Cc = 2, 10, 14, 16
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, Cc, H, W, generator=g)
    x[0, 0, 0, :2] = 5.0   # tie: first in scan order must win
    ref, ridx = F.max_pool2d(x, 2, return_indices=True)
    buf = torch.zeros(B, H, W, 2 * Cc)
    buf[..., :Cc] = nhwc(x)
    bg = buf.to(dev)
    out = torch.zeros(B, H // 2, W // 2, Cc, device=dev)
    idx = torch.zeros(B, H // 2, W // 2, Cc, dtype=torch.uint8, device=dev)
    assert lib.cad_op_maxpool_fwd(_p(bg), 2 * Cc, Cc, B, H, W, _p(out), _p(idx), _s()) == 0
    torch.cuda.synchronize()
    assert torch.equal(nchw(out.cpu()), ref)
    # argmax code k = 2*dy + dx must point at the same element as torch's flat index
    k = nchw(idx.cpu()).long()
    yo = torch.arange(H // 2).view(1, 1, -1, 1)
    xo = torch.arange(W // 2).view(1, 1, 1, -1)
    flat = (2 * yo + k // 2) * W + 2 * xo + k % 2
    assert torch.equal(flat, ridx)


def test_ray_directions(cad, dev, oracle):
    B, H, W = 3, 24, 32
    _, _, K = oracle.synth_batch(B, H, W)
    rays = cad.ray_directions(torch.from_numpy(K).to(dev), H, W).cpu()
    Kt = torch.from_numpy(K).double()
    u = torch.arange(W, dtype=torch.float64).view(1, 1, W)
    v = torch.arange(H, dtype=torch.float64).view(1, H, 1)
    x = (u - Kt[:, 0, 2].view(B, 1, 1)) / Kt[:, 0, 0].view(B, 1, 1)
    y = (v - Kt[:, 1, 2].view(B, 1, 1)) / Kt[:, 1, 1].view(B, 1, 1)
    n = torch.sqrt(x * x + y * y + 1)
    ref = torch.stack([x / n, y / n, (1 / n).expand(B, H, W)], 1)
    assert (rays.double() - ref).abs().max().item() < 1e-6
    assert torch.allclose(rays.double().norm(dim=1), torch.ones(B, H, W, dtype=torch.float64), atol=1e-6)


@pytest.mark.parametrize("cin,cout,H,W", [(64, 64, 48, 64), (512, 512, 12, 16), (1024, 512, 8, 10)])
def test_s3_engine_accuracy_matches_fp32(cad, dev, cin, cout, H, W):
    """S3 (bf16 split) vs exact-fp32 MFMA, both against fp64, at the U-Net's K = 9*Cin: the S3
    error must stay within the fp32 engine's own (fp32 accumulation) error band."""
    lib = cad.load_library()
    prev = lib.cad_get_gemm_engine()
    B = 2
    g = torch.Generator().manual_seed(cin + H)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    ref = F.conv2d(x.double(), w.double(), None, 1, 1)
    xg, wg = nhwc(x).to(dev), w.permute(0, 2, 3, 1).contiguous().to(dev)
    errs = {}
    for eng in (0, 1):
        assert lib.cad_set_gemm_engine(eng) == 0
        y = torch.zeros(B, H, W, cout, device=dev)
        assert lib.cad_op_conv3x3_fwd(_p(xg), cin, 0, cin, _p(wg), cout, _p(y), cout, 0, B, H, W, _s()) == 0
        torch.cuda.synchronize()
        errs[eng] = max_rel_err(nchw(y.cpu()), ref)
    lib.cad_set_gemm_engine(prev)
    assert errs[1] < max(2.0 * errs[0], 2e-6), errs


def _profile(lib):
    import json
    n = lib.cad_profile_report(None, 0)
    buf = C.create_string_buffer(n)
    lib.cad_profile_report(buf, n)
    return json.loads(buf.value.decode())


# (engine, B, H, W): K = B*H*W pixels large enough for >= 48 split-K slabs of the 64 x 576 L0-type
# weight gradient, so finish_slabs takes its two-level reduction (conv_kernels.hip): 24-slab groups,
# then the group heads, then the remainder slabs
SLAB2 = [("s3", 1, 96, 256, 48, 0), ("s3", 1, 100, 256, 50, 2), ("f32", 1, 100, 256, 50, 2),
         ("bf16", 2, 96, 256, 48, 0)]


@pytest.mark.parametrize("eng,B,H,W,splits,rem", SLAB2)
def test_wgrad_two_level_slab_reduction(cad, dev, eng, B, H, W, splits, rem):
    """The many-slab weight-gradient path that only the 480x640 L0 layers take in the U-Net: both
    remainder branches (rem == 0: 2 reduction launches, the level-2 total written straight to dw;
    rem > 0: 3) against fp64, and the launch profile proves which plan ran (every k_slab_reduce launch
    is recorded)."""
    lib = cad.load_library()
    prev = lib.cad_get_gemm_engine()
    assert lib.cad_set_gemm_engine(ENGINES[eng]) == 0
    cin = cout = 64
    g = torch.Generator().manual_seed(H * 7 + B)
    x = torch.randn(B, cin, H, W, generator=g)
    dy = torch.randn(B, cout, H, W, generator=g) / (H * W) ** 0.5
    xd = q(x, eng).double()
    wd = torch.zeros(cout, cin, 3, 3, dtype=torch.float64, requires_grad=True)
    F.conv2d(xd, wd, None, 1, 1).backward(q(dy, eng).double())
    dw = torch.zeros(cout, 3, 3, cin, device=dev)
    xg, dyg = nhwc(x).to(dev), nhwc(dy).to(dev)
    torch.cuda.synchronize()
    lib.cad_profile_reset()
    lib.cad_profile_enable(1)
    try:
        assert lib.cad_op_conv3x3_wgrad(_p(dyg), cout, _p(xg), cin, 0, cin, _p(dw), B, H, W, _s()) == 0
        torch.cuda.synchronize()
        prof = _profile(lib)
    finally:
        lib.cad_profile_enable(0)
        lib.cad_set_gemm_engine(prev)
    reduce_launches = sum(r["launches"] for r in prof if "k_slab_reduce" in r["name"])
    assert reduce_launches == (2 if rem == 0 else 3), prof
    assert max_rel_err(dw.cpu().permute(0, 3, 1, 2), wd.grad) < TOL


B1_WIN_SHAPES = [  # B, H, W, cin, cout: the bf16 engine's window forward / dgrad (k_conv3x3_win_bf16p4) tiles
    (1, 6, 128, 64, 64),    # N == 64: 512 x 64 tile, CW 128; dgrad N = 64 likewise
    (2, 9, 64, 32, 128),    # 256 x 128, CW 64, partial block row; dgrad N = 32 (im2col pre-split)
    (1, 5, 32, 128, 128),   # CW 32
    (2, 7, 16, 64, 256),    # CW 16; dgrad N = 64 with W 16 (512 x 64 needs W % 64: im2col)
    (1, 13, 40, 256, 256),  # CW 8 (40 = 5 x 8), H = 13 < R = 32
    (1, 5, 128, 96, 96),    # f = 96 level 0: 256 x 96 tiles (k_conv3x3_win_bf16p3), CW 128, forward and dgrad
    (2, 6, 64, 192, 96),    # dec4.conv1 at f = 96: forward N = 96; dgrad N = 192 = two 96-column tiles
    (1, 3, 32, 96, 192),    # level 1 at f = 96: N = 192, CW 32; dgrad N = 96
]


@pytest.mark.parametrize("B,H,W,cin,cout", B1_WIN_SHAPES)
def test_conv3x3_bf16_window_kernels(cad, dev, B, H, W, cin, cout):
    """bf16 engine (cad_op_conv3x3_fwd_bf16 / _dgrad_bf16: the pre-split twins the step stores) against the
    fp64 contraction of the bf16-rounded operands: fp32 outputs within TOL; bf16 outputs the fp64 value
    rounded to bf16 (an fp32-accumulated sum next to a rounding boundary may round the other way: at
    most one bf16 spacing — floored at that of 2^-10 of the largest output — on under 1e-2 of the
    outputs); the BN-statistics epilogue produces the same outputs."""
    lib = cad.load_library()
    prev = lib.cad_get_gemm_engine()
    assert lib.cad_set_gemm_engine(2) == 0
    try:
        g = torch.Generator().manual_seed(7 * B + H + cin + cout)
        x = torch.randn(B, cin, H, W, generator=g).bfloat16()
        w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
        dz = torch.randn(B, cout, H, W, generator=g).bfloat16()
        xd, wd, dzd = x.double().requires_grad_(), w.bfloat16().double().requires_grad_(), dz.double()
        y_ref = F.conv2d(xd, wd, None, 1, 1)
        y_ref.backward(dzd)
        xg, wg, dzg = nhwc(x).to(dev), w.permute(0, 2, 3, 1).contiguous().to(dev), nhwc(dz).to(dev)
        for stats in (0, 1):
            y = torch.zeros(B, H, W, cout, device=dev)
            assert lib.cad_op_conv3x3_fwd_bf16(_p(xg), cin, 0, cin, _p(wg), cout, _p(y), cout, 0, 0, stats, B, H, W,
                                               _s()) == 0, lib.cad_last_error()
            torch.cuda.synchronize()
            assert max_rel_err(nchw(y.cpu()), y_ref.detach()) < TOL, stats
        yb = torch.zeros(B, H, W, cout, dtype=torch.bfloat16, device=dev)
        assert lib.cad_op_conv3x3_fwd_bf16(_p(xg), cin, 0, cin, _p(wg), cout, _p(yb), cout, 0, 1, 1, B, H, W, _s()) == 0
        torch.cuda.synchronize()
        want = nhwc(y_ref.detach()).bfloat16().float()
        got = yb.cpu().float()
        diff = (got - want).abs()
        # one bf16 spacing of the larger of the two, floored at the spacing of 2^-10 of the layer's largest
        # value (an output whose terms cancel to ~0 carries fp32 accumulation error far above its own ulp)
        big = torch.maximum(got.abs(), want.abs()).clamp_min(2.0 ** -10 * want.abs().max().item())
        ulp = torch.exp2(torch.floor(torch.log2(big)) - 7)
        assert (diff <= ulp).all() and (diff > 0).float().mean().item() < 1e-2, (diff / ulp).max().item()
        dx = torch.zeros(B, H, W, cin, device=dev)
        assert lib.cad_op_conv3x3_dgrad_bf16(_p(dzg), cout, cout, _p(wg), cin, _p(dx), cin, 0, B, H, W, _s()) == 0, \
            lib.cad_last_error()
        torch.cuda.synchronize()
        assert max_rel_err(nchw(dx.cpu()), xd.grad) < TOL
    finally:
        lib.cad_set_gemm_engine(prev)


def test_alias_guard_refuses_overlapping_launch(cad, dev):
    """The launch-level aliasing guard (cad.h cad_set_alias_check; on for every GPU test through
    tests/conftest.py): a bf16 window dgrad asked to write its input gradient into the buffer it reads
    as dZ — round 5's config-5 race in miniature — is refused with CAD_ERR_INVALID naming both operands,
    and nothing is launched; the same call on separate buffers runs."""
    lib = cad.load_library()
    prev_engine = lib.cad_get_gemm_engine()
    prev = lib.cad_set_alias_check(1)
    assert lib.cad_set_gemm_engine(2) == 0
    try:
        B, H, W, c = 2, 16, 64, 64
        dz = torch.randn(B, H, W, c, device=dev).bfloat16()
        w = torch.randn(c, c, 3, 3, device=dev) * 0.05
        st = lib.cad_op_conv3x3_dgrad_bf16(_p(dz), c, c, _p(w), c, _p(dz), c, 1, B, H, W, _s())
        msg = lib.cad_last_error().decode()
        assert st == 1, (st, msg)
        assert "alias" in msg and "dx" in msg and "dz" in msg, msg
        dx = torch.empty(B, H, W, c, device=dev).bfloat16()
        assert lib.cad_op_conv3x3_dgrad_bf16(_p(dz), c, c, _p(w), c, _p(dx), c, 1, B, H, W, _s()) == 0, \
            lib.cad_last_error()
        torch.cuda.synchronize()
    finally:
        lib.cad_set_gemm_engine(prev_engine)
        lib.cad_set_alias_check(prev)
