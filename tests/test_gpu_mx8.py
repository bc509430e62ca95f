"""MX-fp8 operators (gemm_mx8.hpp / mx8_kernels.hip, the config-5 network's forward conv-GEMMs) through
the C ABI against the oracle's torch restatement (oracle/resunet_oracle.py mx8_quantize / mx8_dequant).

* quantiser: element and scale bytes bit-exact with torch's float8_e4m3fn cast of the same block
  arithmetic (fp32 and bf16 sources, zero / tiny / saturating / mixed-magnitude blocks, offsets);
* dense and window-conv GEMMs: against the fp64 contraction of the DEQUANTISED operands the GPU
  quantised (so the only admitted difference is accumulation: normalised max error <= 1e-4 — the
  block-scaled MFMA does not sum a 64-deep product block as an fp32 chain; measured 0.6e-5 .. 2.5e-5
  on MI355X at K = 128 .. 2048, where the bf16 MFMA engine stays below 2e-5),
  and the whole quantise -> GEMM chain against the fp64 result of the unquantised operands within the
  MXFP8 rounding (E4M3: 3 mantissa bits, 2^-4 relative per element; the MX shared exponent lets a
  block's top values saturate at 448, up to 2^-3): normalised max error < 0.1 (measured 0.05-0.057).
Parity unpinned in the SURVEY §8(c) sense: the reference has no fp8 path (BASELINE.json configs[4])."""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

from conftest import max_rel_err

pytestmark = pytest.mark.gpu
X8_TOL = 1e-4


def _p(t):
    return C.c_void_p(t.data_ptr())


def _s():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


@pytest.fixture(scope="module")
def R():
    from oracle import resunet_oracle
    return resunet_oracle


def quantize(lib, dev, src, C_, ld, coff=0, src_bf16=False, lds=None, scoff=0):
    """GPU quantiser: src [M][lds] (fp32 or bf16), channels [scoff, scoff + C_) -> (q [M][ld], s [M][ld/32])"""
    M = src.shape[0]
    q = torch.zeros((M, ld), dtype=torch.uint8, device=dev)
    s = torch.zeros((M, ld // 32), dtype=torch.uint8, device=dev)
    rc = lib.cad_op_mx8_quantize(_p(src), int(src_bf16), lds or src.shape[1], scoff, C_, M, _p(q), _p(s), ld, coff, _s())
    assert rc == 0, lib.cad_last_error()
    torch.cuda.synchronize()
    return q, s


def test_quantize_bit_exact(cad, dev, R):
    lib = cad.load_library()
    g = torch.Generator().manual_seed(3)
    M, Cc = 257, 320
    x = torch.randn(M, Cc, generator=g) * torch.exp2(torch.randint(-30, 30, (M, Cc // 32), generator=g).float()).repeat_interleave(32, 1)
    x[0, :32] = 0.0                                     # zero block
    x[1, :32] = 1e-41                                   # subnormal block
    x[2, :32] = torch.linspace(-511.0, 511.0, 32)       # saturates at +-448 after scaling
    x[3, 32:64] = torch.tensor([1.0] * 31 + [255.99])   # block max just below a binade
    x[4, 64:96] = torch.tensor([3.0 * 2 ** -9] * 32) * 2.0 ** -110   # deep shared exponent
    q, s = quantize(lib, dev, x.to(dev), Cc, 384, coff=64)
    rq, rs, _ = R.mx8_quantize(x)
    assert torch.equal(q[:, 64:64 + Cc].cpu(), rq), (q[:, 64:64 + Cc].cpu() != rq).nonzero()[:8]
    assert torch.equal(s[:, 2:2 + Cc // 32].cpu(), rs)
    # bf16 source rows with a channel offset
    xb = (torch.randn(100, 256, generator=g) * 3).bfloat16()
    q2, s2 = quantize(lib, dev, xb.to(dev), 128, 128, src_bf16=True, lds=256, scoff=64)
    rq2, rs2, _ = R.mx8_quantize(xb[:, 64:192].float())
    assert torch.equal(q2.cpu(), rq2) and torch.equal(s2.cpu(), rs2)


@pytest.mark.parametrize("M,K,N", [(1000, 256, 128), (4096, 1152, 256), (300, 128, 64), (2050, 2048, 512), (77, 512, 1024)])
def test_dense_x8(cad, dev, R, M, K, N):
    lib = cad.load_library()
    g = torch.Generator().manual_seed(M + K + N)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    ld = (K + 127) // 128 * 128
    xq, xs = quantize(lib, dev, x.to(dev), K, ld)
    wq, ws = quantize(lib, dev, w.to(dev), K, ld)
    y = torch.empty((M, N), device=dev)
    assert lib.cad_op_dense_x8(_p(xq), _p(xs), ld, K, _p(wq), _p(ws), ld, N, _p(y), M, _s()) == 0, lib.cad_last_error()
    torch.cuda.synchronize()
    xd = R.mx8_dequant(xq.cpu(), xs.cpu())[:, :K]
    wd = R.mx8_dequant(wq.cpu(), ws.cpu())[:, :K]
    ref = xd @ wd.T
    assert max_rel_err(y.cpu(), ref) < X8_TOL
    # the whole chain against the unquantised operands: MXFP8 rounding (~2^-4 per element, averaged down)
    exact = x.double() @ w.double().T
    assert max_rel_err(y.cpu(), exact) < 0.1


@pytest.mark.parametrize("B,H,W,cin,cout", [(2, 12, 16, 64, 128), (1, 10, 40, 128, 256), (2, 7, 64, 64, 64),
                                            (1, 9, 8, 256, 512), (2, 16, 32, 192, 128)])
def test_conv3x3_x8(cad, dev, R, B, H, W, cin, cout):
    lib = cad.load_library()
    g = torch.Generator().manual_seed(B * H * W + cin)
    x = torch.randn(B, H, W, cin, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (9 * cin) ** 0.5
    ldx = (cin + 127) // 128 * 128
    xq, xs = quantize(lib, dev, x.reshape(-1, cin).to(dev), cin, ldx)
    wk = w.permute(0, 2, 3, 1).reshape(cout, 9 * cin)   # (tap, ci) order
    ldw = (9 * cin + 127) // 128 * 128
    wq, ws = quantize(lib, dev, wk.contiguous().to(dev), 9 * cin, ldw)
    y = torch.empty((B * H * W, cout), device=dev)
    rc = lib.cad_op_conv3x3_x8(_p(xq), _p(xs), ldx, cin, _p(wq), _p(ws), ldw, cout, _p(y), B, H, W, _s())
    assert rc == 0, lib.cad_last_error()
    torch.cuda.synchronize()
    xd = R.mx8_dequant(xq.cpu(), xs.cpu())[:, :cin].reshape(B, H, W, cin).permute(0, 3, 1, 2)
    wd = R.mx8_dequant(wq.cpu(), ws.cpu())[:, :9 * cin].reshape(cout, 3, 3, cin).permute(0, 3, 1, 2)
    ref = F.conv2d(xd, wd, None, 1, 1).permute(0, 2, 3, 1).reshape(-1, cout)
    assert max_rel_err(y.cpu(), ref) < X8_TOL
    exact = F.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), None, 1, 1).permute(0, 2, 3, 1).reshape(-1, cout)
    assert max_rel_err(y.cpu(), exact) < 0.1


def test_x8_shape_errors(cad, dev):
    lib = cad.load_library()
    t = torch.zeros(4096, dtype=torch.uint8, device=dev)
    y = torch.zeros(1024, device=dev)
    assert lib.cad_op_dense_x8(_p(t), _p(t), 128, 96, _p(t), _p(t), 128, 64, _p(y), 4, _s()) != 0   # K % 128
    assert lib.cad_op_conv3x3_x8(_p(t), _p(t), 128, 32, _p(t), _p(t), 384, 64, _p(y), 1, 2, 8, _s()) != 0   # cin % 64
