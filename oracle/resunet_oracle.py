"""Test infrastructure only (tests/, bench.py's cpu_baseline leg): a torch CPU restatement of the
config-5 network — ResNet-50 encoder + U-Net decoder (resunet.cpp) — that the HIP path
is checked against.

PARITY UNPINNED: the reference repository has no such model (BASELINE.json configs[4] names it,
SURVEY.md §8(f) rank 4), so there is nothing of the reference to pin this restatement to.  What it
pins instead: the module semantics are torch's own (F.conv2d, F.batch_norm, F.max_pool2d,
F.conv_transpose2d — the same functions torchvision's ResNet-50 and the reference's U-Net decoder
blocks are made of, baseline_unet.h:83-102), parameter names and shapes are torchvision's, and the
loss / clip / Adam are the U-Net oracle's (cad_oracle.py, pinned to the reference's fixtures).

operands="bf16" rounds every contraction operand to bf16 (forward x and w, dgrad dy, wgrad dy) and the
stored pre-BN conv outputs, as the GPU path does (cad_oracle._GEMM); "mx8" is the fp8 network
(cad_resunet_set_fp8): the eligible forward contractions on MXFP8 E4M3 operands (x8_eligible,
mx8_quantize), everything else as "bf16"; "exact" is plain fp32 (or fp64 with dtype=float64).
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn.functional as F

from . import cad_oracle as O

WIDTHS, NBLOCKS = (64, 128, 256, 512), (3, 4, 6, 3)
DEC = [(4, 2048, 512, 1024), (3, 512, 256, 512), (2, 256, 128, 256), (1, 128, 64, 64), (0, 64, 32, 0)]   # (l, cin_up, C, skipC)


def param_spec():
    """(name, shape) in the C++ registration order (cad_resunet_tensor_info)."""
    spec = [("encoder.conv1.weight", (64, 3, 7, 7)), ("encoder.bn1.weight", (64,)), ("encoder.bn1.bias", (64,))]
    cin = 64
    for L, (w, n) in enumerate(zip(WIDTHS, NBLOCKS)):
        for i in range(n):
            pre = f"encoder.layer{L + 1}.{i}."
            spec += [(pre + "conv1.weight", (w, cin, 1, 1)), (pre + "bn1.weight", (w,)), (pre + "bn1.bias", (w,)),
                     (pre + "conv2.weight", (w, w, 3, 3)), (pre + "bn2.weight", (w,)), (pre + "bn2.bias", (w,)),
                     (pre + "conv3.weight", (4 * w, w, 1, 1)), (pre + "bn3.weight", (4 * w,)),
                     (pre + "bn3.bias", (4 * w,))]
            if i == 0:
                spec += [(pre + "downsample.0.weight", (4 * w, cin, 1, 1)), (pre + "downsample.1.weight", (4 * w,)),
                         (pre + "downsample.1.bias", (4 * w,))]
            cin = 4 * w
    for l, cu, C, sk in DEC:
        pre = f"dec{l}."
        spec += [(pre + "up.weight", (cu, C, 2, 2)), (pre + "up.bias", (C,)),
                 (pre + "conv.conv1.weight", (C, sk + C, 3, 3)), (pre + "conv.bn1.weight", (C,)),
                 (pre + "conv.bn1.bias", (C,)), (pre + "conv.conv2.weight", (C, C, 3, 3)),
                 (pre + "conv.bn2.weight", (C,)), (pre + "conv.bn2.bias", (C,))]
    spec += [("out_conv.weight", (1, 32, 1, 1)), ("out_conv.bias", (1,))]
    return spec


def buffer_spec():
    out = []
    for n, s in param_spec():
        if n.endswith(".weight") and len(s) == 1:
            pre = n[: -len("weight")]
            out += [(pre + "running_mean", s), (pre + "running_var", s)]
    return out


def init(seed=0):
    """Random parameters (conv / ConvT U(+-1/sqrt(fan_in)), BN gamma U(0.5, 1.5), beta U(-0.2, 0.2)) and
    the default buffers — a generic point, not the GPU default init."""
    g = torch.Generator().manual_seed(seed)
    p = OrderedDict()
    for n, s in param_spec():
        if len(s) == 1 and (".bn" in n or "downsample.1" in n or "encoder.bn1" in n):
            p[n] = (torch.rand(s, generator=g) + 0.5) if n.endswith("weight") else (torch.rand(s, generator=g) - 0.5) * 0.4
        else:
            if n.endswith("up.weight"):
                fan = s[1] * 4
            elif n.endswith("up.bias"):
                fan = 4 * s[0]
            elif n.startswith("out_conv"):
                fan = 32
            else:
                fan = s[1] * s[2] * s[3]
            p[n] = (torch.rand(s, generator=g) * 2 - 1) / fan ** 0.5
    bufs = OrderedDict((n, torch.zeros(s) if "mean" in n else torch.ones(s)) for n, s in buffer_spec())
    return p, bufs


# ---- MX-fp8 (OCP MXFP8 E4M3, gemm_mx8.hpp): the config-5 network's forward conv-GEMM operands ----
def mx8_quantize(x):
    """Quantise along the last dim in blocks of 32 (gemm_mx8.hpp mx8_quant_block): returns (e4m3 element
    codes as uint8, e8m0 scale codes as uint8, the dequantised fp32 values).  shared exponent =
    floor(log2 amax) (fp32 exponent field; 0 / subnormal blocks: -127) - 8, clamped to [-127, 127];
    element = e4m3 round-to-nearest-even of clamp(v * 2^-shared, +-448)."""
    v = x.float().reshape(*x.shape[:-1], x.shape[-1] // 32, 32)
    amax = v.abs().amax(-1)
    e = ((amax.view(torch.int32) >> 23) & 0xFF) - 127
    sh = (e - 8).clamp(-127, 127)
    one = torch.ones_like(amax)
    inv = torch.ldexp(one, (-sh.clamp(max=126)).to(torch.int32))
    q = (v * inv.unsqueeze(-1)).clamp(-448.0, 448.0).to(torch.float8_e4m3fn)
    deq = (q.float().double() * torch.ldexp(one.double(), sh.to(torch.int32)).unsqueeze(-1)).float()
    return q.view(torch.uint8).reshape(x.shape), (sh + 127).to(torch.uint8), deq.reshape(x.shape)


def mx8_dequant(q, s):
    """(element codes [.., K] uint8, scale codes [.., K/32] uint8) -> fp64 values"""
    vals = q.view(torch.float8_e4m3fn).double().reshape(*q.shape[:-1], q.shape[-1] // 32, 32)
    sc = torch.ldexp(torch.ones(s.shape, dtype=torch.float64, device=s.device), s.to(torch.int32) - 127)
    return (vals * sc.unsqueeze(-1)).reshape(q.shape)


def x8_eligible(k, stride, cin, cout, width):
    """resunet.cpp x8_eligible: which forward contractions run on MX-fp8 operands (cin = the stored
    input channels; width = the input width).  3x3 stride 1: the window kernel (mx8_kernels.hip
    pick_win_x8: cin % 64, cout 64 with a 128/64 block width dividing W, or cout % 128 with 64/32/16/8);
    other convolutions: the dense GEMM on K = k*k*cin (padded to 8) with K % 128 and cout % 64."""
    if k == 3 and stride == 1 and cin % 8 == 0:
        if cin % 64 or cout % 64:
            return False
        if cout == 64:
            return width % 128 == 0 or width % 64 == 0
        return cout % 128 == 0 and any(width % c == 0 for c in (64, 32, 16, 8))
    kp = (k * k * cin + 7) // 8 * 8
    return kp % 128 == 0 and cout % 64 == 0


def _mx8_channels(t):
    """MX-quantise-dequantise along dim 1 (channels; per (kh, kw) tap for a weight tensor)"""
    return mx8_quantize(t.movedim(1, -1).contiguous())[2].to(t.dtype).movedim(-1, 1)


class _X8Conv(torch.autograd.Function):
    """The fp8 network's eligible convolutions (cad_resunet_set_fp8): forward on MX-fp8 operands — the
    bf16 activation twin and the fp32 weights, each quantised along channels — and the backward on
    bf16 operands (dgrad: bf16 w, wgrad: the bf16 twin x; the incoming dy is rounded by the caller)."""

    @staticmethod
    def forward(ctx, x, w, stride, pad):
        xb = x.to(torch.bfloat16).to(x.dtype)
        ctx.save_for_backward(xb, w.to(torch.bfloat16).to(w.dtype))
        ctx.stride, ctx.pad = stride, pad
        return F.conv2d(_mx8_channels(xb), _mx8_channels(w), None, stride, pad)

    @staticmethod
    def backward(ctx, g):
        xb, wb = ctx.saved_tensors
        gx = torch.nn.grad.conv2d_input(xb.shape, wb, g, ctx.stride, ctx.pad)
        gw = torch.nn.grad.conv2d_weight(xb, wb.shape, g, ctx.stride, ctx.pad)
        return gx, gw, None, None


def _rnd(x):
    return O._RoundOperand.apply(x) if O._GEMM["operands"] in ("bf16", "mx8") else x


def _conv(x, w, stride, pad, name=None):
    mode = O._GEMM["operands"]
    if mode == "mx8" and x8_eligible(w.shape[2], stride, x.shape[1], w.shape[0], x.shape[3]):
        y = _X8Conv.apply(x, w, stride, pad)
    else:
        y = F.conv2d(_rnd(x), _rnd(w), None, stride, pad)
    # bf16 / mx8: the dy operand of dgrad / wgrad rounded, and the pre-BN output stored as bf16
    y = O._RoundOperand.apply(O._RoundGradOperand.apply(y)) if mode in ("bf16", "mx8") else y
    # test hook (cad_oracle.Y_FORCE): the full-size test imposes the GPU's stored pre-BN outputs, keyed
    # by the convolution's parameter name without ".weight"; Y_OWN records this restatement's own
    forced = O.Y_FORCE.get(name) if name else None
    if forced is None:
        return y
    O.Y_OWN[name] = y.detach().clone()
    return _impose(y, forced)


# Test hooks of the full-size test, which imposes the GPU run's forward values so that every convolution
# of this restatement reads operands bit-identical to the GPU's (an fp32 ulp of a BN coefficient or of an
# accumulation order flips the bf16 rounding of ~1e-4 of an activation, and behind the MX-fp8 quantiser
# such a flip moves a product by 2^-4..2^-3 of itself: round 6 measured up to 481 bf16 ulps on 2-5% of a
# decoder convolution's outputs without these hooks).  The backward still runs through this
# restatement's own graph (straight-through, as cad_oracle.Y_FORCE).
#   TRACE      when a dict, records each block's own output ("encoder.stem", "encoder.layer<L>.<i>", "dec<l>")
#   OUT_FORCE  {block name: the GPU's fp32 block output (NCHW)} (cad_resunet_debug_buffer "out:<block>")
#   COEF_FORCE {BN prefix: (scale, shift)} of a BN-ReLU: z = fma(y, scale, shift) rounded once to fp32
#              (k_bn_relu_fwd), "scale:/shift:<bn>"
#   CAT_FORCE  {"dec<l>": the decoder's bf16 input [skip, up] (NCHW)} ("cat:dec<l>": the ConvT output
#              as the GPU stored it)
TRACE = None
OUT_FORCE = {}
COEF_FORCE = {}
CAT_FORCE = {}


def _impose(y, forced):
    # forced + (y - y) carries y's gradient and the forced value exactly (y + (forced - y) rounds twice)
    return y if forced is None else forced.to(y.device, y.dtype) + (y - y.detach())


def _trace(name, y):
    if TRACE is not None:   # this restatement's own value, before OUT_FORCE
        TRACE[name] = y.detach().clone()
    return _impose(y, OUT_FORCE.get(name))


def _relu(z, name):
    """ReLU with the test hook cad_oracle.RELU_FORCE (the GPU run's decisions, keyed by the BN prefix or
    "<block>.out" for a bottleneck's relu(bn3 + shortcut))."""
    m = O.RELU_FORCE.get(name)
    return F.relu(z) if m is None else z * m.to(z.device, z.dtype)


def _bn_relu(y, p, bufs, name, train):
    """BatchNorm2d + ReLU with the test hooks COEF_FORCE and cad_oracle.RELU_FORCE"""
    z = O._bn(y, p, bufs, name, train)
    cf = COEF_FORCE.get(name)
    if cf is not None:
        sc, sh = (t.to(y.device, torch.float64).view(1, -1, 1, 1) for t in cf)
        z = _impose(z, (y.detach().double() * sc + sh).to(y.dtype))
    return _relu(z, name)


def _rgrad(x):
    """bf16 / mx8: the input gradient of this convolution stored as bf16 (resunet.cpp unit_bwd dx_bf16:
    a bottleneck's conv3 and stride-1 conv2, a decoder's conv2 — read only by the BN backward below)"""
    return O._RoundGradOperand.apply(x) if O._GEMM["operands"] in ("bf16", "mx8") else x


def _bottleneck(x, p, bufs, pre, stride, down, train):
    t = _bn_relu(_conv(x, p[pre + "conv1.weight"], 1, 0, pre + "conv1"), p, bufs, pre + "bn1", train)
    t = _bn_relu(_conv(_rgrad(t) if stride == 1 else t, p[pre + "conv2.weight"], stride, 1, pre + "conv2"), p, bufs,
                 pre + "bn2", train)
    t = O._bn(_conv(_rgrad(t), p[pre + "conv3.weight"], 1, 0, pre + "conv3"), p, bufs, pre + "bn3", train)
    sc = (O._bn(_conv(x, p[pre + "downsample.0.weight"], stride, 0, pre + "downsample.0"), p, bufs,
                pre + "downsample.1", train) if down else x)
    return _trace(pre[:-1], _relu(t + sc, pre + "out"))


def forward(x, p, bufs, train=True, max_depth=10.0):
    x1 = _trace("encoder.stem", _bn_relu(_conv(x, p["encoder.conv1.weight"], 2, 3, "encoder.conv1"), p, bufs,
                                         "encoder.bn1", train))
    y = F.max_pool2d(x1, 3, 2, 1)
    feats = []
    for L, n in enumerate(NBLOCKS):
        for i in range(n):
            y = _bottleneck(y, p, bufs, f"encoder.layer{L + 1}.{i}.", 2 if (L > 0 and i == 0) else 1, i == 0, train)
        feats.append(y)
    skips = {4: feats[2], 3: feats[1], 2: feats[0], 1: x1}
    for l, cu, C, sk in DEC:
        pre = f"dec{l}."
        # (bias_bf16: the bias gradient sums the bf16 up-half gradient the ConvT GEMMs read, as resunet.cpp)
        up = O._convT2x2(y, p[pre + "up.weight"], p[pre + "up.bias"], bias_bf16=True)
        y = _impose(torch.cat([skips[l], up], 1) if sk else up, CAT_FORCE.get(f"dec{l}"))
        y = _bn_relu(_conv(y, p[pre + "conv.conv1.weight"], 1, 1, pre + "conv.conv1"), p, bufs, pre + "conv.bn1", train)
        y = _trace(f"dec{l}", _bn_relu(_conv(_rgrad(y), p[pre + "conv.conv2.weight"], 1, 1, pre + "conv.conv2"), p,
                                       bufs, pre + "conv.bn2", train))
    z = F.conv2d(y, p["out_conv.weight"], p["out_conv.bias"])
    return torch.sigmoid(z) * max_depth


class Trainer:
    """forward, CombinedDepthLoss, backward, clip_grad_norm_(1.0), Adam — the GPU train_step's sequence."""

    def __init__(self, params, buffers, weights=(1.0, 0.1, 0.001, 0.01), lr=1e-4, wd=1e-5, clip=1.0,
                 dtype=torch.float32, operands="bf16", device=None):
        # device: where ATen evaluates the restatement (host by default; the full-size test evaluates
        # its fp64 witness with ATen's GPU kernels)
        self.dtype, self.operands = dtype, operands
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.p = OrderedDict((k, v.clone().to(self.device, dtype)) for k, v in params.items())
        self.bufs = OrderedDict((k, v.clone().to(self.device, dtype)) for k, v in buffers.items())
        self.weights, self.clip = weights, clip
        self.opt = O.Adam(self.p, lr=lr, weight_decay=wd)

    def step(self, rgb, gt, K):
        rgb, gt, K = (t.to(self.device, self.dtype) for t in (rgb, gt, K))
        for v in self.p.values():
            v.requires_grad_(True)
            v.grad = None
        prev, O._GEMM["operands"] = O._GEMM["operands"], self.operands
        try:
            pred = forward(rgb, self.p, self.bufs, True)
            loss, comps = O.combined_loss(pred, gt, rgb, K, self.weights)
            loss.sum().backward()
        finally:
            O._GEMM["operands"] = prev
        grads = [v.grad.detach().clone() for v in self.p.values()]
        for v in self.p.values():
            v.requires_grad_(False)
        pre = [g.clone() for g in grads]
        norm = O.clip_grad_norm_(grads, self.clip)
        self.opt.step(grads)
        return dict(pred=pred.detach(), loss=float(loss), comps=comps, grads=pre, norm=norm)

    @torch.no_grad()
    def predict_eval(self, rgb):
        prev, O._GEMM["operands"] = O._GEMM["operands"], self.operands
        try:
            return forward(rgb.to(self.device, self.dtype), self.p, self.bufs, False)
        finally:
            O._GEMM["operands"] = prev
