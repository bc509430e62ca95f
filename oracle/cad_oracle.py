"""ORACLE / TEST INFRASTRUCTURE ONLY.

CPU restatement (PyTorch CPU, fp32, autograd) of the reference training step that the MI355X path
replaces.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the CHECKER: the product path (libcad_hip.so and its bindings) never calls it.

Every function cites the reference file:line it restates (paths relative to /root/reference):

  * BaselineUNetImpl            src/models/baseline_unet.h:14-208
  * FiLMLayerImpl               src/layers/film_layer.h:26-108
  * FiLMDoubleConv / FiLMEncoderBlock / FiLMDecoderBlock / IntrinsicsConditionedUNetImpl
                                src/models/intrinsics_unet.h:16-270
  * RayEnhancedConvImpl         src/models/geometry_aware_network.h:17-65
  * computeRayDirections (a18)  src/preprocessing/ray_direction_computer.cpp:17-62
  * ScaleInvariantLoss          src/loss/depth_loss.h:20-69
  * GradientMatchingLoss        src/loss/depth_loss.h:82-167
  * SmoothnessLoss              src/loss/depth_loss.h:178-238
  * ReprojectionLoss            src/loss/depth_loss.h:255-355
  * CombinedDepthLoss           src/loss/depth_loss.h:366-479
  * train step                  src/training/tensorboard_trainer_enhanced.h:287-304
  * clip_grad_norm_             torch/csrc/api/include/torch/nn/utils/clip_grad.h:22-85 (LibTorch)
  * Adam (coupled L2)           torch::optim::Adam, options built at enhanced.h:97-101
  * computeDepthMetrics (a20)   src/training/tensorboard_trainer_enhanced.h:400-439
  * SunRGBDLoader::getSample    src/data/sunrgbd_loader.cpp:105-169 (load :221-259, augment
                                :352-443, resize :445-489), decode excluded

Parity pin: tests/test_oracle_golden.py checks this restatement against fixtures produced by the
REFERENCE itself (oracle/ref_harness.cpp compiled in place against /root/reference/src by
oracle/Makefile, fixtures committed under tests/golden/ by oracle/gen_golden.py).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

EPS = 1e-6

# --------------------------------------------------------------------------------------------
# Synthetic SUN-RGB-D-shaped batches; byte-identical to ref_harness.cpp.
# --------------------------------------------------------------------------------------------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(seed: int, idx: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx.astype(np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def u01(seed: int, idx: np.ndarray) -> np.ndarray:
    u = (splitmix64(seed, idx) >> np.uint64(32)).astype(np.uint32)
    return (u >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def intrinsics_for(B: int, H: int, W: int) -> np.ndarray:
    """Per-sample K (B,3,3): NYU/kv1 and Xtion calibrations scaled like sunrgbd_loader.cpp:480-488."""
    K = np.zeros((B, 3, 3), np.float32)
    sx, sy = np.float32(W / 640.0), np.float32(H / 480.0)
    for b in range(B):
        if b % 2 == 0:
            fx, fy, cx, cy = 518.858, 519.470, 325.582, 253.736
        else:
            fx, fy, cx, cy = 570.342, 570.342, 320.0, 240.0
        K[b, 0, 0] = np.float32(fx) * sx
        K[b, 0, 2] = np.float32(cx) * sx
        K[b, 1, 1] = np.float32(fy) * sy
        K[b, 1, 2] = np.float32(cy) * sy
        K[b, 2, 2] = 1.0
    return K


def synth_batch(B: int, H: int, W: int, rgb_seed: int = 0xC0FFEE, hole_seed: int = 0xD3E7):
    """rgb (B,3,H,W) U[0,1); gt (B,1,H,W) smooth field with holes; K (B,3,3). numpy float32."""
    rgb = u01(rgb_seed, np.arange(B * 3 * H * W, dtype=np.uint64)).reshape(B, 3, H, W)
    b = np.arange(B, dtype=np.float64)[:, None, None]
    v = np.arange(H, dtype=np.float64)[None, :, None]
    u = np.arange(W, dtype=np.float64)[None, None, :]
    ph = 2.0 * math.pi * (u / W * 1.3 + v / H * 0.7 + 0.1 * b)
    d = np.clip(0.5 + 9.0 * (0.5 + 0.5 * np.sin(ph)), 0.5, 9.5)
    holes = u01(hole_seed, np.arange(B * H * W, dtype=np.uint64)).reshape(B, H, W) < np.float32(0.15)
    holes |= (np.arange(H)[None, :, None] < H // 16)
    gt = np.where(holes, 0.0, d).astype(np.float32).reshape(B, 1, H, W)
    return rgb, gt, intrinsics_for(B, H, W)


# --------------------------------------------------------------------------------------------
# Model: BaselineUNetImpl (baseline_unet.h:122-208) as named parameter/buffer dictionaries.
# --------------------------------------------------------------------------------------------
MODELS = ("baseline", "film", "rayfilm", "geo", "geolite")
GEO_LEVELS = {"geo": 6, "geolite": 5}   # GeometryAwareNetworkImpl / LightweightGeometryNetworkImpl
FILM_CAMERA_DIM, FILM_H1, FILM_HIDDEN = 4, 128, 256   # FiLMLayerImpl(4, C) defaults (film_layer.h:47-66)


def _film_spec(prefix, C):
    # FiLMLayerImpl ctor (film_layer.h:47-72): registration order fc1, fc2, fc_gamma, fc_beta, bn1, bn2
    return [(prefix + "fc1.weight", (FILM_H1, FILM_CAMERA_DIM)), (prefix + "fc1.bias", (FILM_H1,)),
            (prefix + "fc2.weight", (FILM_HIDDEN, FILM_H1)), (prefix + "fc2.bias", (FILM_HIDDEN,)),
            (prefix + "fc_gamma.weight", (C, FILM_HIDDEN)), (prefix + "fc_gamma.bias", (C,)),
            (prefix + "fc_beta.weight", (C, FILM_HIDDEN)), (prefix + "fc_beta.bias", (C,)),
            (prefix + "bn1.weight", (FILM_H1,)), (prefix + "bn1.bias", (FILM_H1,)),
            (prefix + "bn2.weight", (FILM_HIDDEN,)), (prefix + "bn2.bias", (FILM_HIDDEN,))]


def _double_conv_spec(prefix, cin, cout, film=False):
    # DoubleConvImpl ctor (baseline_unet.h:20-30): conv1 (no bias), bn1, conv2 (no bias), bn2;
    # FiLMDoubleConvImpl / RayEnhancedConvImpl (intrinsics_unet.h:23-36, geometry_aware_network.h:25-45)
    # register the same four modules, then `film`
    spec = [(prefix + "conv1.weight", (cout, cin, 3, 3)),
            (prefix + "bn1.weight", (cout,)), (prefix + "bn1.bias", (cout,)),
            (prefix + "conv2.weight", (cout, cout, 3, 3)),
            (prefix + "bn2.weight", (cout,)), (prefix + "bn2.bias", (cout,))]
    return spec + (_film_spec(prefix + "film.", cout) if film else [])


def _cbam_spec(prefix, C):
    # CBAMImpl(C) (spatial_attention.h:150-157): ChannelAttentionImpl fc1/fc2 (reduction 16, :38-50),
    # SpatialAttentionImpl conv 2 -> 1, 7x7, no bias (:93-99)
    cr = max(1, C // 16)
    return [(prefix + "channel_attention.fc1.weight", (cr, C)), (prefix + "channel_attention.fc1.bias", (cr,)),
            (prefix + "channel_attention.fc2.weight", (C, cr)), (prefix + "channel_attention.fc2.bias", (C,)),
            (prefix + "spatial_attention.conv.weight", (1, 2, 7, 7))]


def _pcl_spec(prefix, C, hidden=128):
    # PerspectiveCorrectionLayerImpl(C, 4, 128) (pcl_layer.h:45-63): loc_fc1, loc_fc2, fc_transform
    return [(prefix + "loc_fc1.weight", (hidden, C + 4)), (prefix + "loc_fc1.bias", (hidden,)),
            (prefix + "loc_fc2.weight", (hidden, hidden)), (prefix + "loc_fc2.bias", (hidden,)),
            (prefix + "fc_transform.weight", (6, hidden)), (prefix + "fc_transform.bias", (6,))]


def _geo_names(model):
    nl = GEO_LEVELS[model]
    enc = ["enc1"] + [f"enc{l + 1}" for l in range(1, nl - 1)] + ["bottleneck"]
    return nl, enc


def _geo_spec(f, in_ch, model, use_pcl=True, use_attention=True):
    # GeometryAwareNetworkImpl ctor (geometry_aware_network.h:241-278) / LightweightGeometryNetworkImpl
    # (:368-383): enc1 = RayEnhancedConv(in, f, 4, true); GeometryEncoderBlock = pool, conv, attention;
    # GeometryDecoderBlock = up, conv, pcl, attention (:74-170); out_conv
    nl, enc = _geo_names(model)
    spec = _double_conv_spec("enc1.", in_ch + 3, f, True)
    for l in range(1, nl):
        spec += _double_conv_spec(f"{enc[l]}.conv.", f << (l - 1), f << l, True)
        if use_attention:
            spec += _cbam_spec(f"{enc[l]}.attention.", f << l)
    for l in range(nl - 2, -1, -1):
        cin, cout = f << (l + 1), f << l
        pre = f"dec{l + 1}."
        spec += [(pre + "up.weight", (cin, cout, 2, 2)), (pre + "up.bias", (cout,))]
        spec += _double_conv_spec(pre + "conv.", cin, cout, True)
        if use_pcl:
            spec += _pcl_spec(pre + "pcl.", cout)
        if use_attention:
            spec += _cbam_spec(pre + "attention.", cout)
    return spec + [("out_conv.weight", (1, f, 1, 1)), ("out_conv.bias", (1,))]


def param_spec(f: int = 64, in_ch: int = 3, model: str = "baseline"):
    """named_parameters() order of BaselineUNetImpl(in_ch, f) (registration order, :144-166),
    IntrinsicsConditionedUNetImpl(in_ch, f, 4) (intrinsics_unet.h:168-195), or the config-3
    composite "rayfilm" (enc1 = RayEnhancedConv(in_ch, f, 4, use_rays) with in_ch + 3 inputs);
    "geo" / "geolite": GeometryAwareNetworkImpl / LightweightGeometryNetworkImpl."""
    assert model in MODELS, model
    if model in GEO_LEVELS:
        return _geo_spec(f, in_ch, model)
    film = model != "baseline"
    spec = _double_conv_spec("enc1.", in_ch + (3 if model == "rayfilm" else 0), f, film)
    for i, name in enumerate(["enc2", "enc3", "enc4", "bottleneck"]):
        spec += _double_conv_spec(f"{name}.conv.", f << i, f << (i + 1), film)
    for i, name in enumerate(["dec4", "dec3", "dec2", "dec1"]):
        cin = f << (4 - i)
        spec += [(f"{name}.up.weight", (cin, cin // 2, 2, 2)), (f"{name}.up.bias", (cin // 2,))]
        spec += _double_conv_spec(f"{name}.conv.", cin, cin // 2, film)
    spec += [("out_conv.weight", (1, f, 1, 1)), ("out_conv.bias", (1,))]
    return spec


def buffer_spec(f: int = 64, in_ch: int = 3, model: str = "baseline"):
    """Float BatchNorm buffers (running_mean/var) in named_buffers() order."""
    out = []
    for name, shape in param_spec(f, in_ch, model):
        if name.endswith(".bias") and ".bn" in name:
            base = name[: -len(".bias")]
            out += [(base + ".running_mean", shape), (base + ".running_var", shape)]
    return out


def num_params(f: int = 64, in_ch: int = 3, model: str = "baseline") -> int:
    return int(sum(np.prod(s) for _, s in param_spec(f, in_ch, model)))


def init_params(f: int = 64, seed: int = 42, in_ch: int = 3, model: str = "baseline"):
    """torch.nn default init (kaiming_uniform(a=sqrt 5) weights, U(-1/sqrt(fan_in),..) biases,
    BN weight 1 / bias 0) — same distributions as the LibTorch modules; not bitwise the C++ stream.
    FiLM heads: fc_gamma/fc_beta weights N(0, 0.01), biases 1 / 0 (film_layer.h:68-71)."""
    g = torch.Generator().manual_seed(seed)
    params = OrderedDict()
    spec = dict(param_spec(f, in_ch, model))
    for name, shape in param_spec(f, in_ch, model):
        if ".bn" in name:
            params[name] = torch.ones(shape) if name.endswith("weight") else torch.zeros(shape)
            continue
        if ".fc_transform." in name:   # identity transform (pcl_layer.h:61-63)
            params[name] = (torch.zeros(shape) if name.endswith("weight")
                            else torch.tensor([1.0, 1.0, 0.0, 0.0, 0.0, 0.0]))
            continue
        if ".fc_gamma." in name or ".fc_beta." in name:
            if name.endswith("weight"):
                params[name] = torch.randn(shape, generator=g) * 0.01
            else:
                params[name] = torch.full(shape, 1.0 if ".fc_gamma." in name else 0.0)
            continue
        if name.endswith("weight"):
            fan_in = shape[1] * int(np.prod(shape[2:])) if "up." not in name else shape[1] * 4
            bound = 1.0 / math.sqrt(fan_in)  # kaiming_uniform_(a=sqrt(5)) => gain sqrt(2/6)*sqrt(3/fan)
            params[name] = (torch.rand(shape, generator=g) * 2 - 1) * bound
        else:
            wshape = spec[name[: -len("bias")] + "weight"]
            fan_in = wshape[1] * int(np.prod(wshape[2:])) if "up." not in name else wshape[1] * 4
            bound = 1.0 / math.sqrt(fan_in)
            params[name] = (torch.rand(shape, generator=g) * 2 - 1) * bound
    return params


def init_buffers(f: int = 64, in_ch: int = 3, model: str = "baseline"):
    return OrderedDict((n, torch.zeros(s) if n.endswith("mean") else torch.ones(s))
                       for n, s in buffer_spec(f, in_ch, model))


def synth_init(f: int = 64, in_ch: int = 3, model: str = "baseline"):
    """Counter-stream initial weights of ref_harness.cpp `--init synth` (bit-identical): u = u01(0x1A17,
    running offset); >=2-D: (2u-1)/sqrt(numel/size(0)); 1-D *.weight and *.fc_gamma.bias:
    1 + 0.1(2u-1); other 1-D: 0.1(2u-1)."""
    params = OrderedDict()
    off = 0
    one, two, tenth = np.float32(1.0), np.float32(2.0), np.float32(0.1)
    for name, shape in param_spec(f, in_ch, model):
        n = int(np.prod(shape))
        u = u01(0x1A17, np.arange(off, off + n, dtype=np.uint64))
        if len(shape) >= 2:
            bound = one / np.sqrt(np.float32(n // shape[0]))
            v = (two * u - one) * bound
        elif name.endswith(".weight") or name.endswith(".fc_gamma.bias"):
            v = one + tenth * (two * u - one)
        else:
            v = tenth * (two * u - one)
        params[name] = torch.from_numpy(v.astype(np.float32).reshape(shape))
        off += n
    return params


def cam_from_K(K):
    """a15 (no reference code): (B,3,3) -> (B,4) [fx, fy, cx, cy] = [K00, K11, K02, K12]."""
    return torch.stack([K[:, 0, 0], K[:, 1, 1], K[:, 0, 2], K[:, 1, 2]], 1).contiguous()


def normalize_cam(c, width, height):
    """IntrinsicsConditionedUNetImpl::normalizeCameraIntrinsics (intrinsics_unet.h:252-268)."""
    n = c.clone()
    n[:, 0] = c[:, 0] / width
    n[:, 1] = c[:, 1] / height
    n[:, 2] = (c[:, 2] / width) * 2.0 - 1.0
    n[:, 3] = (c[:, 3] / height) * 2.0 - 1.0
    return n


def rays_from_K(K, H, W):
    """a18: computeRayDirections (ray_direction_computer.cpp:17-62) per sample, laid out (B,3,H,W)
    (sunrgbd_loader.cpp:346-347), float32 like the reference: x = (u - cx) * (1/fx), ..., r / |r|."""
    K = K.to(torch.float32)
    fxi = (1.0 / K[:, 0, 0]).view(-1, 1, 1)
    fyi = (1.0 / K[:, 1, 1]).view(-1, 1, 1)
    cx, cy = K[:, 0, 2].view(-1, 1, 1), K[:, 1, 2].view(-1, 1, 1)
    u = torch.arange(W, dtype=torch.float32, device=K.device).view(1, 1, W)
    v = torch.arange(H, dtype=torch.float32, device=K.device).view(1, H, 1)
    x = ((u - cx) * fxi).expand(-1, H, W)
    y = ((v - cy) * fyi).expand(-1, H, W)
    n = torch.sqrt(x * x + y * y + 1.0)
    return torch.stack([x / n, y / n, 1.0 / n], 1).contiguous()


# GEMM operand precision of the conv / ConvT contractions.  "exact": the reference's fp32 (or the
# fp64 yardstick).  "bf16": the bf16 configs' arithmetic (BASELINE configs 3-5, cad.h CAD_GEMM_BF16):
# every contraction multiplies bf16-rounded operands — forward (x, w), dgrad (dy, w) and wgrad
# (dy, x) — and accumulates in the working dtype; the conv outputs (pre-BN) are stored as bf16, and
# in the U-Net family so is each DoubleConv's conv2 input gradient;
# BN, FiLM, the 1x1 head, the loss and the optimizer stay in the working dtype.  Not a reference behaviour (the reference has no bf16 path):
# the yardstick the GPU bf16 engine is checked against.
_GEMM = {"operands": "exact"}


class _RoundOperand(torch.autograd.Function):
    """bf16 rounding of a GEMM input in the forward; straight-through gradient."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g


class _RoundGradOperand(torch.autograd.Function):
    """Identity forward; bf16 rounding of the incoming gradient (the dy operand of dgrad/wgrad)."""

    @staticmethod
    def forward(ctx, y):
        return y.view_as(y)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


# Test hook for the bf16 arithmetic: {conv name ("enc1.conv1", "dec2.conv.conv2", ...): tensor (B,C,H,W)}.
# A listed convolution computes its output as usual, records it in Y_OWN[name], and passes the given
# value on instead (its gradient flows to its own output unchanged).  The full-size bf16 tests impose
# the GPU run's stored (bf16) pre-BN outputs this way, layer by layer, so each convolution is judged
# on identical inputs — otherwise a one-ulp fp32 difference next to a bf16 rounding boundary makes the
# two runs' stored values differ by 2^-8 and the difference compounds over the 18 layers.
Y_FORCE = {}
Y_OWN = {}


def _conv3x3(x, w, name=None):
    if _GEMM["operands"] == "bf16":
        y = _RoundGradOperand.apply(F.conv2d(_RoundOperand.apply(x), _RoundOperand.apply(w), None, 1, 1))
        # the bf16 engine stores the pre-BN outputs of its pre-split convolutions as bf16 (all but the
        # one on the raw 3-channel image, which runs the in-loader kernel with fp32 outputs)
        y = y if x.shape[1] == 3 else _RoundOperand.apply(y)
    else:
        y = F.conv2d(x, w, None, 1, 1)
    forced = Y_FORCE.get(name) if name else None
    if forced is None:
        return y
    Y_OWN[name] = y.detach().clone()
    return y + (forced.to(y.dtype) - y).detach()


def _convT2x2(x, w, b, bias_bf16=False):
    if _GEMM["operands"] in ("bf16", "mx8"):   # (mx8: the config-5 fp8 network keeps its ConvTs on bf16)
        y = F.conv_transpose2d(_RoundOperand.apply(x), _RoundOperand.apply(w), None, stride=2)
        if bias_bf16:   # U-Net family: the bias gradient sums the same bf16 gradient the GEMMs read
            return _RoundGradOperand.apply(y + b.view(1, -1, 1, 1))
        return _RoundGradOperand.apply(y) + b.view(1, -1, 1, 1)
    return F.conv_transpose2d(x, w, b, stride=2)


def _bn(x, p, bufs, prefix, train):
    # torch::nn::BatchNorm2d defaults (eps 1e-5, momentum 0.1, affine, track_running_stats)
    return F.batch_norm(x, bufs[prefix + ".running_mean"], bufs[prefix + ".running_var"],
                        p[prefix + ".weight"], p[prefix + ".bias"], train, 0.1, 1e-5)


# Test hook: {BatchNorm prefix ("enc1.bn1", "dec2.conv.bn2", ...): bool mask (B,C,H,W)}.  A BN-ReLU
# listed here takes the given ReLU decisions instead of sign(z): the tests impose the decisions of the
# GPU run they judge (read back from its stored pre-BN outputs), so that a pre-activation within
# rounding of 0 — a tie either fp32 path may break either way — does not move a whole BN gradient
# (one flipped element of a bias gradient whose per-pixel terms cancel 50-2000x is a percent of it).
RELU_FORCE = {}


def _bn_relu(x, p, bufs, prefix, train):
    z = _bn(x, p, bufs, prefix, train)
    m = RELU_FORCE.get(prefix)
    return F.relu(z) if m is None else z * m.to(z.dtype)


# Test hook: {FiLM prefix ("enc1.film.", ...): (gamma, beta) of shape (B, C)}.  A FiLM listed here
# applies the given modulation values (gradients still flow through its own MLP): the full-size bf16
# test imposes the GPU run's, so the conv after it sees identical bf16 operands (an fp32 ulp of gamma
# flips the bf16 rounding of a few 1e-4 of the modulated activations, and with them ~2% of the next
# convolution's rounded outputs).
FILM_FORCE = {}
FILM_OWN = {}


def _film(x, c, p, bufs, pre, train):
    # FiLMLayerImpl::forward (film_layer.h:82-108): BatchNorm1d only when the batch has > 1 sample
    def bn1d(h, name):
        if h.shape[0] <= 1:
            return h
        return F.batch_norm(h, bufs[pre + name + ".running_mean"], bufs[pre + name + ".running_var"],
                            p[pre + name + ".weight"], p[pre + name + ".bias"], train, 0.1, 1e-5)
    h = F.relu(bn1d(F.linear(c, p[pre + "fc1.weight"], p[pre + "fc1.bias"]), "bn1"))
    h = F.relu(bn1d(F.linear(h, p[pre + "fc2.weight"], p[pre + "fc2.bias"]), "bn2"))
    gamma = F.linear(h, p[pre + "fc_gamma.weight"], p[pre + "fc_gamma.bias"])
    beta = F.linear(h, p[pre + "fc_beta.weight"], p[pre + "fc_beta.bias"])
    forced = FILM_FORCE.get(pre)
    if forced is not None:
        FILM_OWN[pre] = (gamma.detach().clone(), beta.detach().clone())
        gamma = gamma + (forced[0].to(gamma.dtype) - gamma).detach()
        beta = beta + (forced[1].to(beta.dtype) - beta).detach()
    return gamma[:, :, None, None] * x + beta[:, :, None, None]


def _double_conv(x, p, bufs, pre, train, cam=None, da1_bf16=False):
    # DoubleConvImpl::forward (baseline_unet.h:32-43); with `cam`: FiLMDoubleConvImpl::forward
    # (intrinsics_unet.h:38-52) = RayEnhancedConvImpl::forward after its cat (geometry_aware_network.h:47-64)
    x = _conv3x3(x, p[pre + "conv1.weight"], pre + "conv1")
    x = _bn_relu(x, p, bufs, pre + "bn1", train)
    if cam is not None:
        x = _film(x, cam, p, bufs, pre + "film.", train)
    if da1_bf16 and _GEMM["operands"] == "bf16":
        # the U-Net family's bf16 engine stores conv2's input gradient (its dgrad output, read by the
        # FiLM and bn1 backward) as bf16 (cad_api.cpp double_conv_bwd)
        x = _RoundGradOperand.apply(x)
    x = _conv3x3(x, p[pre + "conv2.weight"], pre + "conv2")
    return _bn_relu(x, p, bufs, pre + "bn2", train)


def _decoder(x, skip, p, bufs, pre, train, cam=None, da1_bf16=False):
    # DecoderBlockImpl::forward (baseline_unet.h:83-102): up, pad-if-needed, cat({skip, up}), conv
    # (FiLMDecoderBlockImpl::forward, intrinsics_unet.h:91-110, is the same with a FiLM conv)
    if da1_bf16 and _GEMM["operands"] == "bf16":
        # the U-Net family's bf16 engine stores the ConvT's input gradient (its dgrad output: the
        # gradient of the block below's output, read by that block's bn2 backward) as bf16
        x = _RoundGradOperand.apply(x)
    x = _convT2x2(x, p[pre + "up.weight"], p[pre + "up.bias"], da1_bf16)
    dh, dw = skip.shape[2] - x.shape[2], skip.shape[3] - x.shape[3]
    if dh > 0 or dw > 0:
        x = F.pad(x, (dw // 2, dw - dw // 2, dh // 2, dh - dh // 2))
    if da1_bf16 and _GEMM["operands"] == "bf16":
        # ... and the skip half of the concat's gradient (the decoder conv1 dgrad's lower columns), to
        # which the max-pool path's fp32 gradient is then added
        skip = _RoundGradOperand.apply(skip)
    return _double_conv(torch.cat([skip, x], 1), p, bufs, pre + "conv.", train, cam, da1_bf16)


def _cbam(x, p, pre):
    """CBAMImpl::forward (spatial_attention.h:165-175): channel then spatial attention.
    Test hook GEO_DEBUG["force"][pre] = (argmax pixel [B][C], argmax channel [B*H*W]): the two max
    reductions select those elements instead (same values up to rounding; the gradients are routed
    as the run that made the decisions routed them)."""
    B, C = x.shape[:2]
    force = GEO_DEBUG.get("force", {}).get(pre)
    def mlp(v):   # ChannelAttentionImpl::forward (:58-75), shared fc1 -> relu -> fc2
        h = F.relu(F.linear(v, p[pre + "channel_attention.fc1.weight"], p[pre + "channel_attention.fc1.bias"]))
        return F.linear(h, p[pre + "channel_attention.fc2.weight"], p[pre + "channel_attention.fc2.bias"])
    if force is None:
        mx = F.adaptive_max_pool2d(x, 1).view(B, C)
    else:
        mx = x.reshape(B, C, -1).gather(2, force[0].view(B, C, 1)).view(B, C)
        true = F.adaptive_max_pool2d(x, 1).view(B, C)   # how far the forced choice is from a true argmax
        GEO_DEBUG.setdefault("gap", []).append(((true - mx).abs().max() / true.abs().max().clamp_min(1e-30)).item())
    att = torch.sigmoid(mlp(F.adaptive_avg_pool2d(x, 1).view(B, C)) + mlp(mx))
    x = x * att.view(B, C, 1, 1)
    # SpatialAttentionImpl::forward (:105-117)
    if force is None:
        smax = torch.max(x, 1, keepdim=True)[0]
    else:
        smax = x.gather(1, force[1].view(B, 1, x.shape[2], x.shape[3]))
        true = torch.max(x, 1, keepdim=True)[0]
        GEO_DEBUG.setdefault("gap", []).append(((true - smax).abs().max() / true.abs().max().clamp_min(1e-30)).item())
    s = torch.cat([torch.mean(x, 1, keepdim=True), smax], 1)
    return x * torch.sigmoid(F.conv2d(s, p[pre + "spatial_attention.conv.weight"], None, 1, 3))


def _pcl(x, cam, p, pre):
    """PerspectiveCorrectionLayerImpl::forward (pcl_layer.h:76-111) + buildAffineMatrix (:148-178)."""
    B = x.shape[0]
    loc = torch.cat([F.adaptive_avg_pool2d(x, 1).view(B, -1), cam], 1)
    h = F.relu(F.linear(loc, p[pre + "loc_fc1.weight"], p[pre + "loc_fc1.bias"]))
    h = F.relu(F.linear(h, p[pre + "loc_fc2.weight"], p[pre + "loc_fc2.bias"]))
    t = F.linear(h, p[pre + "fc_transform.weight"], p[pre + "fc_transform.bias"])
    c, s = torch.cos(t[:, 4]), torch.sin(t[:, 4])
    theta = torch.stack([torch.stack([t[:, 0] * c, -s + t[:, 5], t[:, 2]], 1),
                         torch.stack([s, t[:, 1] * c, t[:, 3]], 1)], 1)
    grid = F.affine_grid(theta, list(x.shape), align_corners=False)
    return F.grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=False)


GEO_DEBUG = {}


def geo_forward(x, p, bufs, train, max_depth, model, K):
    """GeometryAwareNetworkImpl::forward (geometry_aware_network.h:289-318) /
    LightweightGeometryNetworkImpl::forward (:385-402) fed (rgb, rays_from_K(K), cam_from_K(K));
    getDownsampledRays only feeds PCL's unused ray argument (pcl_layer.h:76-111) and is omitted."""
    nl, enc = _geo_names(model)
    keep = GEO_DEBUG.get("keep")   # test hook: {name: tensor} of the intermediate activations
    cam = normalize_cam(cam_from_K(K.to(x.dtype)), x.shape[3], x.shape[2])
    x = torch.cat([x, rays_from_K(K, x.shape[2], x.shape[3]).to(x.dtype)], 1)
    skips = [_double_conv(x, p, bufs, "enc1.", train, cam)]
    for l in range(1, nl):   # GeometryEncoderBlockImpl::forward (:92-103)
        y = _double_conv(F.max_pool2d(skips[-1], 2), p, bufs, f"{enc[l]}.conv.", train, cam)
        skips.append(_cbam(y, p, f"{enc[l]}.attention."))
    x = skips[-1]
    for l in range(nl - 2, -1, -1):   # GeometryDecoderBlockImpl::forward (:141-167)
        pre = f"dec{l + 1}."
        u0 = _convT2x2(x, p[pre + "up.weight"], p[pre + "up.bias"])
        u = _pcl(u0, cam, p, pre + "pcl.")
        cat = torch.cat([skips[l], u], 1)
        y = _double_conv(cat, p, bufs, pre + "conv.", train, cam)
        x = _cbam(y, p, pre + "attention.")
        if keep is not None:
            for k, t in ((f"cat{l}", cat), (f"u{l}", u0), (f"x{l}", x)):
                if t.requires_grad:
                    t.retain_grad()
                keep[k] = t
    x = F.conv2d(x, p["out_conv.weight"], p["out_conv.bias"])
    return torch.sigmoid(x) * max_depth


def unet_forward(x, p, bufs, train=True, max_depth=10.0, model="baseline", K=None):
    """BaselineUNetImpl::forward (baseline_unet.h:174-195); model "film":
    IntrinsicsConditionedUNetImpl::forward(x, cam_from_K(K)) (intrinsics_unet.h:204-228); "rayfilm":
    the same wiring with enc1 fed cat(x, rays_from_K(K)); "geo" / "geolite": geo_forward."""
    if model in GEO_LEVELS:
        return geo_forward(x, p, bufs, train, max_depth, model, K)
    cam = None
    if model != "baseline":
        cam = normalize_cam(cam_from_K(K.to(x.dtype)), x.shape[3], x.shape[2])
        if model == "rayfilm":
            x = torch.cat([x, rays_from_K(K, x.shape[2], x.shape[3]).to(x.dtype)], 1)
    # (the GPU's pre-split path, and with it the bf16 conv2 input gradient, needs f % 8 == 0)
    r = p["enc1.conv1.weight"].shape[0] % 8 == 0
    s1 = _double_conv(x, p, bufs, "enc1.", train, cam, r)
    # the bf16 engine pools the encoder outputs' bf16 twin (same pooled values; ties of the rounded
    # values go to the first in scan order, as in max_pool2d)
    rb = r and _GEMM["operands"] == "bf16"
    pool = lambda t: F.max_pool2d(_RoundOperand.apply(t) if rb else t, 2)
    s2 = _double_conv(pool(s1), p, bufs, "enc2.conv.", train, cam, r)
    s3 = _double_conv(pool(s2), p, bufs, "enc3.conv.", train, cam, r)
    s4 = _double_conv(pool(s3), p, bufs, "enc4.conv.", train, cam, r)
    xb = _double_conv(pool(s4), p, bufs, "bottleneck.conv.", train, cam, r)
    x = _decoder(xb, s4, p, bufs, "dec4.", train, cam, r)
    x = _decoder(x, s3, p, bufs, "dec3.", train, cam, r)
    x = _decoder(x, s2, p, bufs, "dec2.", train, cam, r)
    x = _decoder(x, s1, p, bufs, "dec1.", train, cam, r)
    x = F.conv2d(x, p["out_conv.weight"], p["out_conv.bias"])
    return torch.sigmoid(x) * max_depth


# --------------------------------------------------------------------------------------------
# Losses (depth_loss.h)
# --------------------------------------------------------------------------------------------
def si_loss(pred, gt, lam=0.5, eps=EPS, valid_mask=None):
    """ScaleInvariantLoss::forward (depth_loss.h:33-64): 0-dim result, zeros(1) when n == 0;
    valid_mask (bool) replaces gt > eps (:38-40)."""
    mask = valid_mask if valid_mask is not None else gt > eps
    pred = torch.clamp(pred, eps, 1000.0)
    gt = torch.clamp(gt, eps, 1000.0)
    d = (torch.log(pred) - torch.log(gt)).masked_select(mask)
    n = d.numel()
    if n == 0:
        return torch.zeros(1, dtype=pred.dtype, device=pred.device)
    return torch.pow(d, 2).sum() / n - lam * torch.pow(d.sum(), 2) / (n * n)


def _grad_scale(pred, gt):
    # GradientMatchingLoss::computeGradientLoss (depth_loss.h:135-166); the mask is unused (:137)
    px = pred[..., 1:] - pred[..., :-1]
    gx = gt[..., 1:] - gt[..., :-1]
    py = pred[..., 1:, :] - pred[..., :-1, :]
    gy = gt[..., 1:, :] - gt[..., :-1, :]
    return torch.abs(px - gx).mean() + torch.abs(py - gy).mean()


def grad_loss(pred, gt, num_scales=4, eps=EPS):
    """GradientMatchingLoss::forward (depth_loss.h:95-124): shape-[1] result."""
    total = torch.zeros(1, dtype=pred.dtype, device=pred.device)
    for s in range(num_scales):
        ps, gs = pred, gt
        if s > 0:
            k = 2 ** s
            ps = F.avg_pool2d(pred, k, k)
            gs = F.avg_pool2d(gt, k, k)
        ps = torch.log(torch.clamp(ps, eps, 1000.0))
        gs = torch.log(torch.clamp(gs, eps, 1000.0))
        total = total + _grad_scale(ps, gs)
    return total / num_scales


def smooth_loss(pred, image, eps=EPS):
    """SmoothnessLoss::forward (depth_loss.h:189-234)."""
    m = pred.mean((2, 3), keepdim=True)
    n = pred / (m + eps)
    dx = torch.abs(n[..., 1:] - n[..., :-1])
    dy = torch.abs(n[..., 1:, :] - n[..., :-1, :])
    ix = torch.abs(image[..., 1:] - image[..., :-1]).mean(1, keepdim=True)
    iy = torch.abs(image[..., 1:, :] - image[..., :-1, :]).mean(1, keepdim=True)
    return (dx * torch.exp(-ix)).mean() + (dy * torch.exp(-iy)).mean()


def reproj_loss(pred, gt, K, eps=EPS, valid_mask=None):
    """ReprojectionLoss::forward (depth_loss.h:268-331); valid_mask replaces gt > eps (:320-322)."""
    B, _, H, W = pred.shape
    if K.dim() == 2:
        K = K.unsqueeze(0).expand(B, 3, 3)
    gy = torch.arange(0, H, dtype=pred.dtype, device=pred.device).view(1, H, 1).expand(1, H, W)
    gx = torch.arange(0, W, dtype=pred.dtype, device=pred.device).view(1, 1, W).expand(1, H, W)
    fx = K[:, 0, 0].view(B, 1, 1, 1)
    fy = K[:, 1, 1].view(B, 1, 1, 1)
    cx = K[:, 0, 2].view(B, 1, 1, 1)
    cy = K[:, 1, 2].view(B, 1, 1, 1)
    pX = (gx - cx) * pred / (fx + eps)
    pY = (gy - cy) * pred / (fy + eps)
    tX = (gx - cx) * gt / (fx + eps)
    tY = (gy - cy) * gt / (fy + eps)
    dX, dY, dZ = pX - tX, pY - tY, pred - gt
    err = torch.sqrt(dX * dX + dY * dY + dZ * dZ + eps)
    e = err.masked_select(valid_mask if valid_mask is not None else gt > eps)
    if e.numel() == 0:
        return torch.zeros(1, dtype=pred.dtype, device=pred.device)
    return e.mean()


def combined_loss(pred, gt, image, K, weights=(1.0, 0.1, 0.001, 0.01), valid_mask=None):
    """CombinedDepthLoss::forwardWithIntrinsics (depth_loss.h:416-433). Returns (total, comps).
    valid_mask reaches the SI and reprojection terms; the gradient-matching term ignores it (:137)."""
    si = si_loss(pred, gt, valid_mask=valid_mask)
    gr = grad_loss(pred, gt)
    sm = smooth_loss(pred, image)
    rp = reproj_loss(pred, gt, K, valid_mask=valid_mask)
    w = [torch.tensor(float(x), dtype=torch.float32).item() for x in weights]
    total = w[0] * si + w[1] * gr + w[2] * sm + w[3] * rp
    comps = {"si_loss": float(si.detach()), "grad_loss": float(gr.detach()), "smooth_loss": float(sm.detach()),
             "reproj_loss": float(rp.detach())}
    return total, comps


def loss_and_dpred(pred, gt, image, K, weights=(1.0, 0.1, 0.001, 0.01), valid_mask=None):
    """Fused-loss reference: (total, comps, dL/dpred) for the GPU loss kernels' parity tests."""
    p = pred.detach().clone().requires_grad_(True)
    total, comps = combined_loss(p, gt, image, K, weights, valid_mask)
    total.sum().backward()
    return float(total), comps, p.grad.detach()


# --------------------------------------------------------------------------------------------
# Optimizer: clip_grad_norm_ (LibTorch clip_grad.h) + torch::optim::Adam (coupled L2)
# --------------------------------------------------------------------------------------------
def clip_grad_norm_(grads, max_norm=1.0):
    # parameters without a gradient (None: e.g. FiLM BatchNorm1d at batch 1) are skipped (clip_grad.h:29-35)
    grads = [g for g in grads if g is not None]
    norms = torch.stack([g.norm(2) for g in grads])
    total = norms.norm(2) if len(grads) > 1 else norms[0]
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for g in grads:
        g.mul_(coef)
    return float(total)


class Adam:
    """torch::optim::Adam with coupled L2 weight decay (AdamOptions(lr).weight_decay(wd))."""

    def __init__(self, params, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-5):
        self.params = params
        self.lr, self.b1, self.b2, self.eps, self.wd = lr, betas[0], betas[1], eps, weight_decay
        self.m = OrderedDict((k, torch.zeros_like(v)) for k, v in params.items())
        self.v = OrderedDict((k, torch.zeros_like(v)) for k, v in params.items())
        self.t = OrderedDict((k, 0) for k in params)   # per-parameter step (torch Adam state "step")
        self.t_global = 0

    @torch.no_grad()
    def step(self, grads):
        self.t_global += 1
        for (k, p), g in zip(self.params.items(), grads):
            if g is None:   # no gradient: the parameter and its state are left untouched (adam.cpp)
                continue
            self.t[k] += 1
            bc1 = 1 - self.b1 ** self.t[k]
            bc2 = 1 - self.b2 ** self.t[k]
            if self.wd != 0:
                g = g.add(p, alpha=self.wd)
            self.m[k].mul_(self.b1).add_(g, alpha=1 - self.b1)
            self.v[k].mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            denom = (self.v[k].sqrt() / math.sqrt(bc2)).add_(self.eps)
            p.addcdiv_(self.m[k], denom, value=-(self.lr / bc1))


class Trainer:
    """One replica of TensorBoardTrainerEnhanced's step (enhanced.h:287-304) on host cores."""

    def __init__(self, params, buffers, weights=(1.0, 0.1, 0.001, 0.01), lr=1e-4, wd=1e-5,
                 clip=1.0, max_depth=10.0, dtype=torch.float32, model="baseline", gemm_operands="exact",
                 device=None):
        # dtype=float64 gives the exact-arithmetic yardstick the fp32 paths are both measured against;
        # gemm_operands="bf16" the bf16 configs' contraction arithmetic (see _GEMM).  device: where
        # ATen evaluates this restatement — the host by default; the full-size test evaluates the
        # fp64 yardstick with ATen's GPU kernels (any exact-enough arithmetic serves as a yardstick)
        self.dtype = dtype
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.gemm_operands = gemm_operands
        self.model = model
        self.p = OrderedDict((k, v.clone().to(self.device, dtype)) for k, v in params.items())
        self.bufs = OrderedDict((k, v.clone().to(self.device, dtype)) for k, v in buffers.items())
        self.weights, self.clip, self.max_depth = weights, clip, max_depth
        self.opt = Adam(self.p, lr=lr, weight_decay=wd)

    def forward_backward(self, rgb, gt, K):
        rgb, gt, K = (t.to(self.device, self.dtype) for t in (rgb, gt, K))
        for v in self.p.values():
            v.requires_grad_(True)
            v.grad = None
        prev, _GEMM["operands"] = _GEMM["operands"], self.gemm_operands
        try:
            pred = unet_forward(rgb, self.p, self.bufs, True, self.max_depth, self.model, K)
            pred.retain_grad()
            loss, comps = combined_loss(pred, gt, rgb, K, self.weights)
            loss.sum().backward()
        finally:
            _GEMM["operands"] = prev
        grads = [v.grad.detach().clone() if v.grad is not None else None for v in self.p.values()]
        for v in self.p.values():
            v.requires_grad_(False)
        return pred.detach(), pred.grad.detach(), float(loss), comps, grads

    def apply(self, grads):
        total = clip_grad_norm_(grads, self.clip)
        self.opt.step(grads)
        return total

    def step(self, rgb, gt, K):
        pred, dpred, loss, comps, grads = self.forward_backward(rgb, gt, K)
        pre_clip = [g.clone() if g is not None else None for g in grads]
        total = self.apply(grads)
        return dict(pred=pred, dpred=dpred, loss=loss, comps=comps, grads=pre_clip, norm=total)

    @torch.no_grad()
    def predict_eval(self, rgb, K=None):
        Kd = K.to(self.device, self.dtype) if K is not None else None
        prev, _GEMM["operands"] = _GEMM["operands"], self.gemm_operands
        try:
            return unet_forward(rgb.to(self.device, self.dtype), self.p, self.bufs, False, self.max_depth, self.model,
                                Kd)
        finally:
            _GEMM["operands"] = prev


def depth_metrics(pred, gt):
    """computeDepthMetrics (enhanced.h:400-439) on flattened tensors."""
    p, g = pred.reshape(-1), gt.reshape(-1)
    m = g > 0
    p, g = p[m], g[m]
    if p.numel() == 0:
        return {}
    ad = (p - g).abs()
    ld = (torch.log(p + 1e-8) - torch.log(g + 1e-8)).abs()
    ratio = torch.maximum(p / g, g / p)
    return {"abs_rel": float((ad / g).mean()), "sq_rel": float((ad * ad / g).mean()),
            "rmse": float(torch.sqrt((ad * ad).mean())), "rmse_log": float(torch.sqrt((ld * ld).mean())),
            "a1": float((ratio < 1.25).float().mean()), "a2": float((ratio < 1.5625).float().mean()),
            "a3": float((ratio < 1.953125).float().mean())}


def abs_rel_per_sample(pred, gt):
    vals = [depth_metrics(pred[b], gt[b]).get("abs_rel") for b in range(pred.shape[0])]
    vals = [v for v in vals if v is not None]
    return sum(vals) / pred.shape[0]


# --------------------------------------------------------------------------------------------
# Batch assembly: SunRGBDLoader::getSample (src/data/sunrgbd_loader.cpp), decode excluded
# --------------------------------------------------------------------------------------------
def load_sample(rgb_u8_hwc, depth_u16, K, bgr=False, depth_scale=1.0 / 1000.0):
    """loadRGB :221-233 (cv::COLOR_BGR2RGB, matToTensor HWC->CHW, / 255.0f) and loadDepth :235-259
    (CV_16UC1 convertTo CV_32F with scale 1/1000: one single-precision product per pixel)."""
    rgb = torch.from_numpy(np.ascontiguousarray(rgb_u8_hwc)).float()
    if bgr:
        rgb = rgb.flip(2)
    rgb = rgb.permute(2, 0, 1).contiguous() / 255.0
    d = torch.from_numpy(depth_u16.astype(np.float32) * np.float32(depth_scale))[None]
    return rgb, d, torch.as_tensor(np.asarray(K, dtype=np.float32).reshape(3, 3)).clone()


def resize_sample(rgb, depth, K, H, W):
    """resizeSample :445-489: rgb bilinear (align_corners false), depth nearest, K scaled (float32)."""
    h, w = rgb.shape[1], rgb.shape[2]
    if (h, w) == (H, W):
        return rgb, depth, K
    rgb = F.interpolate(rgb[None], size=(H, W), mode="bilinear", align_corners=False)[0]
    depth = F.interpolate(depth[None], size=(H, W), mode="nearest")[0]
    sx, sy = np.float32(W) / np.float32(w), np.float32(H) / np.float32(h)
    K = K.clone()
    K[0, 0] = K[0, 0] * sx
    K[1, 1] = K[1, 1] * sy
    K[0, 2] = K[0, 2] * sx
    K[1, 2] = K[1, 2] * sy
    return rgb, depth, K


def augment_sample(rgb, depth, K, aug):
    """augmentSample :352-387 with the draws given: applyCrop :389-414 (slices clamp like torch's),
    applyHorizontalFlip :416-430, applyColorJitter :432-443."""
    K = K.clone()
    if aug.get("crop"):
        H, W = rgb.shape[1], rgb.shape[2]
        s = np.float32(aug["crop_scale"])
        ch, cw = int(np.float32(H) * s), int(np.float32(W) * s)
        cx, cy = int(aug["crop_x"]), int(aug["crop_y"])
        rgb = rgb[:, cy:cy + ch, cx:cx + cw]
        depth = depth[:, cy:cy + ch, cx:cx + cw]
        K[0, 2] = K[0, 2] - cx
        K[1, 2] = K[1, 2] - cy
    if aug.get("flip"):
        rgb, depth = torch.flip(rgb, [2]), torch.flip(depth, [2])
        K[0, 2] = rgb.shape[2] - K[0, 2] - 1
    if aug.get("jitter"):
        rgb = torch.clamp(rgb * np.float32(aug["contrast"]) + np.float32(aug["brightness"]) - 1.0, 0.0, 1.0)
    return rgb, depth, K


def get_sample(rgb_u8_hwc, depth_u16, K, H, W, aug=None, bgr=False, depth_scale=1.0 / 1000.0):
    """getSample :105-169: load, resize, then (train + augmentation) augment and resize again."""
    rgb, depth, K = load_sample(rgb_u8_hwc, depth_u16, K, bgr, depth_scale)
    rgb, depth, K = resize_sample(rgb, depth, K, H, W)
    if aug and aug.get("aug"):
        rgb, depth, K = augment_sample(rgb, depth, K, aug)
        rgb, depth, K = resize_sample(rgb, depth, K, H, W)
    return rgb, depth, K


class StdMt19937Draws:
    """augmentSample's draws as libstdc++ makes them: std::mt19937 (== numpy RandomState's legacy
    init_genrand seeding and 32-bit outputs), uniform_real_distribution<float> via
    generate_canonical<float, 24> (one 32-bit draw, sum / 2^32 in float, nudged below 1), and
    uniform_int_distribution<int> by Lemire's nearly-divisionless downscaling (libstdc++ 11,
    bits/uniform_int_dist.h _S_nd for 32-bit engines)."""

    def __init__(self, seed, cfg):
        self.rs = np.random.RandomState(seed)
        self.cfg = cfg

    def _u32(self):
        return int(self.rs.randint(0, 2 ** 32, dtype=np.uint64))

    def _real(self, a, b):
        a, b = np.float32(a), np.float32(b)
        r = np.float32(self._u32()) / np.float32(2.0 ** 32)
        if r >= np.float32(1.0):
            r = np.nextafter(np.float32(1.0), np.float32(0.0))
        return np.float32(r * (b - a) + a)

    def _int(self, a, b):
        rng = (b - a) + 1
        prod = self._u32() * rng
        low = prod & 0xFFFFFFFF
        if low < rng:
            thr = (2 ** 32 - rng) % rng
            while low < thr:
                prod = self._u32() * rng
                low = prod & 0xFFFFFFFF
        return a + (prod >> 32)

    def draw(self, H, W):
        c = self.cfg
        out = {"aug": 1, "crop": int(c["enable_random_crop"]), "flip": 0, "jitter": int(c["enable_color_jitter"])}
        if c["enable_random_crop"]:
            s = self._real(c["crop_scale_min"], c["crop_scale_max"])
            ch, cw = int(np.float32(H) * s), int(np.float32(W) * s)
            out["crop_scale"] = float(s)
            out["crop_x"] = self._int(0, max(1, W - cw))
            out["crop_y"] = self._int(0, max(1, H - ch))
        if c["enable_horizontal_flip"]:
            out["flip"] = int(self._real(0.0, 1.0) < np.float32(c["horizontal_flip_prob"]))
        if c["enable_color_jitter"]:
            one, bd, cd = np.float32(1.0), np.float32(c["brightness_delta"]), np.float32(c["contrast_delta"])
            out["brightness"] = float(self._real(one - bd, one + bd))
            out["contrast"] = float(self._real(one - cd, one + cd))
        return out


# --------------------------------------------------------------------------------------------
# Golden fixture I/O (written by oracle/ref_harness.cpp)
# --------------------------------------------------------------------------------------------
def load_fixture(path):
    import json
    import os
    with open(os.path.join(path, "manifest.json")) as fh:
        man = json.load(fh)
    raw = np.fromfile(os.path.join(path, "tensors.bin"), dtype="<f4")
    out = OrderedDict()
    for t in man["tensors"]:
        n = int(np.prod(t["shape"])) if t["shape"] else 1
        out[t["name"]] = torch.from_numpy(raw[t["offset"]: t["offset"] + n].reshape(t["shape"]).copy())
    return out, man["meta"]
