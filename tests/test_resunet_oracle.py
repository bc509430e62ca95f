"""CPU checks of the config-5 restatement (oracle/resunet_oracle.py; parity unpinned: the reference
has no ResNet-50 model): torchvision's ResNet-50 encoder parameter count, the
decoder's shapes, and that the bf16-operand emulation stays close to the fp32 network."""
import torch

from oracle import resunet_oracle as R


def test_encoder_is_torchvision_resnet50():
    spec = R.param_spec()
    enc = sum(int(torch.tensor(s).prod()) for n, s in spec if n.startswith("encoder."))
    assert enc == 23_508_032   # torchvision resnet50: 25,557,032 parameters minus fc (2048*1000 + 1000)
    names = [n for n, _ in spec]
    assert len(names) == len(set(names))
    assert names[:3] == ["encoder.conv1.weight", "encoder.bn1.weight", "encoder.bn1.bias"]
    assert "encoder.layer4.2.bn3.bias" in names and "encoder.layer3.0.downsample.0.weight" in names
    assert names[-2:] == ["out_conv.weight", "out_conv.bias"]
    assert len(R.buffer_spec()) == 2 * sum(1 for n, s in spec if n.endswith(".weight") and len(s) == 1)


def test_forward_shapes_and_bf16_emulation():
    p, b = R.init(seed=3)
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(1))
    t32 = R.Trainer(p, b, operands="exact").predict_eval(x)
    t16 = R.Trainer(p, b, operands="bf16").predict_eval(x)
    assert t32.shape == (2, 1, 64, 64) and bool(((t32 > 0) & (t32 < 10)).all())
    assert (t16 - t32).abs().max() / t32.abs().max() < 5e-2


def test_mx8_quantize_known_answers():
    """MXFP8 E4M3 (gemm_mx8.hpp): shared exponent floor(log2 amax) - 8, e4m3fn RNE elements saturated at
    448; the GPU quantiser is held bit-exact to this function on the box (tests/test_gpu_mx8.py)."""
    v = torch.zeros(4, 32)
    v[0, 0] = 1.0                   # amax 1 -> scale 2^-8 (code 119); 1.0 -> 256 = e4m3 0x78
    v[0, 1] = 1.0625                # 272: a tie between 256 and 288 -> even mantissa (256)
    v[0, 2] = 1.0625 + 2 ** -20     # just above the tie -> 288 (0x79)
    v[0, 3] = -0.5                  # 128 -> 0xF0
    v[1, :] = 500.0                 # amax 500 -> scale 2^0; 500 saturates at 448 (0x7E)
    v[2, 5] = 2.0 ** -40            # tiny block: shared exponent -48 (code 79), element 256
    # v[3]: a zero block -> scale code 0 (2^-127), elements 0
    q, s, d = R.mx8_quantize(v)
    assert s[:, 0].tolist() == [119, 127, 79, 0]
    assert q[0, :4].tolist() == [0x78, 0x78, 0x79, 0xF0]
    assert q[1].unique().tolist() == [0x7E] and d[1, 0].item() == 448.0
    assert q[2, 5].item() == 0x78 and d[2, 5].item() == 2.0 ** -40
    assert q[3].abs().sum().item() == 0 and d[3].abs().sum().item() == 0
    assert torch.equal(R.mx8_dequant(q, s).float(), d)


def test_mx8_emulation_and_eligibility():
    """operands="mx8" (the fp8 network, cad_resunet_set_fp8): the eligible forward contractions on MX
    operands; at 480x640 that is every 1x1 / strided / window conv of the encoder and decoder except
    the stem, the 64-wide layer-1 convolutions at W = 160 and the 32-channel dec0 block."""
    assert R.x8_eligible(1, 1, 256, 64, 160) and R.x8_eligible(3, 2, 128, 128, 160)
    assert not R.x8_eligible(1, 1, 64, 64, 160)      # K = 64 (< one 128-deep stage)
    assert not R.x8_eligible(3, 1, 64, 64, 160)      # 256x64 window tiles need W % 64
    assert R.x8_eligible(3, 1, 1536, 512, 40) and not R.x8_eligible(3, 1, 32, 32, 640)
    assert not R.x8_eligible(7, 2, 4, 64, 640)       # stem: K = 196 -> 200
    p, b = R.init(seed=3)
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(1))
    t16 = R.Trainer(p, b, operands="bf16").predict_eval(x)
    t8 = R.Trainer(p, b, operands="mx8").predict_eval(x)
    e = ((t8 - t16).abs().max() / t16.abs().max()).item()
    assert 1e-6 < e < 0.2, e   # fp8 changes the result, boundedly


def test_convT_bias_gradient_from_bf16_operand():
    """The U-Net family's ConvT bias gradient sums the bf16-rounded up-half gradient the ConvT GEMMs read
    (resunet.cpp colsum_bf16 over dup; cad_oracle._convT2x2 bias_bf16).  Against the fp64 sum of the
    unrounded gradient the error per channel is at most 2^-9 * sum |g| (round-to-nearest-even to bf16,
    relative error <= 2^-9 per term), and this records how large it is relative to the bias gradient
    itself on a random-sign gradient (where the sum cancels)."""
    from oracle import cad_oracle as O
    gen = torch.Generator().manual_seed(7)
    x = torch.randn(2, 16, 12, 10, generator=gen, dtype=torch.float64)
    w = torch.randn(16, 8, 2, 2, generator=gen, dtype=torch.float64) * 0.1
    g = torch.randn(2, 8, 24, 20, generator=gen, dtype=torch.float64)
    prev, O._GEMM["operands"] = O._GEMM["operands"], "bf16"
    try:
        grads = []
        for flag in (True, False):
            b = torch.zeros(8, dtype=torch.float64, requires_grad=True)
            (O._convT2x2(x, w, b, bias_bf16=flag) * g).sum().backward()
            grads.append(b.grad)
    finally:
        O._GEMM["operands"] = prev
    g16, g64 = grads
    assert torch.equal(g64, g.sum((0, 2, 3)))
    bound = 2.0 ** -9 * g.abs().sum((0, 2, 3))
    assert bool(((g16 - g64).abs() <= bound).all()), ((g16 - g64).abs() / bound).max()
    # recorded: relative to |sum g| the error is ~2^-9 * sqrt(n) / |mean-free sum| — at most a few 1e-3
    # here (960 terms per channel), the size of the per-tensor 1-cos the full-size tests see on up.bias
    rel = ((g16 - g64).abs() / g64.abs()).max().item()
    assert rel < 2e-2, rel


def test_forcing_hooks_with_own_values_are_identity():
    """The full-size test's hooks (OUT_FORCE, COEF_FORCE, CAT_FORCE, cad_oracle.Y_FORCE / RELU_FORCE):
    imposing this restatement's own forward values reproduces its step bit for bit (the straight-through
    form forced + (y - y) carries the value exactly and the gradient unchanged)."""
    from oracle import cad_oracle as O
    p, b = R.init(seed=3)
    B, H, W = 1, 64, 64
    rgb, gt, K = [torch.from_numpy(a) for a in O.synth_batch(B, H, W)]
    r0 = R.Trainer(p, b, operands="bf16").step(rgb, gt, K)
    R.TRACE = {}
    try:
        R.Trainer(p, b, operands="bf16").step(rgb, gt, K)
        own = R.TRACE
    finally:
        R.TRACE = None
    R.CAT_FORCE.update({"dec0": torch.zeros(B, 32, H, W)})   # a forced decoder input must change the step
    try:
        r1 = R.Trainer(p, b, operands="bf16").step(rgb, gt, K)
    finally:
        R.CAT_FORCE.clear()
    assert not torch.equal(r0["pred"], r1["pred"])
    R.OUT_FORCE.update(own)
    try:
        r2 = R.Trainer(p, b, operands="bf16").step(rgb, gt, K)
    finally:
        R.OUT_FORCE.clear()
    assert torch.equal(r0["pred"], r2["pred"]) and r0["loss"] == r2["loss"]
    for g0, g2 in zip(r0["grads"], r2["grads"]):
        assert torch.equal(g0, g2)
