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
