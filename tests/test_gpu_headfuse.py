"""Level-0 head fusion (nn_kernels.hip bn_relu_head_fwd / head_bwd_y / bn_relu_bwd's HeadGrad form,
wired in cad_api.cpp): decoder level 0's bn2 + ReLU feed the depth head without storing the fp32
activation, and the backward rebuilds the head's input gradient per row.  The fused passes keep
the unfused arithmetic and summation order, so two training steps with and without the fusion
(CAD_HEADFUSE=0, read once per process) must agree BIT FOR BIT: predictions, losses, every gradient
and every parameter after the Adam steps.  Widths cover C/4 = 1, 2 (k_head_fwd's sequential sum)
and the butterfly forms, and 24 (not fusable: both runs take the unfused path)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, fuse, args, var="CAD_HEADFUSE"):
    out = tmp_path / f"{var}{fuse}.pt"
    env = dict(os.environ, **{var: str(fuse)})
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "headfuse_ab.py"), *map(str, args), str(out)],
                   check=True, env=env, timeout=300)
    return torch.load(out, weights_only=True)


@pytest.mark.parametrize("kind,eng,f,B,H,W", [("baseline", 2, 4, 2, 64, 64), ("baseline", 2, 8, 2, 48, 64),
                                              ("baseline", 1, 64, 2, 64, 96), ("film", 1, 32, 2, 64, 64),
                                              ("rayfilm", 2, 16, 3, 64, 96), ("baseline", 2, 96, 1, 32, 32)])
def test_head_fusion_bit_identical(tmp_path, kind, eng, f, B, H, W):
    a = _run(tmp_path, 0, (kind, eng, f, B, H, W))
    b = _run(tmp_path, 1, (kind, eng, f, B, H, W))
    assert a.keys() == b.keys()
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    assert not bad, bad[:8]


@pytest.mark.parametrize("var,kind,eng,f,B,H,W", [("CAD_POOLFOLD", "baseline", 2, 16, 2, 64, 96),
                                                  ("CAD_POOLFOLD", "rayfilm", 2, 32, 2, 48, 64),
                                                  ("CAD_DCATSPLIT", "baseline", 1, 64, 2, 64, 64),
                                                  ("CAD_DCATSPLIT", "rayfilm", 1, 32, 2, 48, 64),
                                                  ("CAD_DCATSPLIT", "film", 1, 16, 2, 64, 96),
                                                  ("CAD_BNPOOL", "baseline", 2, 16, 2, 64, 96),
                                                  ("CAD_BNPOOL", "rayfilm", 2, 32, 2, 48, 64),
                                                  ("CAD_BNPOOL", "baseline", 1, 64, 2, 64, 64),
                                                  ("CAD_BNPOOL", "film", 0, 16, 2, 64, 96),
                                                  ("CAD_BNSUMS", "baseline", 1, 16, 2, 64, 96),
                                                  ("CAD_BNSUMS", "baseline", 1, 64, 2, 64, 128),
                                                  ("CAD_BNSUMS", "baseline", 1, 64, 2, 64, 64),
                                                  ("CAD_BNSUMS", "baseline", 1, 32, 2, 48, 64),
                                                  ("CAD_POOLQ", "baseline", 2, 16, 2, 64, 96),
                                                  ("CAD_POOLQ", "rayfilm", 2, 32, 2, 48, 64),
                                                  ("CAD_POOLQ", "baseline", 1, 64, 2, 64, 64)])
def test_backward_fusions_bit_identical(tmp_path, var, kind, eng, f, B, H, W):
    """CAD_POOLFOLD (fp32 engines; the bf16 engine always folds): the max-pool backward folded into the
    encoder's bn2 backward (nn_kernels.hip pool_add) makes the scatter's fp32 add per element.
    CAD_DCATSPLIT (bf16 engine): the decoder conv1 dgrad writes dcat's two halves straight into their
    bf16 buffers (EpiStoreSplit2B16) with the rounding split_rows applies.  CAD_BNPOOL (all engines):
    each encoder block's bn2 + ReLU pass also writes the next level's max-pool (nn_kernels.hip
    bn_relu_pool_fwd: the same affine, rounding and comparison).  CAD_BNSUMS (S3 engine): bn1's
    backward sums come from conv2's input-gradient window epilogue (EpiStoreBnSums: fp64 sums of the
    same fp32 terms in another order).  CAD_POOLQ: the encoder bn2 backward with the folded max-pool walked
    over pooled pixels (OpBnBwdPoolQ, k_bn_relu_bwd_poolq: the same adds per element, fp64 sums in another
    order).  Two training steps with and without each agree bit for bit."""
    a = _run(tmp_path, 0, (kind, eng, f, B, H, W), var)
    b = _run(tmp_path, 1, (kind, eng, f, B, H, W), var)
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    assert not bad, bad[:8]
