"""ORACLE / TEST INFRASTRUCTURE ONLY — regenerates tests/golden/ from the compiled reference.

Runs oracle/_ref/ref_harness (built by `make -C oracle` from /root/reference/src headers, in this
container only) and writes the fixtures the test-suite pins the oracle and the HIP path against.
Run:  make -C oracle && python oracle/gen_golden.py
All fixtures are generated single-threaded (torch::set_num_threads(1)) with manual_seed(42).
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
GOLDEN = os.path.join(ROOT, "tests", "golden")

FIXTURES = {
    # whole train step(s), default 4-term weights (train_config.yaml:89-92), f=4, 64x64
    "train_f4_b2_64x64": ["--mode", "golden", "--f", "4", "--B", "2", "--H", "64", "--W", "64",
                          "--steps", "3"],
    # config-2 semantics: SI-only weights, non-square 96x128, batch 3 (odd: mixed K per sample)
    "train_f4_b3_96x128_si": ["--mode", "golden", "--f", "4", "--B", "3", "--H", "96", "--W", "128",
                              "--steps", "2", "--weights", "1,0,0,0"],
    # config-3 model families: FiLM-conditioned U-Net on (B,4) intrinsics, and
    # the RayEnhancedConv + FiLM composite fed cat(rgb, rays); full 4-term loss
    "train_film_f4_b2_64x64": ["--mode", "golden", "--model", "film", "--init", "synth", "--f", "4", "--B", "2", "--H", "64",
                               "--W", "64", "--steps", "3"],
    "train_rayfilm_f4_b3_64x96": ["--mode", "golden", "--model", "rayfilm", "--init", "synth", "--f", "4", "--B", "3", "--H", "64",
                                  "--W", "96", "--steps", "2"],
    # geometry-aware family: GeometryAwareNetwork (6 levels, CBAM + PCL, B = 2:
    # FiLM's BatchNorm1d over two samples) and LightweightGeometryNetwork (5 levels, B = 3); lean: the
    # parameters after the last step are not stored (the losses, BN buffers and the eval prediction
    # pin the trajectory)
    "train_geo_f4_b2_64x64": ["--mode", "golden", "--model", "geo", "--init", "synth", "--f", "4", "--B", "2",
                              "--H", "64", "--W", "64", "--steps", "2", "--lean", "1"],
    "train_geolite_f4_b3_48x64": ["--mode", "golden", "--model", "geolite", "--init", "synth", "--f", "4", "--B", "3",
                                  "--H", "48", "--W", "64", "--steps", "2", "--lean", "1"],
    # loss-only goldens (depth_loss.h) incl. a size whose pyramid floors (50x70 -> 6x8 at k=8)
    "loss_b2_120x160": ["--mode", "loss", "--B", "2", "--H", "120", "--W", "160"],
    "loss_b3_50x70": ["--mode", "loss", "--B", "3", "--H", "50", "--W", "70"],
    "loss_b2_32x48_allholes": ["--mode", "loss", "--B", "2", "--H", "32", "--W", "48", "--holes-all", "1"],
    # forwardWithIntrinsics' optional valid_mask (depth_loss.h:416-433), independent of gt
    "loss_b2_48x64_mask": ["--mode", "loss", "--B", "2", "--H", "48", "--W", "64", "--mask-seed", "77"],
    # a checkpoint written by the reference's own torch::save(model_, path) (enhanced.h:656-662) after
    # one training step from LibTorch's default init (seed 42): only the archive is kept
    "ckpt_baseline_f4": ["--mode", "save", "--f", "4", "--B", "2", "--H", "32", "--W", "32", "--steps", "1",
                         "--ckpt", "{out}/baseline_unet_epoch_1.pt"],
}


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the harness first: make -C oracle")
    only = set(sys.argv[1:])
    for name, args in FIXTURES.items():
        if only and name not in only:
            continue
        out = os.path.join(GOLDEN, name)
        os.makedirs(out, exist_ok=True)
        if "--ckpt" in args:   # keep the archive, not the tensor dump
            with tempfile.TemporaryDirectory() as tmp:
                subprocess.run([HARNESS, "--threads", "1", "--out", tmp] + [a.format(out=out) for a in args], check=True)
            continue
        subprocess.run([HARNESS, "--threads", "1", "--out", out] + args, check=True)


if __name__ == "__main__":
    main()
