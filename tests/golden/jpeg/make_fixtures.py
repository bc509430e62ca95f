"""Writes the JPEG decoder fixtures of tests/test_jpeg.py (run in the build container, where PIL is
importable; the files are committed): <name>.jpg encoded by PIL and <name>.npy = PIL's decode of it
(libjpeg-turbo, the library behind the reference's cv::imread(IMREAD_COLOR), sunrgbd_loader.cpp:86,222,
with its default settings: ISLOW IDCT, fancy upsampling).  RGB (H, W, 3) or gray (H, W) uint8.

  python tests/golden/jpeg/make_fixtures.py"""
import io
import json
import os

import numpy as np
from PIL import Image, features

OUT = os.path.dirname(os.path.abspath(__file__))
CASES = {
    # name: (H, W, gray, save kwargs)
    "yuv420_odd_37x53_q90": (37, 53, False, dict(quality=90, subsampling=2)),
    "yuv422_48x64_q75": (48, 64, False, dict(quality=75, subsampling=1)),
    "yuv444_16x24_q95": (16, 24, False, dict(quality=95, subsampling=0)),
    "gray_33x17_q85": (33, 17, True, dict(quality=85)),
    "yuv420_120x160_q100": (120, 160, False, dict(quality=100, subsampling=2)),
    "yuv420_121x161_q50_optimized": (121, 161, False, dict(quality=50, subsampling=2, optimize=True)),
    "yuv420_2x2_q90": (2, 2, False, dict(quality=90, subsampling=2)),
    "yuv422_5x3_q90": (5, 3, False, dict(quality=90, subsampling=1)),
    "yuv420_64x64_restart3": (64, 64, False, dict(quality=90, subsampling=2, restart_marker_blocks=3)),
    "yuv420_96x128_restart_rows": (96, 128, False, dict(quality=80, subsampling=2, restart_marker_rows=1)),
}
# progressive (libjpeg's jpeg_simple_progression script: DC first / refine, spectral bands, successive
# approximation with end-of-band runs); image seeds 50+ so the sequential cases keep theirs
PROG_CASES = {
    "prog_yuv420_odd_37x53_q90": (37, 53, False, dict(quality=90, subsampling=2, progressive=True)),
    "prog_yuv444_40x24_q95": (40, 24, False, dict(quality=95, subsampling=0, progressive=True)),
    "prog_yuv422_48x64_q75_optimized": (48, 64, False, dict(quality=75, subsampling=1, progressive=True, optimize=True)),
    "prog_gray_33x17_q85": (33, 17, True, dict(quality=85, progressive=True)),
    "prog_yuv420_64x64_restart3": (64, 64, False, dict(quality=90, subsampling=2, progressive=True,
                                                        restart_marker_blocks=3)),
    "prog_yuv420_120x160_q100": (120, 160, False, dict(quality=100, subsampling=2, progressive=True)),
    "prog_yuv420_16x16_q90": (16, 16, False, dict(quality=90, subsampling=2, progressive=True)),
}


def image(h, w, gray, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = np.stack([128 + 100 * np.sin(x / 7.0 + c) * np.cos(y / 5.0 - c) for c in range(3)], -1)
    a = np.clip(base + rng.normal(0, 25, base.shape), 0, 255).astype(np.uint8)
    return Image.fromarray(a[..., 0] if gray else a)


def _exif_be(o):
    """An Exif APP1 body with a big-endian ("MM") TIFF header whose IFD0 holds one entry: orientation o."""
    import struct
    tiff = b"MM" + struct.pack(">HI", 42, 8) + struct.pack(">H", 1) + struct.pack(">HHIHH", 0x0112, 3, 1, o, 0) \
        + struct.pack(">I", 0)
    return b"Exif\x00\x00" + tiff


def main():
    meta = {"libjpeg": features.version("jpg"), "libjpeg_turbo": bool(features.check_feature("libjpeg_turbo")),
            "cases": {}}
    for k, (name, (h, w, gray, kw)) in enumerate(sorted(CASES.items())):
        bio = io.BytesIO()
        image(h, w, gray, k).save(bio, "JPEG", **kw)
        data = bio.getvalue()
        with open(os.path.join(OUT, name + ".jpg"), "wb") as fh:
            fh.write(data)
        dec = np.asarray(Image.open(io.BytesIO(data)).convert("L" if gray else "RGB"))
        np.save(os.path.join(OUT, name + ".npy"), dec)
        meta["cases"][name] = {"shape": list(dec.shape), "bytes": len(data)}
    for k, (name, (h, w, gray, kw)) in enumerate(sorted(PROG_CASES.items())):
        bio = io.BytesIO()
        image(h, w, gray, 50 + k).save(bio, "JPEG", **kw)
        data = bio.getvalue()
        with open(os.path.join(OUT, name + ".jpg"), "wb") as fh:
            fh.write(data)
        dec = np.asarray(Image.open(io.BytesIO(data)).convert("L" if gray else "RGB"))
        np.save(os.path.join(OUT, name + ".npy"), dec)
        meta["cases"][name] = {"shape": list(dec.shape), "bytes": len(data), "progressive": True}
    # EXIF orientation 1..8 (APP1, both TIFF byte orders): the expected pixels are the decode with the
    # orientation applied (PIL ImageOps.exif_transpose; OpenCV's imread(IMREAD_COLOR) applies the tag
    # the same way, loadsave.cpp ExifTransform)
    from PIL import ImageOps
    for o in range(1, 9):
        name = f"exif_orient{o}_yuv420_24x40"
        ex = Image.Exif()
        ex[0x0112] = o
        exb = ex.tobytes() if o % 2 else _exif_be(o)   # big-endian TIFF header for the even cases
        bio = io.BytesIO()
        image(24, 40, False, 200 + o).save(bio, "JPEG", quality=90, subsampling=2, exif=exb)
        data = bio.getvalue()
        with open(os.path.join(OUT, name + ".jpg"), "wb") as fh:
            fh.write(data)
        dec = np.asarray(ImageOps.exif_transpose(Image.open(io.BytesIO(data))).convert("RGB"))
        np.save(os.path.join(OUT, name + ".npy"), dec)
        meta["cases"][name] = {"shape": list(dec.shape), "bytes": len(data), "orientation": o}
    # a progressive file cut after its first three scans (the AC coefficients never refined to bit 0):
    # libjpeg-turbo would smooth its blocks (jdcoefct.c smoothing_ok); the decoder refuses it
    bio = io.BytesIO()
    image(48, 64, False, 99).save(bio, "JPEG", quality=90, subsampling=2, progressive=True)
    data = bio.getvalue()
    sos = [i for i in range(len(data) - 1) if data[i] == 0xFF and data[i + 1] == 0xDA]
    with open(os.path.join(OUT, "progressive_partial_48x64.jpg"), "wb") as fh:
        fh.write(data[:sos[3]] + b"\xff\xd9")
    with open(os.path.join(OUT, "fixtures.json"), "w") as fh:
        json.dump(meta, fh, indent=1)


if __name__ == "__main__":
    main()
