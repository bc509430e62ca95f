"""JPEG decoding of the data path (csrc/host/jpeg.cpp): the reference loads SUN
RGB-D's RGB frames with cv::imread(path, IMREAD_COLOR) (src/data/sunrgbd_loader.cpp:86,222), i.e.
libjpeg-turbo's default decompression.  Fixtures (tests/golden/jpeg, made by make_fixtures.py in the
build container): files PIL encoded and PIL's own libjpeg-turbo decode of them — 4:2:0 / 4:2:2 /
4:4:4 / gray, odd and tiny sizes, quality 50..100, optimised Huffman tables, restart intervals.
The bar is bit-exact.  CPU only (host decoder)."""
import ctypes as C
import glob
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

JDIR = os.path.join(GOLDEN, "jpeg")
CASES = sorted(json.load(open(os.path.join(JDIR, "fixtures.json")))["cases"])


def _decode(cad, data):
    lib = cad.load_library()
    buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
    h, w, c = C.c_int(), C.c_int(), C.c_int()
    st = lib.cad_jpeg_decode(buf, len(data), None, 0, C.byref(h), C.byref(w), C.byref(c))
    if st != 0:
        raise cad.CadError(lib.cad_last_error().decode())
    out = np.empty(h.value * w.value * c.value, np.uint8)
    assert lib.cad_jpeg_decode(buf, len(data), out.ctypes.data, out.size, None, None, None) == 0
    out = out.reshape(h.value, w.value, c.value)
    return out[..., 0] if c.value == 1 else out


@pytest.mark.parametrize("name", CASES)
def test_decode_matches_libjpeg_turbo_fixture(cad, name):
    data = open(os.path.join(JDIR, name + ".jpg"), "rb").read()
    want = np.load(os.path.join(JDIR, name + ".npy"))
    got = _decode(cad, data)
    assert got.shape == want.shape and got.dtype == np.uint8
    diff = np.abs(got.astype(int) - want.astype(int))
    assert diff.max() == 0, (name, int(diff.max()), int((diff > 0).sum()))


def test_fixture_set_covers_the_decoder_paths():
    names = set(CASES)
    assert {"yuv420_odd_37x53_q90", "yuv422_48x64_q75", "yuv444_16x24_q95", "gray_33x17_q85"} <= names
    assert any("restart" in n for n in names) and any("optimized" in n for n in names)


def test_decoder_errors(cad):
    prog = open(os.path.join(JDIR, "progressive_16x16.jpg"), "rb").read()
    with pytest.raises(cad.CadError, match="progressive"):
        _decode(cad, prog)
    with pytest.raises(cad.CadError, match="not a JPEG"):
        _decode(cad, b"\x89PNG\r\n\x1a\n" + b"\0" * 32)
    good = open(os.path.join(JDIR, "yuv420_odd_37x53_q90.jpg"), "rb").read()
    for cut in (10, 200, len(good) // 2):   # truncated headers / data: an error or a decode, never a crash
        try:
            _decode(cad, good[:cut])
        except cad.CadError:
            pass


def test_loader_reads_jpeg_frames(cad, tmp_path):
    """cad_dataset_read of a manifest sample whose <path>/image holds a .jpg: the frame decoded as
    imread(IMREAD_COLOR) + BGR2RGB would (RGB; a gray JPEG replicated to three channels)."""
    PIL = pytest.importorskip("PIL.Image")
    for k, name in enumerate(("yuv420_odd_37x53_q90", "gray_33x17_q85")):
        d = tmp_path / f"s{k}"
        (d / "image").mkdir(parents=True)
        (d / "depth").mkdir(parents=True)
        (d / "image" / "frame.jpg").write_bytes(open(os.path.join(JDIR, name + ".jpg"), "rb").read())
        want = np.load(os.path.join(JDIR, name + ".npy"))
        PIL.fromarray(np.full(want.shape[:2], 1234, np.uint16)).save(d / "depth" / "d.png")
        (d / "intrinsics.txt").write_text("1 0 2\n0 3 4\n0 0 1\n")
        m = tmp_path / f"m{k}.json"
        m.write_text(json.dumps({"images": [{"path": str(d), "sensor_type": "kv1", "valid": True}]}))
        s = cad.SunRGBDDataset(m).read(0)
        rgb = want if want.ndim == 3 else np.repeat(want[..., None], 3, axis=2)
        assert np.array_equal(s["rgb"], rgb), name
