"""The loader's host side on the CPU (csrc/host/dataset.cpp; SunRGBDLoader, sunrgbd_loader.cpp):
the JSON manifest reader against the reference's own manifest (tests/golden/manifest, copied from the
reference's data/manifest), its filters (valid, sensor type, intrinsics.txt present), file discovery,
and the PNG / PNM decoders against PIL on images of every colour type, bit depth and scanline filter
the reader supports.  Parity with cv::imread is restated, not run (OpenCV is absent): IMREAD_COLOR
-> RGB u8 (gray replicated, alpha dropped, 16-bit -> high byte), IMREAD_UNCHANGED depth 16-bit ->
value / 1000 m.  The prefetch ring on the device is tested in test_gpu_loader.py."""
import json
import os
import zlib
import struct

import numpy as np
import pytest

from conftest import ROOT

PIL = pytest.importorskip("PIL.Image")
MANIFEST = os.path.join(ROOT, "tests", "golden", "manifest", "sunrgbd_manifest.json")


def _tree(tmp, manifest, with_intrinsics, rgb_ext=".png", depth_ext=".png", size=(48, 64), seed=0):
    """Materialise the sample directories of `manifest` (paths relative to `tmp`, the cwd)."""
    rng = np.random.default_rng(seed)
    H, W = size
    out = []
    for k, im in enumerate(manifest["images"]):
        d = tmp / im["path"]
        (d / "image").mkdir(parents=True, exist_ok=True)
        (d / "depth").mkdir(parents=True, exist_ok=True)
        rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        dep = rng.integers(0, 10000, (H + k, W + 2 * k), dtype=np.uint16)
        if rgb_ext == ".png":
            PIL.fromarray(rgb).save(d / "image" / f"img_{k}.png")
        else:
            PIL.fromarray(rgb).save(d / "image" / f"img_{k}.ppm")
        if depth_ext == ".png":
            PIL.fromarray(dep).save(d / "depth" / f"d_{k}.png")
        else:
            (d / "depth" / f"d_{k}.pgm").write_bytes(f"P5\n{dep.shape[1]} {dep.shape[0]}\n65535\n".encode()
                                                     + dep.astype(">u2").tobytes())
        K = [500.0 + k, 0, 320.5, 0, 501.25 + k, 240.0, 0, 0, 1]
        if with_intrinsics(k):
            (d / "intrinsics.txt").write_text(" ".join(f"{v:.6f}" for v in K[:3]) + "\n" +
                                               " ".join(f"{v:.6f}" for v in K[3:6]) + "\n" +
                                               " ".join(f"{v:.6f}" for v in K[6:]) + "\n")
        out.append((rgb, dep, np.array(K, np.float32).reshape(3, 3)))
    return out


def test_reference_manifest_parses(cad, tmp_path, monkeypatch):
    man = json.load(open(MANIFEST))
    monkeypatch.chdir(tmp_path)
    data = _tree(tmp_path, man, with_intrinsics=lambda k: k != 2)   # realsense entry has no intrinsics.txt
    ds = cad.SunRGBDDataset(MANIFEST)
    kept = [0, 1, 3]
    assert len(ds) == 3
    assert [ds.image_dir(i) for i in range(3)] == [man["images"][k]["path"] for k in kept]
    for i, k in enumerate(kept):
        s = ds.read(i)
        rgb, dep, K = data[k]
        assert np.array_equal(s["rgb"], rgb) and np.array_equal(s["depth"], dep)
        assert s["depth_scale"] == np.float32(1 / 1000) and np.array_equal(s["K"], K)
    # sensor filter (filterBySensorType) and invalid entries
    assert len(cad.SunRGBDDataset(MANIFEST, ["kv2", "xtion"])) == 2
    man["images"][0]["valid"] = False
    p = tmp_path / "m2.json"
    p.write_text(json.dumps(man, indent=1, ensure_ascii=True))
    assert [cad.SunRGBDDataset(p).image_dir(i) for i in range(2)] == [man["images"][k]["path"] for k in (1, 3)]


def test_raw_pnm_formats(cad, tmp_path, monkeypatch):
    man = json.load(open(MANIFEST))
    monkeypatch.chdir(tmp_path)
    data = _tree(tmp_path, man, with_intrinsics=lambda k: True, rgb_ext=".ppm", depth_ext=".pgm")
    ds = cad.SunRGBDDataset(MANIFEST)
    for i in range(4):
        s = ds.read(i)
        assert np.array_equal(s["rgb"], data[i][0]) and np.array_equal(s["depth"], data[i][1])


def _write_png_filters(path, img, ctype, bits, filters):
    """A PNG whose scanlines use the given filter types in turn (PIL picks its own): covers all five."""
    H, W = img.shape[:2]
    ch = {0: 1, 2: 3, 4: 2, 6: 4}[ctype]
    bpp = ch * bits // 8
    raw = img.astype(">u2").tobytes() if bits == 16 else img.astype(np.uint8).tobytes()
    stride = W * bpp
    rows = [np.frombuffer(raw[y * stride:(y + 1) * stride], np.uint8).astype(np.int32) for y in range(H)]
    out = bytearray()
    for y, row in enumerate(rows):
        ft = filters[y % len(filters)]
        up = rows[y - 1] if y else np.zeros_like(row)
        left = np.concatenate([np.zeros(bpp, np.int32), row[:-bpp]])
        ul = np.concatenate([np.zeros(bpp, np.int32), up[:-bpp]])
        if ft == 0:
            f = row
        elif ft == 1:
            f = row - left
        elif ft == 2:
            f = row - up
        elif ft == 3:
            f = row - (left + up) // 2
        else:
            p = left + up - ul
            pa, pb, pc = abs(p - left), abs(p - up), abs(p - ul)
            pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, up, ul))
            f = row - pred
        out.append(ft)
        out += (f & 255).astype(np.uint8).tobytes()

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    ihdr = struct.pack(">IIBBBBB", W, H, bits, ctype, 0, 0, 0)
    path.write_bytes(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", zlib.compress(bytes(out), 6))
                     + chunk(b"IEND", b""))


def _one_sample(tmp, rgb_file_writer, depth_file_writer):
    d = tmp / "s0"
    (d / "image").mkdir(parents=True)
    (d / "depth").mkdir(parents=True)
    rgb_file_writer(d / "image")
    depth_file_writer(d / "depth")
    (d / "intrinsics.txt").write_text("1 0 2\n0 3 4\n0 0 1\n")
    m = tmp / "m.json"
    m.write_text(json.dumps({"images": [{"path": str(d), "sensor_type": "kv1", "valid": True}]}))
    return m


@pytest.mark.parametrize("ctype,bits", [(0, 8), (0, 16), (2, 8), (2, 16), (4, 8), (6, 8), (6, 16)])
def test_png_decoder_colour_types_and_filters(cad, tmp_path, ctype, bits):
    rng = np.random.default_rng(ctype * 100 + bits)
    ch = {0: 1, 2: 3, 4: 2, 6: 4}[ctype]
    H, W = 23, 37
    img = rng.integers(0, 1 << bits, (H, W, ch)).astype(np.uint16 if bits == 16 else np.uint8)
    dep = rng.integers(0, 65536, (H, W)).astype(np.uint16)
    m = _one_sample(tmp_path, lambda d: _write_png_filters(d / "a.png", img, ctype, bits, [0, 1, 2, 3, 4]),
                    lambda d: _write_png_filters(d / "a.png", dep, 0, 16, [4, 3, 2, 1, 0]))
    s = cad.SunRGBDDataset(m).read(0)
    # imread(IMREAD_COLOR) semantics: gray replicated, alpha dropped, 16-bit -> high byte
    want = img[..., :3] if ch >= 3 else np.repeat(img[..., :1], 3, axis=2)
    if bits == 16:
        want = (want >> 8).astype(np.uint8)
    assert np.array_equal(s["rgb"], want)
    assert np.array_equal(s["depth"], dep) and np.array_equal(s["K"], np.array([[1, 0, 2], [0, 3, 4], [0, 0, 1]], np.float32))


def test_png_palette_and_8bit_depth_and_pil_files(cad, tmp_path):
    rng = np.random.default_rng(7)
    rgb = rng.integers(0, 256, (31, 17, 3), dtype=np.uint8)
    pal = PIL.fromarray(rgb).convert("P", palette=PIL.Palette.ADAPTIVE, colors=40)
    dep8 = rng.integers(0, 256, (31, 17), dtype=np.uint8)
    m = _one_sample(tmp_path, lambda d: pal.save(d / "p.png"), lambda d: PIL.fromarray(dep8).save(d / "d.png"))
    s = cad.SunRGBDDataset(m).read(0)
    assert np.array_equal(s["rgb"], np.asarray(pal.convert("RGB")))
    assert np.array_equal(s["depth"], dep8.astype(np.uint16)) and s["depth_scale"] == 1.0   # 8-bit: metres as-is


def test_loader_errors(cad, tmp_path):
    # a progressive frame decodes as libjpeg-turbo decodes it
    rng = np.random.default_rng(1)
    img = PIL.fromarray(rng.integers(0, 256, (8, 8, 3), dtype=np.uint8))
    m = _one_sample(tmp_path, lambda d: img.save(d / "x.jpg", progressive=True),
                    lambda d: PIL.fromarray(np.zeros((8, 8), np.uint16)).save(d / "d.png"))
    s = cad.SunRGBDDataset(m).read(0)
    assert np.array_equal(s["rgb"], np.asarray(PIL.open(tmp_path / "s0" / "image" / "x.jpg").convert("RGB")))
    # a JPEG the decoder does not implement (a progression cut short, which libjpeg-turbo would
    # block-smooth): a clear message naming the file
    data = (tmp_path / "s0" / "image" / "x.jpg").read_bytes()
    sos = [i for i in range(len(data) - 1) if data[i] == 0xFF and data[i + 1] == 0xDA]
    (tmp_path / "s0" / "image" / "x.jpg").write_bytes(data[:sos[2]] + b"\xff\xd9")
    with pytest.raises(cad.CadError, match="block smoothing.*x.jpg"):
        cad.SunRGBDDataset(m).read(0)
    with pytest.raises(cad.CadError, match="Cannot open manifest"):
        cad.SunRGBDDataset(tmp_path / "nope.json")
    bad = tmp_path / "bad.json"
    for text, msg in [('{"images": [ {"path": "a", }', "JSON error"), ('{"x": 1}', 'no "images"'),
                      ('{"images": [1, 2', "JSON error"), ('{"images": []} junk', "trailing")]:
        bad.write_text(text)
        with pytest.raises(cad.CadError, match=msg):
            cad.SunRGBDDataset(bad)
    # escapes, unicode and nesting the reference manifest does not use
    bad.write_text(json.dumps({"images": [{"path": "dir é\n\"q\"", "sensor_type": "kv1", "valid": True,
                                           "x": [{"y": [None, 1.5e3, -2, True]}]}]}))
    assert len(cad.SunRGBDDataset(bad)) == 0   # parses; the directory has no intrinsics.txt
    ds = cad.SunRGBDDataset.synthetic(3, 40, 56)
    a, b = ds.read(1), ds.read(1)
    assert a["rgb"].shape == (40, 56, 3) and np.array_equal(a["rgb"], b["rgb"]) and a["depth"].max() <= 9500
    with pytest.raises(cad.CadError, match="out of range"):
        ds.read(3)
