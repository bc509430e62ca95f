"""Checkpoint compatibility with the reference's torch::save(model_, path)
(tensorboard_trainer_enhanced.h:656-662), on the CPU: libcad's host-only archive writer/reader
(csrc/host/torch_archive.cpp) against LibTorch itself, driven through the reference's model code
compiled in this container (oracle/_ref/ref_harness --mode save|load, torch::save / torch::load).

* writer: for the same weights, data.pkl, every class source and every storage record are
  byte-identical to the archive LibTorch writes (all three model families);
* the reference reads ours: torch::load(model, our.pt) restores every parameter and buffer bit for bit
  (num_batches_tracked included);
* we read the reference's: every tensor of a LibTorch archive, bit for bit;
* PyTorch's own torch.jit.load accepts our archive (an independent reader);
* malformed files fail with an error, never a crash.
The GPU side (cad_unet_save_torch / load_torch on a live model) is in test_gpu_checkpoint.py."""
import ctypes as C
import json
import os
import subprocess
import zipfile

import numpy as np
import pytest
import torch

from conftest import ROOT

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
F = 4


@pytest.fixture(scope="module")
def harness():
    if not os.path.exists(HARNESS):
        pytest.skip("oracle/_ref/ref_harness not built (needs /root/reference; make -C oracle)")
    return HARNESS


def _run(harness, *args):
    subprocess.run([harness, "--threads", "1", *map(str, args)], check=True, capture_output=True, timeout=300)


def _dump(d):
    man = json.load(open(os.path.join(d, "manifest.json")))
    raw = np.fromfile(os.path.join(d, "tensors.bin"), dtype=np.float32)
    return {t["name"]: raw[t["offset"]:t["offset"] + int(np.prod(t["shape"] or [1]))].reshape(t["shape"])
            for t in man["tensors"]}


POOLED = ("enc2.", "enc3.", "enc4.", "bottleneck.")


def _entries(cad, params, buffers, nbt=0, nbt_film=0):
    """cad_archive_entry list in the order cad_unet_save_torch builds it (cad_api.cpp): parameters in
    named_parameters() order with each encoder block's MaxPool2d declared before its DoubleConv,
    then buffers with num_batches_tracked after each running_var."""
    from cad_amd._abi import ArchiveEntry
    keep, ents = [], []

    def add(name, kind, arr=None):
        e = ArchiveEntry()
        e.name = name.encode()
        e.kind = kind
        if arr is not None:
            arr = np.require(arr, requirements="C")   # (ascontiguousarray would make a 0-d array 1-d)
            keep.append(arr)
            e.dtype = 1 if arr.dtype == np.int64 else 0
            e.ndim = arr.ndim
            for k, s in enumerate(arr.shape):
                e.shape[k] = s
            e.data = arr.ctypes.data
        ents.append(e)

    placed = set()
    for n, v in params.items():
        for p in POOLED:
            if p not in placed and n.startswith(p + "conv."):
                add(p + "pool", 2)
                placed.add(p)
        add(n, 0, np.asarray(v, np.float32))
    for n, v in buffers.items():
        add(n, 1, np.asarray(v, np.float32))
        if n.endswith(".running_var"):
            add(n[:-len("running_var")] + "num_batches_tracked", 1,
                np.array(nbt_film if ".film." in n else nbt, np.int64))
    arr = (ArchiveEntry * len(ents))(*ents)
    return arr, keep


def _write(cad, path, params, buffers, **kw):
    arr, keep = _entries(cad, params, buffers, **kw)
    lib = cad.load_library()
    assert lib.cad_archive_write(str(path).encode(), arr, len(arr)) == 0, lib.cad_last_error()


def _members(path):
    z = zipfile.ZipFile(path)
    pre = z.namelist()[0].split("/")[0]
    return {n[len(pre) + 1:]: z.read(n) for n in z.namelist()}


@pytest.mark.parametrize("model", ["baseline", "film", "rayfilm"])
def test_writer_byte_identical_to_libtorch(cad, oracle, harness, tmp_path, model):
    ref = tmp_path / "ref.pt"
    _run(harness, "--mode", "save", "--model", model, "--init", "synth", "--f", F, "--steps", 0, "--ckpt", ref,
         "--out", tmp_path)
    ours = tmp_path / "ours.pt"
    _write(cad, ours, oracle.synth_init(F, model=model), oracle.init_buffers(F, model=model))
    a, b = _members(ref), _members(ours)
    ref_names = {n for n in a if not n.endswith(".debug_pkl") and n != ".data/serialization_id"}
    assert ref_names == {n for n in b if n != ".data/serialization_id"}
    assert a["data.pkl"] == b["data.pkl"]
    for n in ref_names:
        assert a[n] == b[n], n


@pytest.mark.parametrize("model", ["baseline", "rayfilm"])
def test_reference_torch_load_reads_ours(cad, oracle, harness, tmp_path, model):
    g = torch.Generator().manual_seed(3)
    params = {n: torch.randn(v.shape, generator=g) for n, v in oracle.synth_init(F, model=model).items()}
    bufs = {n: (torch.rand(v.shape, generator=g) + (0.5 if n.endswith("var") else 0.0))
            for n, v in oracle.init_buffers(F, model=model).items()}
    ours = tmp_path / "ours_epoch_3.pt"
    _write(cad, ours, params, bufs, nbt=7, nbt_film=5)
    _run(harness, "--mode", "load", "--model", model, "--f", F, "--ckpt", ours, "--out", tmp_path)
    got = _dump(tmp_path)
    for n, v in params.items():
        assert np.array_equal(got["param." + n], v.numpy()), n
    for n, v in bufs.items():
        assert np.array_equal(got["buffer." + n], v.numpy()), n
    nbt = {n: int(v) for n, v in got.items() if n.endswith("num_batches_tracked")}
    assert nbt and all(v == (5 if ".film." in n else 7) for n, v in nbt.items())


def _read_all(cad, path):
    lib = cad.load_library()
    h = C.c_void_p()
    assert lib.cad_archive_open(str(path).encode(), C.byref(h)) == 0, lib.cad_last_error()
    out = {}
    try:
        for i in range(lib.cad_archive_count(h)):
            name, dt, nd = C.c_char_p(), C.c_int(), C.c_int()
            shp = (C.c_int64 * 8)()
            assert lib.cad_archive_info(h, i, C.byref(name), C.byref(dt), C.byref(nd), shp) == 0
            npdt = {0: np.float32, 1: np.int64}[dt.value]
            a = np.empty([shp[k] for k in range(nd.value)], npdt)
            assert lib.cad_archive_read(h, i, a.ctypes.data, a.nbytes) == 0, lib.cad_last_error()
            out[name.value.decode()] = a
    finally:
        lib.cad_archive_close(h)
    return out


@pytest.mark.parametrize("model", ["baseline", "film"])
def test_reader_reads_libtorch_archive(cad, harness, tmp_path, model):
    ref = tmp_path / "ref.pt"
    # default (LibTorch) init, two training steps: running statistics and counters are not defaults
    _run(harness, "--mode", "save", "--model", model, "--f", F, "--B", 2, "--H", 32, "--W", 32, "--steps", 2,
         "--ckpt", ref, "--out", tmp_path)
    want = _dump(tmp_path)
    got = _read_all(cad, ref)
    assert set(got) == {n.split(".", 1)[1] for n in want}
    for n, v in want.items():
        g = got[n.split(".", 1)[1]]
        assert g.shape == v.shape and np.array_equal(g.astype(np.float32), v), n
    assert all(int(v) == 2 for n, v in got.items() if n.endswith("num_batches_tracked") and ".film." not in n)


def test_committed_reference_checkpoint_readable(cad):
    """tests/golden/ckpt_baseline_f4: an archive the reference's torch::save wrote (oracle/gen_golden.py);
    the GPU test loads it into the model."""
    got = _read_all(cad, os.path.join(ROOT, "tests", "golden", "ckpt_baseline_f4", "baseline_unet_epoch_1.pt"))
    assert len([n for n in got if n.endswith("num_batches_tracked")]) == 18
    assert got["enc1.conv1.weight"].shape == (4, 3, 3, 3) and got["out_conv.bias"].shape == (1,)


def test_pytorch_jit_load_reads_ours(cad, oracle, tmp_path):
    params, bufs = oracle.synth_init(F), oracle.init_buffers(F)
    ours = tmp_path / "ours.pt"
    _write(cad, ours, params, bufs, nbt=4)
    m = torch.jit.load(str(ours))
    sd = m.state_dict()
    for n, v in params.items():
        assert torch.equal(sd[n], v), n
    assert int(sd["enc3.conv.bn2.num_batches_tracked"]) == 4
    assert [n for n, _ in m.named_parameters()] == list(params)


def test_reader_rejects_malformed(cad, tmp_path):
    lib = cad.load_library()
    h = C.c_void_p()
    junk = tmp_path / "junk.pt"
    junk.write_bytes(b"not a zip archive at all" * 10)
    assert lib.cad_archive_open(str(junk).encode(), C.byref(h)) != 0
    assert b"zip" in lib.cad_last_error()
    assert lib.cad_archive_open(str(tmp_path / "missing.pt").encode(), C.byref(h)) != 0
    # a zip without data.pkl
    z = tmp_path / "other.zip"
    with zipfile.ZipFile(z, "w") as f:
        f.writestr("x/readme.txt", "hello")
    assert lib.cad_archive_open(str(z).encode(), C.byref(h)) != 0
    assert b"data.pkl" in lib.cad_last_error()
    # truncated pickle
    with zipfile.ZipFile(z, "w") as f:
        f.writestr("x/data.pkl", b"\x80\x02}q\x00(X\x01\x00")
    assert lib.cad_archive_open(str(z).encode(), C.byref(h)) != 0
    # a pickle calling something: never executed, the object is just not a tensor -> no tensors
    with zipfile.ZipFile(z, "w") as f:
        f.writestr("x/data.pkl", b"\x80\x02cos\nsystem\nq\x00X\x04\x00\x00\x00trueq\x01\x85q\x02Rq\x03.")
    assert lib.cad_archive_open(str(z).encode(), C.byref(h)) == 0
    assert lib.cad_archive_count(h) == 0
    lib.cad_archive_close(h)


def _pkl_str(s):
    b = s.encode()
    return b"X" + len(b).to_bytes(4, "little") + b


def _tensor_pkl(offset, sizes, strides):
    """data.pkl of {'w': _rebuild_tensor_v2(storage '0' FloatStorage, offset, sizes, strides, False)}."""
    def ints(v):
        return b"(" + b"".join(b"J" + int(x).to_bytes(4, "little", signed=True) for x in v) + b"t"
    return (b"\x80\x02}" + _pkl_str("w") + b"ctorch._utils\n_rebuild_tensor_v2\n(" +
            b"(" + _pkl_str("storage") + b"ctorch\nFloatStorage\n" + _pkl_str("0") + _pkl_str("cpu") + b"K\x10tQ" +
            b"J" + int(offset).to_bytes(4, "little", signed=True) + ints(sizes) + ints(strides) + b"\x89tRs.")


def _dag_pkl(levels=60):
    """data.pkl of a dict tree whose every level holds the previous level's (memoised) dict twice: a
    DAG, not a cycle, with 2^levels root-to-leaf paths."""
    out = b"\x80\x02}q\x00"
    for k in range(1, levels + 1):
        out += b"}q" + bytes([k]) + b"(" + _pkl_str("a") + b"h" + bytes([k - 1]) + _pkl_str("b") + b"h" + bytes([k - 1]) + b"u"
    return out + b"."


@pytest.mark.parametrize("what,pkl,msg", [
    ("memoised dict shared twice per level (DAG, 2^60 paths)", _dag_pkl(), b"too large"),
    ("BINUNICODE8 length that wraps pos + n", b"\x80\x02\x8d" + (2 ** 64 - 1).to_bytes(8, "little") + b"abc.",
     b"truncated"),
    ("BINUNICODE8 length past the end", b"\x80\x02\x8d" + (1 << 40).to_bytes(8, "little") + b"abc.", b"truncated"),
    ("dict that contains itself through the memo", b"\x80\x02}q\x00" + _pkl_str("a") + b"h\x00s.", b"self-referencing"),
    ("strides shorter than sizes", _tensor_pkl(0, [2, 2], [2]), b"rank"),
    ("negative size", _tensor_pkl(0, [-2, 2], [2, 1]), b"bad size"),
    ("negative storage offset", _tensor_pkl(-5, [2, 2], [2, 1]), b"negative storage offset"),
    ("storage record too small", _tensor_pkl(14, [2, 2], [2, 1]), b"too small"),
])
def test_reader_rejects_hostile_pickles(cad, tmp_path, what, pkl, msg):
    """the .pt reader (cad_archive_open, used by --resume and load) bounds-checks every
    length and index taken from the file: wrapped lengths, cyclic module trees and inconsistent tensor
    records end in a clean error, never an out-of-bounds read or unbounded recursion."""
    lib = cad.load_library()
    z = tmp_path / "bad.pt"
    with zipfile.ZipFile(z, "w") as f:
        f.writestr("bad/data.pkl", pkl)
        f.writestr("bad/data/0", np.zeros(16, np.float32).tobytes())
    h = C.c_void_p()
    assert lib.cad_archive_open(str(z).encode(), C.byref(h)) != 0, what
    assert msg in lib.cad_last_error(), (what, lib.cad_last_error())


def test_reader_accepts_the_well_formed_twin(cad, tmp_path):
    """The hand-built record of test_reader_rejects_hostile_pickles, made consistent, reads back."""
    lib = cad.load_library()
    z = tmp_path / "ok.pt"
    with zipfile.ZipFile(z, "w") as f:
        f.writestr("ok/data.pkl", _tensor_pkl(4, [2, 3], [3, 1]))
        f.writestr("ok/data/0", np.arange(16, dtype=np.float32).tobytes())
    h = C.c_void_p()
    assert lib.cad_archive_open(str(z).encode(), C.byref(h)) == 0, lib.cad_last_error()
    assert lib.cad_archive_count(h) == 1
    out = np.empty(6, np.float32)
    assert lib.cad_archive_read(h, 0, out.ctypes.data_as(C.c_void_p), out.nbytes) == 0
    assert np.array_equal(out, np.arange(4, 10, dtype=np.float32))
    lib.cad_archive_close(h)
