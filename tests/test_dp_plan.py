"""Data-parallel plumbing on the CPU (no GPU): the flat-gradient layout of every model family and the
decoder-first bucket plan the RCCL exchange uses (cad_model_grad_layout / cad_plan_grad_buckets in
libcad_hip.so, host-only entry points), checked against the invariants the overlapped all-reduce
relies on (csrc/host/dp.cpp), and against the Python GradBucketer (model.py)."""
import ctypes as C

import pytest

MODELS = {0: ("baseline", 31037633), 1: ("film", 32860737), 2: ("rayfilm", 32862465)}


def _layout(lib, model, f=64):
    ns = C.c_int()
    off, cnt = (C.c_int64 * 16)(), (C.c_int64 * 16)()
    nf = C.c_int64()
    assert lib.cad_model_grad_layout(model, 3, f, C.byref(ns), off, cnt, C.byref(nf)) == 0
    return [(off[i], cnt[i]) for i in range(ns.value)], nf.value


def _plan(lib, stages, bucket_elems):
    n = len(stages)
    so = (C.c_int64 * n)(*[o for o, _ in stages])
    sc = (C.c_int64 * n)(*[c for _, c in stages])
    bo, bc, bl = (C.c_int64 * n)(), (C.c_int64 * n)(), (C.c_int * n)()
    nb = lib.cad_plan_grad_buckets(so, sc, n, bucket_elems, bo, bc, bl)
    assert nb > 0
    return [(bo[i], bc[i], bl[i]) for i in range(nb)]


@pytest.mark.parametrize("model", list(MODELS))
def test_grad_layout_stages(cad, model):
    lib = cad.load_library()
    stages, n_flat = _layout(lib, model)
    assert len(stages) == 10   # head, dec1..dec4, bottleneck, enc4..enc1
    # backward order = strictly decreasing, disjoint slices of the slab, all inside it
    for (a, na), (b, nb) in zip(stages, stages[1:]):
        assert b + nb <= a
    assert stages[-1][0] == 0 and stages[0][0] + stages[0][1] <= n_flat
    # the slab holds every parameter (plus alignment padding and enc1.conv1's zero input channel)
    assert sum(c for _, c in stages) >= MODELS[model][1]


@pytest.mark.parametrize("bucket_mb", [1, 25, 100, 1000])
def test_bucket_plan_covers_slab_decoder_first(cad, bucket_mb):
    lib = cad.load_library()
    stages, _ = _layout(lib, 0)
    elems = int(bucket_mb * (1 << 20) / 4)
    buckets = _plan(lib, stages, elems)
    # contiguous, decreasing, non-overlapping buckets whose union is the union of the stages
    lo = min(o for o, _ in stages)
    hi = max(o + c for o, c in stages)
    assert buckets[0][0] + buckets[0][1] == hi and buckets[-1][0] == lo
    for (a, na, la), (b, nb, lb) in zip(buckets, buckets[1:]):
        assert b + nb == a and lb > la
    # every bucket but the last reaches the size target; the last closes at the last stage
    assert all(c >= elems for _, c, _ in buckets[:-1])
    assert buckets[-1][2] == len(stages) - 1
    # a bucket is launched as soon as its last stage is enqueued: decoder stages come first
    assert buckets[0][2] <= 4 or bucket_mb >= 100


def test_bucket_plan_matches_python_bucketer(cad):
    """The C ABI plan (used by build/train and cad_unet_backward_allreduce) and the Python
    GradBucketer (model.py, used by bench.py / Trainer over torch.distributed) cut the same buckets."""
    lib = cad.load_library()
    stages, _ = _layout(lib, 0)
    elems = int(25 * (1 << 20) / 4)
    from cad_amd.model import GradBucketer
    bk = GradBucketer(None, len(stages), elems)
    bk.flush = lambda: (bk.buckets.append((bk.lo, bk.hi)), setattr(bk, "lo", None), setattr(bk, "hi", None))
    for s, (o, c) in enumerate(stages):
        bk.on_stage(s, o, c)
    assert [(o, o + c) for o, c, _ in _plan(lib, stages, elems)] == bk.buckets


def test_bucket_plan_rejects_bad_input(cad):
    lib = cad.load_library()
    so = (C.c_int64 * 2)(10, 0)
    sc = (C.c_int64 * 2)(5, -1)
    assert lib.cad_plan_grad_buckets(so, sc, 2, 4, None, None, None) == -1
    assert lib.cad_plan_grad_buckets(so, sc, 0, 4, None, None, None) == -1


def _resunet_layout(lib):
    ns, nf = C.c_int(), C.c_int64()
    off, cnt = (C.c_int64 * 32)(), (C.c_int64 * 32)()
    assert lib.cad_resunet_grad_layout(C.byref(ns), off, cnt, C.byref(nf)) == 0, lib.cad_last_error()
    return [(off[i], cnt[i]) for i in range(ns.value)], nf.value


def _geonet_layout(cad, lib, variant, f, pcl=1, att=1):
    from cad_amd._abi import GeoNetDesc
    d = GeoNetDesc(variant, 3, f, 4, 10.0, pcl, att, 1, 64, 64)
    ns, nf = C.c_int(), C.c_int64()
    off, cnt = (C.c_int64 * 16)(), (C.c_int64 * 16)()
    assert lib.cad_geonet_grad_layout(C.byref(d), C.byref(ns), off, cnt, C.byref(nf)) == 0, lib.cad_last_error()
    return [(off[i], cnt[i]) for i in range(ns.value)], nf.value


@pytest.mark.parametrize("family", ["resunet", "geo_full", "geo_light", "geo_rays_only"])
def test_other_families_stage_layout_and_plan(cad, family):
    """configs[4]'s ResNet-50 + U-Net decoder and the geometry-aware networks exchange gradients the
    same way (cad_resunet_backward_allreduce / cad_geonet_backward_allreduce, dp.cpp): their staged
    backward writes strictly decreasing, disjoint slab ranges that cover every parameter, so every
    bucket of the plan is final once its last stage is enqueued."""
    lib = cad.load_library()
    if family == "resunet":
        stages, n_flat = _resunet_layout(lib)
        assert len(stages) == 1 + 5 + 16 + 1   # head, dec0..dec4, 16 bottlenecks, stem
        n_params = 40918977
    else:
        variant, f, pcl, att = {"geo_full": (0, 64, 1, 1), "geo_light": (1, 32, 1, 1),
                                "geo_rays_only": (0, 16, 0, 0)}[family]
        stages, n_flat = _geonet_layout(cad, lib, variant, f, pcl, att)
        nl = 6 if variant == 0 else 5
        assert len(stages) == 1 + (nl - 1) + (nl - 1) + 1
        n_params = {"geo_full": 129070759}.get(family)
    for (a, na), (b, nb) in zip(stages, stages[1:]):
        assert 0 <= a - (b + nb) < 64
    assert stages[-1][0] == 0 and stages[0][0] + stages[0][1] <= n_flat
    if n_params:
        assert sum(c for _, c in stages) >= n_params
    for mb in (1, 25):
        elems = int(mb * (1 << 20) / 4)
        buckets = _plan(lib, stages, elems)
        assert buckets[0][0] + buckets[0][1] == stages[0][0] + stages[0][1] and buckets[-1][0] == 0
        for (a, na, la), (b, nb, lb) in zip(buckets, buckets[1:]):   # adjacent up to the 64-float alignment
            assert 0 <= a - (b + nb) < 64 and lb > la
        assert all(c >= elems for _, c, _ in buckets[:-1]) and buckets[-1][2] == len(stages) - 1
