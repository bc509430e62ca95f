"""Timing lab for the bf16 engine's convolution kernels at the configs[3] shapes (bs32 480x640,
f=64: levels 0-4): each operator launched `reps` times on random bf16 operands (not zeros: the chip
holds a different clock on zeros, MI355X_MICROARCH.md DVFS item 1) and timed with HIP events.
  python tools/winlab.py [--reps 20] [--only fwd|dgrad|wgrad|convT]      (CAD_LIB=libcad_hip_<variant>.so for A/B)"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import cad_pkg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--only", default="")
ap.add_argument("--B", type=int, default=32)
args = ap.parse_args()
cad = cad_pkg.load()
lib = cad.load_library()
assert lib.cad_set_gemm_engine(2) == 0
dev = torch.device("cuda", 0)
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
B, H, W = args.B, 480, 640
# (name, level, cin, cout, kind, epilogue): the U-Net's conv shapes
CASES = []
for l in range(5):
    Cl = 64 << l
    CASES.append((f"enc{l}.conv2", l, Cl, Cl, "fwd", "stats"))
    CASES.append((f"enc{l}.conv2", l, Cl, Cl, "dgrad", "b16"))
    CASES.append((f"enc{l}.conv2", l, Cl, Cl, "wgrad", ""))
for l in range(4):
    Cl = 64 << l
    CASES.append((f"dec{l}.conv1", l, 2 * Cl, Cl, "fwd", "stats"))
    CASES.append((f"dec{l}.conv1", l, 2 * Cl, Cl, "dgrad", "b16"))
for l in range(4):
    Cl = 64 << l
    CASES.append((f"up{l}", l + 1, 2 * Cl, Cl, "convT", ""))
out = []
for name, l, cin, cout, kind, epi in CASES:
    if args.only and kind != args.only:
        continue
    h, w = H >> l, W >> l
    M = B * h * w
    g = torch.Generator(device=dev).manual_seed(l * 7 + cin)
    if kind == "fwd":
        x = torch.randn(M, cin, device=dev, generator=g).bfloat16()
        wt = torch.randn(cout, 3, 3, cin, device=dev, generator=g) * (1.0 / (3 * cin ** 0.5))
        y = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
        call = lambda: lib.cad_op_conv3x3_fwd_bf16(P(x), cin, 0, cin, P(wt), cout, P(y), cout, 0, 1, 1, B, h, w, s)  # noqa
        flop = 2.0 * M * cout * 9 * cin
    elif kind == "dgrad":
        dz = torch.randn(M, cout, device=dev, generator=g).bfloat16()
        wt = torch.randn(cout, 3, 3, cin, device=dev, generator=g) * (1.0 / (3 * cin ** 0.5))
        dx = torch.empty(M, cin, device=dev, dtype=torch.bfloat16)
        call = lambda: lib.cad_op_conv3x3_dgrad_bf16(P(dz), cout, cout, P(wt), cin, P(dx), cin, 1, B, h, w, s)  # noqa
        flop = 2.0 * M * cout * 9 * cin
    elif kind == "convT":
        x = torch.randn(M, cin, device=dev, generator=g).bfloat16()
        wt = torch.randn(cin, 2, 2, cout, device=dev, generator=g) * (1.0 / cin ** 0.5)
        bias = torch.randn(cout, device=dev, generator=g)
        y = torch.empty(4 * M, 2 * cout, device=dev, dtype=torch.bfloat16)
        call = lambda: lib.cad_op_convT_fwd_bf16(P(x), cin, 0, cin, P(wt), P(bias), cout, P(y), 2 * cout, cout, B, h, w, s)  # noqa
        flop = 2.0 * M * 4 * cout * cin
    else:
        dz = torch.randn(M, cout, device=dev, generator=g).bfloat16()
        x = torch.randn(M, cin, device=dev, generator=g).bfloat16()
        dw = torch.empty(cout, 9 * cin, device=dev)
        call = lambda: lib.cad_op_conv3x3_wgrad_bf16(P(dz), cout, cout, P(x), cin, 0, cin, P(dw), B, h, w, s)  # noqa
        flop = 2.0 * M * cout * 9 * cin
    assert call() == 0, lib.cad_last_error()
    lib.cad_profile_reset()
    lib.cad_profile_enable(1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(args.reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    lib.cad_profile_enable(0)
    n = lib.cad_profile_report(None, 0)
    buf = C.create_string_buffer(n)
    lib.cad_profile_report(buf, n)
    prof = json.loads(buf.value.decode())
    gemm = max((r for r in prof if r["gflop"] > 0), key=lambda r: r["ms"])
    kms = gemm["ms"] / gemm["launches"]
    row = {"case": f"{name} {kind}", "level": l, "cin": cin, "cout": cout, "kernel": gemm["name"],
           "kernel_us": round(1e3 * kms, 1), "kernel_tflops": round(gemm["gflop"] / gemm["ms"], 1),
           "op_us": round(1e3 * e0.elapsed_time(e1) / args.reps, 1), "op_tflops": round(flop * args.reps / e0.elapsed_time(e1) / 1e9, 1)}
    out.append(row)
    print(json.dumps(row), flush=True)
    del call
tot = sum(r["kernel_us"] for r in out)
print(json.dumps({"lib": os.environ.get("CAD_LIB", "libcad_hip.so"), "sum_kernel_us": round(tot, 1)}), flush=True)
