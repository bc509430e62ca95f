"""Step-level A/B on one box: alternate bench.py runs of one workload under two environments (a tuning
switch, or CAD_LIB=<variant build>) so both arms see the same box, clock and thermal history.
  python tools/ab_step.py --config 4 --a CAD_BNPOOL=0 --b CAD_BNPOOL=1 --reps 2 [--steps 10]
Prints one JSON line per run and a summary (median ms/step per arm, B/A)."""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=4)
ap.add_argument("--a", default="", help="VAR=value[,VAR=value] of arm A")
ap.add_argument("--b", default="", help="VAR=value[,VAR=value] of arm B")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--extra", default="", help="more bench.py arguments")
ap.add_argument("--c5", action="store_true", help="time configs[4]'s per-GPU step (profiles/c5_step.py) instead")
args = ap.parse_args()


def env_of(spec):
    e = dict(os.environ)
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=", 1)
        e[k] = v
    return e


res = {"A": [], "B": []}
for rep in range(args.reps):
    for arm, spec in (("A", args.a), ("B", args.b)) if rep % 2 == 0 else (("B", args.b), ("A", args.a)):
        if args.c5:
            cmd = [sys.executable, os.path.join(ROOT, "profiles", "c5_step.py"), "--steps", str(args.steps), "--warmup", "3",
                   *args.extra.split()]
        else:
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", str(args.config), "--steps",
                   str(args.steps), "--warmup", "3", "--no-cpu-baseline", "--no-extra", *args.extra.split()]
        r = subprocess.run(cmd, capture_output=True, text=True, env=env_of(spec), timeout=600)
        if r.returncode != 0:
            print(json.dumps({"arm": arm, "spec": spec, "error": r.stderr[-2000:]}), flush=True)
            sys.exit(1)
        d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
        g = (d.get("roofline") or {}).get("all_gemm_kernels") or {}
        out = {"arm": arm, "spec": spec, "rep": rep, "value": d.get("value", d.get("images_per_s")),
               "ms_per_step": d["ms_per_step"], "gemm_ms": g.get("ms_per_step"), "loss": d.get("last_loss")}
        res[arm].append(out)
        print(json.dumps(out), flush=True)
ma = statistics.median(r["ms_per_step"] for r in res["A"])
mb = statistics.median(r["ms_per_step"] for r in res["B"])
print(json.dumps({"summary": True, "A": args.a, "B": args.b, "ms_A": ma, "ms_B": mb, "B_over_A": mb / ma}), flush=True)
