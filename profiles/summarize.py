"""Summarise rocprofv3 CSV output of profiles/collect.sh into committed files:
  profiles/<tag>_kernel_stats.md   per-kernel time table (from --kernel-trace --stats)
  profiles/<tag>_bench_profiled.json  the bench line printed under the profiler
  profiles/pmc_traffic.json        per-kernel HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE
                                   passes, corrected as MI355X_MICROARCH.md §HBM prescribes:
                                   FETCH_SIZE (KB) reads half the bytes of 16-B/lane streaming loads
                                   on gfx950 -> x2; WRITE_SIZE (KB) exact for 16-B stores.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def find(d, pat):
    hits = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return hits[0] if hits else None


def pmc(d, counter):
    path = find(d, "*counter_collection.csv")
    vals = defaultdict(list)
    if not path:
        return vals
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if row.get("Counter_Name") == counter:
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def main():
    out, tag = sys.argv[1], sys.argv[2]
    here = os.path.dirname(os.path.abspath(__file__))
    stats = find(os.path.join(out, "trace"), "*kernel_stats.csv")
    lines = []
    if stats:
        with open(stats) as fh:
            rows = list(csv.DictReader(fh))
        rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        lines.append(f"# rocprofv3 --kernel-trace --stats: bench.py --steps 3 --warmup 1 ({tag})\n")
        lines.append("| kernel | calls | total ms | avg us | % |")
        lines.append("|---|---|---|---|---|")
        for r in rows:
            lines.append(f"| `{r['Name'][:110]}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                         f"{float(r['AverageNs']) / 1e3:.1f} | {100 * float(r['TotalDurationNs']) / tot:.1f} |")
        with open(os.path.join(here, f"{tag}_kernel_stats.md"), "w") as fh:
            fh.write("\n".join(lines) + "\n")
    for name in ("trace", "fetch", "write"):
        p = os.path.join(out, f"{name}.json")
        if os.path.exists(p) and os.path.getsize(p):
            with open(p) as fh:
                txt = fh.read().strip().splitlines()
            if txt:
                with open(os.path.join(here, f"{tag}_bench_{name}_profiled.json"), "w") as fo:
                    fo.write(txt[-1] + "\n")
    fetch = pmc(os.path.join(out, "fetch"), "FETCH_SIZE")
    write = pmc(os.path.join(out, "write"), "WRITE_SIZE")
    traffic = {}
    for k in set(fetch) | set(write):
        f = fetch.get(k, [])
        w = write.get(k, [])
        if not f or not w:
            continue
        fa, wa = sum(f) / len(f), sum(w) / len(w)
        traffic[k] = {"launches": len(f), "fetch_kb_avg": fa, "write_kb_avg": wa,
                      "hbm_bytes_per_launch": round((2 * fa + wa) * 1024)}
    if traffic:
        with open(os.path.join(here, "pmc_traffic.json"), "w") as fh:
            json.dump(traffic, fh, indent=1, sort_keys=True)
    print(f"stats rows: {len(lines)}; pmc kernels: {len(traffic)}")


if __name__ == "__main__":
    main()
