"""Summarise rocprofv3 CSV output of profiles/collect.sh into committed files:
  profiles/<tag>_kernel_stats.md   per-kernel time table (from --kernel-trace --stats)
  profiles/<tag>_bench_profiled.json  the bench line printed under the profiler
  profiles/pmc_traffic.json        per-kernel HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE
                                   passes, corrected as MI355X_MICROARCH.md §HBM prescribes:
                                   FETCH_SIZE (KB) reads half the bytes of 16-B/lane streaming loads
                                   on gfx950 -> x2; WRITE_SIZE (KB) exact for 16-B stores.
  profiles/<tag>_sq_counters.md    per-kernel clock under load (GRBM_GUI_ACTIVE / 8 XCDs / duration),
                                   MFMA busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x
                                   active cycles) and the wave-cycle breakdown (SQ_WAIT_ANY parked,
                                   SQ_WAIT_INST_ANY issue-stalled, SQ_ACTIVE_INST_ANY issuing).
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


def durations(d):
    """Kernel_Name -> list of durations (ns) from a pass's kernel trace, if it wrote one."""
    path = find(d, "*kernel_trace.csv")
    out = defaultdict(list)
    if not path:
        return out
    with open(path) as fh:
        for row in csv.DictReader(fh):
            out[row["Kernel_Name"]].append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
    return out


def sq_table(d, tag, here, avg_ns):
    names = ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
             "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_LDS", "SQ_WAIT_INST_LDS", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]
    c = {n: pmc(d, n) for n in names}
    ks = set(c["GRBM_GUI_ACTIVE"])
    if not ks:
        return
    rows = []
    for k in ks:
        avg = {n: (sum(v) / len(v) if v else 0.0) for n, v in ((n, c[n].get(k, [])) for n in names)}
        dur = avg_ns.get(k)
        clk = avg["GRBM_GUI_ACTIVE"] / 8.0 / dur if dur else float("nan")   # GHz (cycles per ns)
        active = avg["GRBM_GUI_ACTIVE"] / 8.0
        mfma = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * active) if active else 0.0
        wc = avg["SQ_WAVE_CYCLES"] or 1.0
        rows.append((dur or 0.0, k, clk, mfma, avg["SQ_WAIT_ANY"] / wc, avg["SQ_WAIT_INST_ANY"] / wc,
                     avg["SQ_ACTIVE_INST_ANY"] / wc, avg["SQ_WAIT_INST_LDS"] / wc))
    rows.sort(key=lambda r: -r[0])
    lines = [f"# rocprofv3 SQ/GRBM pass: bench.py --steps 1 --warmup 0 ({tag})\n",
             "clock = GRBM_GUI_ACTIVE / 8 / avg duration (kernel-trace pass); MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /",
             "(1024 SIMDs x GRBM_GUI_ACTIVE/8); wave-cycle shares: parked (SQ_WAIT_ANY), issue-stalled",
             "(SQ_WAIT_INST_ANY, of which LDS SQ_WAIT_INST_LDS), issuing (SQ_ACTIVE_INST_ANY).\n",
             "| kernel | avg us | clock GHz | MFMA busy | parked | stalled | issuing | LDS-stall |",
             "|---|---|---|---|---|---|---|---|"]
    for dur, k, clk, mfma, wa, wi, ac, wl in rows[:30]:
        lines.append(f"| `{k[:100]}` | {dur / 1e3:.1f} | {clk:.2f} | {mfma:.3f} | {wa:.2f} | {wi:.2f} | {ac:.2f} | {wl:.2f} |")
    with open(os.path.join(here, f"{tag}_sq_counters.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")


def main():
    out, tag = sys.argv[1], sys.argv[2]
    here = os.path.dirname(os.path.abspath(__file__))
    stats = find(os.path.join(out, "trace"), "*kernel_stats.csv")
    lines = []
    avg_ns = {}
    if stats:
        with open(stats) as fh:
            rows = list(csv.DictReader(fh))
        avg_ns = {r["Name"]: float(r["AverageNs"]) for r in rows}
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
    sq_table(os.path.join(out, "sq"), tag, here, avg_ns)
    for name in ("trace", "fetch", "write", "sq"):
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
    if traffic:   # merged: kernel names differ per engine, so several configs share the file —
        # except config 5 (ResNet U-Net), whose kernels share names with the U-Net's at other shapes:
        # its tags ("*_c5*") go to their own file
        path = os.path.join(here, "pmc_traffic_c5.json" if "_c5" in tag else "pmc_traffic.json")
        merged = {}
        if os.path.exists(path):
            with open(path) as fh:
                merged = json.load(fh)
        merged.update(traffic)
        with open(path, "w") as fh:
            json.dump(merged, fh, indent=1, sort_keys=True)
    print(f"stats rows: {len(lines)}; pmc kernels: {len(traffic)}")


if __name__ == "__main__":
    main()
