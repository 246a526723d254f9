#!/usr/bin/env python3
"""Condense rocprofv3 CSVs from tools/profile.sh into the files committed under profiles/.

Reads gpurun_out/prof_stats (kernel-trace --stats), gpurun_out/prof_fetch and prof_write (one
PMC counter per pass) and writes, into gpurun_out/profiles_<tag>/:
  rocprof_<tag>_kernel_stats.csv   the rocprofv3 --stats summary, as produced
  rocprof_<tag>_summary.md         per-kernel averages + HBM bytes per fill launch
  pmc_traffic.json                 {workload: {"hbm_bytes_per_launch": ..}} read by bench.py
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE counts half the bytes of a wide streaming read, so it is doubled; WRITE_SIZE is exact
for 16-byte-per-lane streaming stores (what the fill kernel issues).
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil


def is_fill(name):
    return re.search(r"fill(_x2)?_kernel", name) is not None

OUT = "gpurun_out"


def find(pattern):
    hits = sorted(glob.glob(os.path.join(OUT, pattern), recursive=True))
    return hits[0] if hits else None


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def col(row, *cands):
    for c in cands:
        for k in row:
            if k.lower() == c.lower():
                return row[k]
    raise KeyError(f"none of {cands} in {list(row)}")


def counters(path, counter):
    """{kernel name: [per-dispatch values]} for one counter."""
    out = {}
    for r in rows(path):
        if col(r, "Counter_Name") != counter:
            continue
        name = col(r, "Kernel_Name")
        out.setdefault(name, []).append(float(col(r, "Counter_Value")))
    return out


def short(name):
    return name.split("(")[0][:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    a = ap.parse_args()
    dst = os.path.join(OUT, f"profiles_{a.tag}")
    os.makedirs(dst, exist_ok=True)
    stats = find("prof_stats/**/*kernel_stats.csv")
    fetch = find("prof_fetch/**/*counter_collection.csv")
    write = find("prof_write/**/*counter_collection.csv")
    bench = json.load(open(os.path.join(OUT, "bench_prof.json")))
    workload = bench["config"]["workload"]
    lines = [f"# rocprofv3 summary ({a.tag}) — workload {workload}", "",
             f"bench line under the profiler: value {bench['value']} GCUPS, fill {bench['fill_ms']} ms "
             f"(HIP events, {bench['roofline']['avg_launch_ms']} ms per fill launch)", ""]
    shutil.copy(stats, os.path.join(dst, f"rocprof_{a.tag}_kernel_stats.csv"))
    lines += ["## kernel-trace --stats", "", "| kernel | calls | avg ms | total ms | % |", "|---|---|---|---|---|"]
    fill_avg_ns = None
    for r in rows(stats):
        name = col(r, "Name", "KernelName", "Kernel_Name")
        avg = float(col(r, "AverageNs")) / 1e6
        lines.append(f"| `{short(name)}` | {col(r, 'Calls')} | {avg:.3f} | {float(col(r, 'TotalDurationNs')) / 1e6:.3f} | "
                     f"{float(col(r, 'Percentage')):.1f} |")
        if is_fill(name):   # the busiest fill variant (the other one's launches return at once)
            fill_avg_ns = max(fill_avg_ns or 0.0, float(col(r, "AverageNs")))
    lines.append("")
    traffic = None
    if fetch and write:
        f = counters(fetch, "FETCH_SIZE")
        w = counters(write, "WRITE_SIZE")
        lines += ["## HBM traffic per dispatch (PMC, separate passes)", "",
                  "| kernel | FETCH_SIZE KiB (raw) | WRITE_SIZE KiB | HBM bytes (2xFETCH + WRITE) |", "|---|---|---|---|"]
        for name in sorted(set(f) | set(w)):
            fv = sum(f.get(name, [0])) / max(len(f.get(name, [1])), 1)
            wv = sum(w.get(name, [0])) / max(len(w.get(name, [1])), 1)
            hbm = (2 * fv + wv) * 1024
            lines.append(f"| `{short(name)}` | {fv:.0f} | {wv:.0f} | {hbm:.4g} |")
            if is_fill(name):
                traffic = max(traffic or 0.0, hbm)
        lines.append("")
    if traffic is not None:
        cells = bench["config"]["pairs_per_gpu"] * bench["config"]["m"] * bench["config"]["n"]
        lines += [f"fill kernel: {traffic / cells:.4f} HBM bytes per cell measured vs "
                  f"{bench['roofline']['bytes_per_cell']} algorithmic (2 traceback bits / cell + end-cell snapshots)", ""]
        if fill_avg_ns:
            lines.append(f"fill kernel average duration (rocprofv3): {fill_avg_ns / 1e6:.3f} ms; "
                         f"HBM rate {traffic / (fill_avg_ns * 1e-9) / 1e9:.1f} GB/s")
        json.dump({workload: {"hbm_bytes_per_launch": traffic, "source": f"profiles/rocprof_{a.tag}_summary.md"}},
                  open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    open(os.path.join(dst, f"rocprof_{a.tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
