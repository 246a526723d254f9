#!/usr/bin/env python3
"""Pipelined-headline kernel timeline from a rocprofv3 --kernel-trace run of bench.py (or any run of
pipelined align_device calls): per fill launch, how long after the previous call's fill-stream work
(fill + end-cell replay + the int32 variant's no-op launches) it started, and where that call's
alphabet scan and T16 decision ran.  Answers "does the scan of call k+1, queued behind fill k, delay
fill k+1?" (VERDICT r05 item 5).

    python tools/pipe_trace.py gpurun_out/<dir> [--fill fill_so]
"""
import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--fill", default="fill_so", help="substring of the headline fill kernel's name")
    a = ap.parse_args()
    ev = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")))
    ev.sort()
    fills = [e for e in ev if a.fill in e[2] and "endcell" not in e[2]]
    scans = [e for e in ev if "alphabet_scan" in e[2]]
    decides = [e for e in ev if "decide_t16" in e[2]]
    endcells = [e for e in ev if "endcell_so" in e[2]]
    tot = sum(e[1] - e[0] for e in ev)
    rows = []
    for k in range(1, len(fills)):
        f0, f1 = fills[k - 1], fills[k]
        # the previous call's fill-stream work ends at its end-cell replay (or later no-op launches)
        prev_end = max([f0[1]] + [e[1] for e in endcells if f0[1] <= e[0] < f1[0]])
        sc = [s for s in scans if f0[0] <= s[0] <= f1[0]]
        dc = [d for d in decides if f0[0] <= d[0] <= f1[0]]
        rows.append({
            "fill": k, "gap_us": round((f1[0] - prev_end) / 1e3, 1),
            "fill_ms": round((f1[1] - f1[0]) / 1e6, 3),
            "scan_start_after_fill_start_ms": round((sc[-1][0] - f0[0]) / 1e6, 3) if sc else None,
            "scan_ms": round((sc[-1][1] - sc[-1][0]) / 1e6, 3) if sc else None,
            "scan_end_before_next_fill_us": round((f1[0] - sc[-1][1]) / 1e3, 1) if sc else None,
            "decide_end_before_next_fill_us": round((f1[0] - dc[-1][1]) / 1e3, 1) if dc else None,
        })
    out = {"fills": len(fills), "rows": rows,
           "scan_share_of_kernel_time": round(sum(s[1] - s[0] for s in scans) / tot, 4) if tot else None,
           "mean_gap_us": round(sum(r["gap_us"] for r in rows) / len(rows), 1) if rows else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
