#!/usr/bin/env python3
"""Average duration of the headline fill dispatches in a rocprofv3 --kernel-trace run of bench.py:
the score-only SW fill (fill_so_kernel<0, 32>) launched on the headline batch's grid (10,000 pairs
x 2 bands x 2 column segments = 40,000 single-wave workgroups = 2,560,000 threads), so the configs legs' launches of
the same kernel on other grids are not mixed in.  Prints one JSON line.
    python3 tools/headline_fill_avg.py gpurun_out/prof_bench [--grid 1280000]"""
import argparse
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--grid", type=int, default=10000 * 2 * 2 * 64)   # pairs x bands x column segments x 64
ap.add_argument("--kernel", default="fill_so_kernel<0, 32>")
a = ap.parse_args()
durs = []
for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if a.kernel in r["Kernel_Name"] and int(r["Grid_Size_X"]) == a.grid:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
print(json.dumps({"kernel": a.kernel, "grid_threads": a.grid, "launches": len(durs),
                  "avg_ms": round(sum(durs) / len(durs), 3) if durs else None,
                  "min_ms": round(min(durs), 3) if durs else None, "max_ms": round(max(durs), 3) if durs else None}))
