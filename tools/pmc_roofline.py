#!/usr/bin/env python3
"""Summarise tools/pmc_roofline.sh: for the LONGEST fill dispatch (the measured call's fill) the
counters of every pass, HBM bytes per launch with the gfx950 corrections of MI355X_MICROARCH.md
(FETCH_SIZE counts half the bytes of wide coalesced streaming reads: x2; WRITE_SIZE exact for
16-B-per-lane stores; both in KiB), the shader clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), VALU
instructions per cell and the kernel-trace stats.  Writes <dir>/summary.json and prints text."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/roofline"
CELLS = 10000 * 4096 * 4096


def fill_like(name):
    return "fill_so_kernel" in name or "fill_so2_kernel" in name or "fill_kernel" in name


out = {"counters": {}, "durations_ms": {}}
for f in sorted(glob.glob(os.path.join(d, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    dur, nm = {}, {}
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if not fill_like(name):
            continue
        k = r["Dispatch_Id"]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        nm[k] = name
    if not dur:
        continue
    k = max(dur, key=lambda x: dur[x])
    p = next((x for x in f.split(os.sep) if x.startswith("pmc_")), f)
    for c, v in acc[k].items():
        out["counters"][c] = v
        if c == "GRBM_GUI_ACTIVE":
            out.setdefault("clock_ghz_per_pass", {})[p] = v / 8 / (dur[k] * 1e-9) / 1e9
    out["durations_ms"][p] = dur[k] / 1e6
    out["kernel"] = nm[k][:200]
c = out["counters"]
res = {"kernel": out.get("kernel"), "durations_ms_per_pass": out["durations_ms"], "counters": c}
if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
    fetch = c["FETCH_SIZE"] * 1024 * 2
    write = c["WRITE_SIZE"] * 1024
    res["hbm_bytes_per_launch"] = fetch + write
    res["hbm_basis"] = "FETCH_SIZE x 1024 x 2 (gfx950 wide-read correction) + WRITE_SIZE x 1024"
    res["fetch_bytes"], res["write_bytes"] = fetch, write
if out.get("clock_ghz_per_pass"):
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs: / 8 / the same dispatch's duration
    res["clock_ghz_per_pass"] = out["clock_ghz_per_pass"]
    res["clock_ghz"] = sum(out["clock_ghz_per_pass"].values()) / len(out["clock_ghz_per_pass"])
if "SQ_INSTS_VALU" in c:
    res["valu_wave_instr_per_cell"] = c["SQ_INSTS_VALU"] * 64 / CELLS
if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
    res["wait_inst_frac"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
stats = glob.glob(os.path.join(d, "stats", "**", "*kernel_stats.csv"), recursive=True)
if stats:
    rows = list(csv.DictReader(open(stats[0])))
    res["kernel_stats"] = [{k: r[k] for k in r if k in ("Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage")}
                           for r in rows[:12]]
json.dump(res, open(os.path.join(d, "summary.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
