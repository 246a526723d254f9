"""Summarise tools/pmc_fill.sh passes: per variant (x2=0 one pair per wave, x2=1 two pairs), the
counters of the LARGEST sa::fill_kernel dispatch (by duration) of the timed step -- the variant
the batch selected; the other variant's launch returns at once.
    python tools/pmc_summary.py gpurun_out > profiles/pmc_fill_r03.txt"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
rows = collections.defaultdict(dict)
names = {}
for f in sorted(glob.glob(os.path.join(d, "pmcf_*_*", "**", "*counter_collection.csv"), recursive=True)):
    x2 = f.split("pmcf_")[1].split(os.sep)[0].split("_")[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    nm = {}
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if "sa::fill_kernel" not in name and "sa::fill_x2_kernel" not in name:
            continue
        key = r["Dispatch_Id"]
        acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        nm[key] = name
    if not dur:
        continue
    key = max(dur, key=lambda k: dur[k])
    for k, v in acc[key].items():
        rows[x2][k] = v
    rows[x2]["duration_ms"] = dur[key] / 1e6
    names[x2] = nm[key]
print("# tools/pmc_fill.sh + tools/pmc_summary.py: 10,000 x 4096^2 SW headline batch, the longest fill")
print("# dispatch of the profiled run (rocprofv3 --pmc, one pass per counter group, so durations differ")
print("# slightly between passes).  SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles.")
for x2, n in sorted(names.items()):
    print(f"# x2={x2}: {n[:150]}")
keys = sorted(set(rows.get("0", {})) | set(rows.get("1", {})))
print(f"{'counter':28s} {'one-pair (x2=0)':>16s} {'two-pair (x2=1)':>16s} {'ratio':>7s}")
for k in keys:
    a, b = rows.get("0", {}).get(k), rows.get("1", {}).get(k)
    ratio = f"{b / a:.3f}" if a and b else ""
    fa = f"{a:16.5g}" if a is not None else f"{'-':>16s}"
    fb = f"{b:16.5g}" if b is not None else f"{'-':>16s}"
    print(f"{k:28s} {fa} {fb} {ratio:>7s}")
cells = 10000 * 4096 * 4096
for x2 in sorted(rows):
    r = rows[x2]
    if "SQ_INSTS_VALU" in r:
        print(f"# x2={x2}: VALU wave-instr per cell {r['SQ_INSTS_VALU'] * 64 / cells:.3f}; ", end="")
    if "SQ_ACTIVE_INST_VALU" in r and "SQ_INSTS_VALU" in r:
        print(f"quad-cycles of VALU activity per VALU instr {r['SQ_ACTIVE_INST_VALU'] / r['SQ_INSTS_VALU']:.3f}", end="")
    print()
