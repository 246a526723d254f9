#!/bin/bash
# Effective shader clock and wave occupancy of the headline fill, one-pair vs two-pair kernel
# (rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES, one pass each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for x2 in 0 1; do
  rm -rf gpurun_out/pmc_clock_$x2
  SEQALIB_X2=$x2 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv \
    -d gpurun_out/pmc_clock_$x2 -o run -- python3 bench.py --no-cpu --steps 1 --warmup 1 > gpurun_out/pmc_clock_$x2.log 2>&1 || { echo "pmc x2=$x2 failed"; tail -5 gpurun_out/pmc_clock_$x2.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for x2 in (0, 1):
    f = glob.glob(f"gpurun_out/pmc_clock_{x2}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", r.get("KernelName", ""))
        if "fill" not in name: continue
        key = (name[:60], r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        acc[key][r.get("Counter_Name", "")] += float(r.get("Counter_Value", 0))
        if "End_Timestamp" in r: dur[key] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e9
    for k, v in acc.items():
        if v.get("SQ_WAVES", 0) < 1000: continue
        t = dur.get(k)
        print(f"x2={x2} {k[0]}  waves {v['SQ_WAVES']:.0f}  GRBM_GUI_ACTIVE {v['GRBM_GUI_ACTIVE']:.3g}  "
              f"time {t if t else float('nan'):.4f} s  clock {v['GRBM_GUI_ACTIVE'] / t / 1e9 if t else float('nan'):.3f} GHz  "
              f"SQ_BUSY_CYCLES {v['SQ_BUSY_CYCLES']:.3g}  SQ_WAVE_CYCLES {v['SQ_WAVE_CYCLES']:.3g}")
PY
