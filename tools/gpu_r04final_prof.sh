#!/bin/bash
# round 4: rocprofv3 kernel-trace summary of the bench command itself (headline leg), so the bench
# line's fill launch time and the profiler's average come from the same run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/fprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof -o run -- python3 bench.py --no-cpu --dropin-pairs 0 --configs '' --latency-reps 0 --out gpurun_out/bench_prof.json > gpurun_out/fprof.log 2>&1 || { tail -20 gpurun_out/fprof.log; exit 1; }
python3 - <<'PY'
import csv, glob, json
f = glob.glob("gpurun_out/fprof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("endcell_so", "traceback_so4", "fill_so")):
        print(f"{r['Name'][:50]:50s} {r['Calls']:>4s} calls {float(r['AverageNs']) / 1e3:9.1f} us avg")
d = json.load(open("gpurun_out/bench_prof.json"))
print("bench", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["fill_kernel_ms"])
PY
