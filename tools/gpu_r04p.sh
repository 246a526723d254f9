#!/bin/bash
# round 4: per-kernel breakdown of HB / MM with the two-per-wave 16-bit sweeps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for algo in hb mm; do
  rm -rf gpurun_out/prof_dc5_$algo
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dc5_$algo -o run -- python3 tools/bench_dc.py --algo $algo --pairs 10000 --len 1024 --cpu-pairs 0 > gpurun_out/prof_dc5_$algo.log 2>&1 || { tail -20 gpurun_out/prof_dc5_$algo.log; exit 1; }
  grep '^{' gpurun_out/prof_dc5_$algo.log | cut -c1-160
  python3 - $algo <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/prof_dc5_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(f"   {int(r['Calls']):5d} calls {float(r['TotalDurationNs']) / 1e6:8.3f} ms total {float(r['AverageNs'])/1e3:9.1f} us avg  {r['Name'][:70]}")
PY
done
