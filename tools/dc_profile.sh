#!/bin/bash
# rocprofv3 kernel breakdown of the linear-space aligners (10,000 x 1024^2, both algorithms)
#   -> gpurun_out/prof_dc_{hb,mm}_kernel_stats.csv
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for algo in hb mm; do
  rm -rf gpurun_out/prof_dc_$algo
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dc_$algo -o run -- python3 tools/bench_dc.py --algo $algo --pairs 10000 --len 1024 --cpu-pairs 0 > gpurun_out/prof_dc_$algo.log 2>&1 || { echo rocprof $algo failed; tail -20 gpurun_out/prof_dc_$algo.log; exit 1; }
  f=$(find gpurun_out/prof_dc_$algo -name '*kernel_stats.csv' | head -1)
  cp "$f" gpurun_out/prof_dc_${algo}_kernel_stats.csv
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f'{r["Name"][:70]:72s} calls {r["Calls"]:>4s} total {float(r["TotalDurationNs"])/1e6:8.2f} ms avg {float(r["AverageNs"])/1e6:8.3f} ms')
PY
done
