#!/bin/bash
# round 4: drop-in chunk tests; HB / MM per-kernel breakdown (10,000 x 1024^2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[n] drop-in + DC tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_dropin_cpp.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "dropin or chunked or hirschberg or myers or dc or Driver or driver or types or wide or bridg" > gpurun_out/pytest_n.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_n.log
[ $rc -eq 0 ] || exit $rc
for algo in hb mm; do
  echo "[n] $algo kernels $(date +%T)"
  rm -rf gpurun_out/prof_dc4_$algo
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dc4_$algo -o run -- python3 tools/bench_dc.py --algo $algo --pairs 10000 --len 1024 --cpu-pairs 0 > gpurun_out/prof_dc4_$algo.log 2>&1 || { tail -20 gpurun_out/prof_dc4_$algo.log; exit 1; }
  grep '^{' gpurun_out/prof_dc4_$algo.log | cut -c1-200
  python3 - $algo <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/prof_dc4_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:14]:
    print(f"   {int(r['Calls']):5d} calls {float(r['TotalDurationNs']) / 1e6:8.3f} ms total  {r['Name'][:80]}")
PY
done
