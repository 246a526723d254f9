#!/bin/bash
# round 4: score-only traceback walk rework -- SO parity tests, round statistics, kernel times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[i] so tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_so.py tests/test_dropin_cpp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_i.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_i.log
[ $rc -eq 0 ] || exit $rc
echo "[i] so4 stats $(date +%T)"
timeout -k 10 200 python3 tools/so4_stats.py 10000 2>&1 | grep -v amdgpu.ids | tee gpurun_out/so4_stats_i.txt
echo "[i] kernel stats $(date +%T)"
rm -rf gpurun_out/prof_i
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_i -o run -- python3 tools/headline_once.py --calls 2 > gpurun_out/prof_i.log 2>&1 || { tail -20 gpurun_out/prof_i.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_i/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:4]:
    print(f"   {int(r['Calls']):4d}  {float(r['AverageNs']) / 1e6:8.3f} ms  {r['Name'][:90]}")
PY
