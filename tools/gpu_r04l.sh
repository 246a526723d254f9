#!/bin/bash
# round 4: sparser chunk-max tracking -- SO parity, kernel times, quick bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[l] so + endcell tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_so.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "so or endcell or headline or sw" > gpurun_out/pytest_l.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_l.log
[ $rc -eq 0 ] || exit $rc
echo "[l] kernel stats $(date +%T)"
rm -rf gpurun_out/prof_l
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_l -o run -- python3 tools/headline_once.py --calls 2 > gpurun_out/prof_l.log 2>&1 || { tail -20 gpurun_out/prof_l.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_l/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:4]:
    print(f"   {int(r['Calls']):4d}  {float(r['AverageNs']) / 1e6:8.3f} ms  {r['Name'][:90]}")
PY
echo "[l] bench $(date +%T)"
timeout -k 10 300 python -u bench.py --configs 3,5 --dropin-pairs 0 --latency-reps 0 --no-cpu > gpurun_out/bench_l.json 2> gpurun_out/bench_l.err; rc=$?
tail -2 gpurun_out/bench_l.err
python3 -c "import json; d=json.loads(open('gpurun_out/bench_l.json').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','ms_per_step','fill_ms','fill_kernel_ms','endcell_ms','traceback_ms','serial_ms_per_step','e2e_ms_per_step','parity')}); print(json.dumps(d.get('configs'))[:1500])"
exit $rc
