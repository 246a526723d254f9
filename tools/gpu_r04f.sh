#!/bin/bash
# round 4: full GPU suite, launch count of single-pair calls, PMC roofline, default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[f] full suite $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -12 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
echo "[f] launch count $(date +%T)"
bash tools/launch_count.sh || exit 1
echo "[f] roofline $(date +%T)"
bash tools/pmc_roofline.sh > gpurun_out/roofline.log 2>&1; rc=$?
tail -30 gpurun_out/roofline.log
[ $rc -eq 0 ] || exit $rc
echo "[f] bench $(date +%T)"
timeout -k 10 600 python -u bench.py > gpurun_out/bench_f.json 2> gpurun_out/bench_f.err; rc=$?
tail -3 gpurun_out/bench_f.err
python3 -c "import json; d=json.loads(open('gpurun_out/bench_f.json').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','ms_per_step','fill_ms','endcell_traceback_ms','serial_ms_per_step','e2e_ms_per_step','parity')}); print(json.dumps(d.get('configs'))[:1500]); print(json.dumps(d.get('dropin_e2e'))); print(json.dumps(d.get('dropin_single_call')))"
exit $rc
