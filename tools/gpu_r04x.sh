#!/bin/bash
# round 4 final: every -m gpu test, smoke(), the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[x] tests $(date +%T)"
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo gpu tests failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
echo "[x] smoke $(date +%T)"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "[x] bench $(date +%T)"
timeout -k 10 900 python3 bench.py --out gpurun_out/bench_final.json > gpurun_out/bench_final.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_final.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_final.json')); print(d['value'], d['ms_per_step'], d['fill_kernel_ms'], d['endcell_ms'], d['traceback_ms'], d['parity'][:40], d['dropin_e2e']['ms_mean'] if d.get('dropin_e2e') else None)"
