#!/bin/bash
# round 4: full GPU suite, configs 2/4 (SPLIT granule per cell type), default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[k] full suite $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -6 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
echo "[k] bench $(date +%T)"
timeout -k 10 600 python -u bench.py > gpurun_out/bench_k.json 2> gpurun_out/bench_k.err; rc=$?
tail -2 gpurun_out/bench_k.err
python3 -c "import json; d=json.loads(open('gpurun_out/bench_k.json').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','ms_per_step','fill_ms','fill_kernel_ms','endcell_ms','traceback_ms','serial_ms_per_step','e2e_ms_per_step')}); print(json.dumps(d['roofline'])[:400]); print(json.dumps(d.get('configs'))[:2500]); print(json.dumps(d.get('dropin_e2e'))); print(json.dumps(d.get('dropin_single_call'))); print(json.dumps(d.get('cpu_baseline')))"
exit $rc
