#!/bin/bash
# round 4: full GPU suite (chunked drop-in check included), drop-in e2e phases, default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[g] full suite $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -12 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
echo "[g] drop-in phases $(date +%T)"
SEQALIB_HOST_TIMING=1 timeout -k 10 300 tests/cpp/dropin_bench 10000 4096 3 > gpurun_out/dropin_g.json 2> gpurun_out/dropin_g.err || { tail -20 gpurun_out/dropin_g.err; exit 1; }
cat gpurun_out/dropin_g.json; tail -24 gpurun_out/dropin_g.err
echo "[g] bench $(date +%T)"
timeout -k 10 600 python -u bench.py > gpurun_out/bench_g.json 2> gpurun_out/bench_g.err; rc=$?
tail -3 gpurun_out/bench_g.err
python3 -c "import json; d=json.loads(open('gpurun_out/bench_g.json').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','ms_per_step','fill_ms','fill_kernel_ms','endcell_ms','traceback_ms','serial_ms_per_step','e2e_ms_per_step')}); print(json.dumps(d['roofline'])); print(json.dumps(d.get('configs'))[:2000]); print(json.dumps(d.get('dropin_e2e'))); print(json.dumps(d.get('dropin_single_call')))"
exit $rc
