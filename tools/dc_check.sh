#!/bin/bash
# Linear-space aligners on the GPU box: their parity tests, then tools/bench_dc.py (10,000 x 1024^2
# and 1,000 x 4096^2, both algorithms) -> gpurun_out/dc.jsonl.  Each GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[dc] tests $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "hirschberg or myers or dc_" --timeout 120 --timeout-method thread > gpurun_out/dc_tests.log 2>&1 || { echo dc tests failed; tail -30 gpurun_out/dc_tests.log; exit 1; }
tail -2 gpurun_out/dc_tests.log
: > gpurun_out/dc.jsonl
for algo in hb mm; do
  for cfg in "10000 1024" "1000 4096"; do
    set -- $cfg
    echo "[dc] bench $algo $1 x $2 $(date +%T)"
    timeout -k 10 300 python tools/bench_dc.py --algo $algo --pairs $1 --len $2 > gpurun_out/dc_run.log 2>&1 || { echo bench failed; tail -20 gpurun_out/dc_run.log; exit 1; }
    grep '^{' gpurun_out/dc_run.log >> gpurun_out/dc.jsonl
  done
done
cat gpurun_out/dc.jsonl
