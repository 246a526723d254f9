#!/bin/bash
# round 4: headline bench (short) + the score-only GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --dropin-pairs 0 --e2e-steps 0 --serial-steps 1 > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { echo bench failed; tail -20 gpurun_out/bench_b.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_b.json')); print({k: d[k] for k in ('value','ms_per_step','fill_ms','endcell_traceback_ms','serial_ms_per_step','parity')})"
timeout -k 10 600 python -u -m pytest tests/test_gpu_so.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_so.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_so.log
exit $rc
