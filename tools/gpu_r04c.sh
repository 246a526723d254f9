#!/bin/bash
# round 4: headline bench (short), score-only + screened-LUT GPU tests, drop-in latency
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --dropin-pairs 0 --e2e-steps 0 --serial-steps 1 > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err || { echo bench failed; tail -20 gpurun_out/bench_c.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c.json')); print({k: d[k] for k in ('value','ms_per_step','fill_ms','endcell_traceback_ms','serial_ms_per_step','parity')})"
timeout -k 10 120 ./tests/cpp/dropin_latency 200 > gpurun_out/latency_c.json 2>&1 || { echo latency failed; cat gpurun_out/latency_c.json; exit 1; }
cat gpurun_out/latency_c.json
timeout -k 10 700 python -u -m pytest tests/test_gpu_so.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "so or screened" > gpurun_out/pytest_c.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_c.log
exit $rc
