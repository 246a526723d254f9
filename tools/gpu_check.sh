#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> bench (args passed through).  Every GPU step
# has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[gpu_check] smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -30 gpurun_out/smoke.log; exit 1; }
echo "[gpu_check] pytest -m gpu $(date +%T)"
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
echo "[gpu_check] bench $* $(date +%T)"
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py "$@" > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
echo "[gpu_check] done $(date +%T)"
