#!/bin/bash
# Full GPU session: every -m gpu test, then the SPLIT session (tools/gpu_split.sh: configs 2/4 and
# per-band timelines).  Each GPU step has its own limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[full] tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo gpu tests failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash tools/gpu_split.sh
