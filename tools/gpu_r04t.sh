#!/bin/bash
# round 4 validation: every -m gpu test, smoke(), then the PMC roofline passes of the shipped fill
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[t] tests $(date +%T)"
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo gpu tests failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
echo "[t] smoke $(date +%T)"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/pmc_roofline.sh
