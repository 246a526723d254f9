#!/bin/bash
# round 4: score-only GPU tests, the full GPU suite, then the PMC roofline passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -8 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/pmc_roofline.sh > gpurun_out/roofline.log 2>&1; rc=$?
tail -40 gpurun_out/roofline.log
exit $rc
