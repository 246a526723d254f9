#!/bin/bash
# Round 6: full GPU suite, then the host-API call trace (kernels + copies).
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r06_b}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gputest_$TAG.txt 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gputest_$TAG.txt; exit 1; }
tail -2 gpurun_out/gputest_$TAG.txt
rm -rf gpurun_out/e2e_trace
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2e_trace -o run -- python3 tools/e2e_trace.py > gpurun_out/e2e_trace.log 2>&1 || { tail -5 gpurun_out/e2e_trace.log; exit 1; }
grep -v amdgpu.ids gpurun_out/e2e_trace.log
