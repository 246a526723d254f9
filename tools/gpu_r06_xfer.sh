#!/bin/bash
# Round 6: 2-bit host-API transfers -- tests, then the host-API call trace and timing.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_xfer.py tests/test_gpu_configs.py > gpurun_out/xfer_tests.txt 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/xfer_tests.txt; exit 1; }
tail -2 gpurun_out/xfer_tests.txt
rm -rf gpurun_out/e2e_trace2
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2e_trace2 -o run -- python3 tools/e2e_trace.py > gpurun_out/e2e_trace2.log 2>&1 || { tail -5 gpurun_out/e2e_trace2.log; exit 1; }
grep -E "call|seqalib host" gpurun_out/e2e_trace2.log
SEQALIB_XFER2=0 timeout -k 10 300 python3 tools/e2e_trace.py 2>&1 | grep -E "call|seqalib host"
timeout -k 10 300 python3 tools/e2e_trace.py 2>&1 | grep -E "call|seqalib host"
