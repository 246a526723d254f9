#!/bin/bash
# Round 6: walk prefetch (8 lanes per pair) -- score-only tests, then serial / host-API A/B.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_so.py tests/test_gpu_handoff.py tests/test_gpu_xfer.py > gpurun_out/pf_tests.txt 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/pf_tests.txt | head; tail -30 gpurun_out/pf_tests.txt; exit 1; }
tail -1 gpurun_out/pf_tests.txt
timeout -k 10 400 python3 -u tools/e2e_ab.py "base;SEQALIB_TB_PF=0" 3 5 2>&1 | grep -v amdgpu.ids
