#!/bin/bash
# round 4: the unstaged-Seq2 many-pairs path (SEQALIB_STAGE_SEQ2=0) vs the oracle, then the staged one
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -q --timeout 150 --timeout-method thread -m gpu \
  -k "unstaged or many_pairs_plan" > gpurun_out/gputest_unstaged.txt 2>&1; rc=$?
grep -E "passed|failed|Error|assert" gpurun_out/gputest_unstaged.txt | head -20
exit $rc
