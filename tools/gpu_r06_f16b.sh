#!/bin/bash
# Round 6: the scaled 4-op f16 cell (F kept per row) -- score-only tests, then alternating pipelined
# headline steps: R = 16 forced (SEQALIB_PLAN=16,1), the default plan, and the 16-bit cell.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_so.py > gpurun_out/f16b_tests.log 2>&1 || { tail -30 gpurun_out/f16b_tests.log; exit 1; }
tail -2 gpurun_out/f16b_tests.log
timeout -k 10 500 python3 -u tools/fill_sweep.py --sizes "" --variants "${F16B_VARIANTS:-SEQALIB_PLAN=16,1;base;SEQALIB_SO2_F16=0}" --rounds 3 --steps 10 2>&1 | grep -E "variant|check"
