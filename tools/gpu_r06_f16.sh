#!/bin/bash
# Round 6: the f16 cell of the two-pairs-per-wave SW fill -- score-only tests, then alternating
# pipelined headline steps against the 16-bit integer cell (SEQALIB_SO2_F16=0).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_so.py ${F16_TESTS} > gpurun_out/f16_tests.log 2>&1 || { tail -30 gpurun_out/f16_tests.log; exit 1; }
tail -2 gpurun_out/f16_tests.log
timeout -k 10 400 python3 -u tools/fill_sweep.py --sizes "" --variants "base;SEQALIB_SO2_F16=0" --rounds 3 --steps 10 2>&1 | grep -E "variant|check"
