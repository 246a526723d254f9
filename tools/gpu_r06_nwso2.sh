#!/bin/bash
# Round 6: NW with two pairs per wave -- NW tests, then pipelined NW steps against one pair per wave.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_so.py tests/test_gpu_handoff.py -k "nw or NW or so2 or scoring1 or segments" > gpurun_out/nwso2_tests.txt 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/nwso2_tests.txt | head -20; tail -30 gpurun_out/nwso2_tests.txt; exit 1; }
tail -2 gpurun_out/nwso2_tests.txt
for L in 4096 1024; do
timeout -k 10 400 python3 -u tools/fill_sweep.py --algo 1 --sizes "" --len $L --variants "base;SEQALIB_SO2=0" --rounds 3 --steps 10 > gpurun_out/nwso2_$L.jsonl 2>&1 || { tail -5 gpurun_out/nwso2_$L.jsonl; exit 1; }
grep -E "variant|check" gpurun_out/nwso2_$L.jsonl | sed "s/^/$L /"
done
