#!/bin/bash
# Round 6 final, part A: full GPU suite and the PMC roofline passes of the shipped headline fill.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gputest_r06_final.txt 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gputest_r06_final.txt; exit 1; }
tail -1 gpurun_out/gputest_r06_final.txt
OUT=gpurun_out/roofline_final bash tools/pmc_roofline.sh > gpurun_out/pmc_final.txt 2>&1 || { tail -20 gpurun_out/pmc_final.txt; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/roofline_final/summary.json')); print({k: d.get(k) for k in ('hbm_bytes_per_launch','clock_ghz','valu_wave_instr_per_cell','durations_ms_per_pass')})"
