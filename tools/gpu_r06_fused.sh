#!/bin/bash
# Round 6: the end-cell replay fused into the packed fill's final units -- SO GPU tests, then the
# headline bench (default) against SEQALIB_SO2=0 (one pair per wave + the end-cell kernel), alternating.
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_so.py tests/test_gpu_handoff.py tests/test_gpu_parity.py > gpurun_out/fused_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/fused_tests.log; exit 1; }
tail -1 gpurun_out/fused_tests.log
B="--steps 10 --warmup 2 --no-cpu --dropin-pairs 0 --latency-reps 0 --configs none --e2e-steps 2 --serial-steps 3 --parity-ops 8"
for k in 1 2; do
  timeout -k 10 300 python3 bench.py $B --out gpurun_out/fused_new_$k.json > /dev/null 2>&1 || exit 1
  SEQALIB_SO2=0 timeout -k 10 300 python3 bench.py $B --out gpurun_out/fused_old_$k.json > /dev/null 2>&1 || exit 1
done
for f in gpurun_out/fused_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], 'fill', d['fill_ms'], 'kern', d['fill_kernel_ms'], 'serial', d['serial_ms_per_step'], 'e2e', d['e2e_ms_per_step'], d['parity_exact'])"; done
